#!/bin/bash
# Path-persistent kernel: shade-batch threshold (refill) and occupancy sweep on c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03p}; mkdir -p $OUT
for lib in paths6 paths5; do
WCPT_LIBRARY=wc-path-tracer_amd/variants/$lib.so timeout -k 10 300 python3 tools/ab.py --config c3 --variants "kernel=3,refill=12" "kernel=3,refill=24" "kernel=3,refill=40" "kernel=3,refill=56" --frames 4 --rounds 2 > $OUT/ab_$lib.log 2>&1 || { tail -3 $OUT/ab_$lib.log; exit 1; }
echo $lib; cat $OUT/ab_$lib.log
done
