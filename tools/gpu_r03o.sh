#!/bin/bash
# Path-persistent kernel (WCPT_KERNEL_PATHS = 3): GPU parity tests, then c3 / ref / c4-block A/B against the wavefront.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03o}; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 tools/ab.py --config c3 --variants "kernel=2" "kernel=3" --frames 5 --rounds 3 > $OUT/ab_c3.log 2>&1 || { tail -3 $OUT/ab_c3.log; exit 1; }
cat $OUT/ab_c3.log
WCPT_LIBRARY=wc-path-tracer_amd/variants/paths6.so timeout -k 10 300 python3 tools/ab.py --config c3 --variants "kernel=3" --frames 5 --rounds 2 > $OUT/ab_c3_w6.log 2>&1 || { tail -3 $OUT/ab_c3_w6.log; exit 1; }
cat $OUT/ab_c3_w6.log
timeout -k 10 300 python3 tools/ab.py --config ref --variants "kernel=0" "kernel=2" "kernel=3" --frames 5 --rounds 2 > $OUT/ab_ref.log 2>&1 || { tail -3 $OUT/ab_ref.log; exit 1; }
cat $OUT/ab_ref.log
timeout -k 10 300 python3 tools/ab.py --config c4 --rows 270 --variants "kernel=2" "kernel=3" --frames 2 --rounds 2 > $OUT/ab_c4.log 2>&1 || { tail -3 $OUT/ab_c4.log; exit 1; }
cat $OUT/ab_c4.log
