#!/bin/bash
# Striped XCD tile bands (orders 3-6: stripes of 1/2/4/8 tile rows) against bands (0) and scattered (1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-orderab3}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_order" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in c2 ref; do
timeout -k 10 300 python3 tools/ab.py --config $cfg --variants "kernel=0,order=0" "kernel=0,order=3" "kernel=0,order=4" "kernel=0,order=5" "kernel=0,order=6" --frames 10 --rounds 4 > $OUT/ab_$cfg.log 2>&1 || { tail -3 $OUT/ab_$cfg.log; exit 1; }
cat $OUT/ab_$cfg.log
done
timeout -k 10 300 python3 tools/ab.py --config c3 --variants "kernel=0,order=0" "kernel=0,order=4" --frames 3 --rounds 2 > $OUT/ab_c3mk.log 2>&1 || exit 1
cat $OUT/ab_c3mk.log
