#!/bin/bash
# Tile orders 0/1/2/3 on c2, ref and the 135-row c2 block, after the tile-order parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-orderab2}; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_order" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in c2 ref; do
timeout -k 10 300 python3 tools/ab.py --config $cfg --variants "kernel=0,order=2" "kernel=0,order=3" "kernel=0,order=1" --frames 10 --rounds 4 > $OUT/ab_$cfg.log 2>&1 || { tail -3 $OUT/ab_$cfg.log; exit 1; }
cat $OUT/ab_$cfg.log
done
timeout -k 10 300 python3 tools/ab.py --config c2 --rows 135 --variants "kernel=0,order=2" "kernel=0,order=3" --frames 10 --rounds 4 > $OUT/ab_c2_135.log 2>&1 || exit 1
cat $OUT/ab_c2_135.log
