#!/bin/bash
# Cost-ordered megakernel tiles (the default order 2): parity tests, then A/B against stripes (3) and bands (0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-costorder}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cost_ordered or tile_order or progressive or renderer or editor or full_size or reference_init" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for cfg in c2 ref; do
timeout -k 10 300 python3 tools/ab.py --config $cfg --variants "kernel=0,order=2" "kernel=0,order=3" "kernel=0,order=0" --frames 20 --rounds 4 > $OUT/ab_$cfg.log 2>&1 || { tail -3 $OUT/ab_$cfg.log; exit 1; }
cat $OUT/ab_$cfg.log
done
timeout -k 10 300 python3 tools/ab.py --config c2 --rows 135 --variants "kernel=0,order=2" "kernel=0,order=1" --frames 20 --rounds 4 > $OUT/ab_c2_135.log 2>&1 || exit 1
cat $OUT/ab_c2_135.log
timeout -k 10 300 python3 tools/ab.py --config c2 --rows 270 --variants "kernel=0,order=2" "kernel=0,order=3" --frames 20 --rounds 4 > $OUT/ab_c2_270.log 2>&1 || exit 1
cat $OUT/ab_c2_270.log
