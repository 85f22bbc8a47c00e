#!/bin/bash
# A/B of the megakernel tile order (WCPT_OPTION_MK_TILE_ORDER) on c2, the reference scene and the c2 row block.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-orderab}; mkdir -p $OUT
for cfg in c2 ref c1; do
timeout -k 10 300 python3 tools/ab.py --config $cfg --variants "kernel=0,order=2" "kernel=0,order=1" "kernel=0,order=0" --frames 10 --rounds 4 > $OUT/ab_$cfg.log 2>&1 || { tail -3 $OUT/ab_$cfg.log; exit 1; }
cat $OUT/ab_$cfg.log
done
timeout -k 10 300 python3 tools/ab.py --config c2 --rows 135 --variants "kernel=0,order=2" "kernel=0,order=1" "kernel=0,order=0" --frames 10 --rounds 4 > $OUT/ab_c2_135.log 2>&1 || exit 1
cat $OUT/ab_c2_135.log
