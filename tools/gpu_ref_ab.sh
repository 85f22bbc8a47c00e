#!/bin/bash
# A/B of megakernel options on the reference's own Init scene (bench config ref).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-refab}; mkdir -p $OUT
timeout -k 10 300 python3 tools/ab.py --config ref --variants "kernel=0" "kernel=0,pairs=0" "kernel=0,order=0" "kernel=0,order=1" "kernel=0,stack=0" "kernel=2" "kernel=2,pipes=1" "kernel=2,pipes=3" --frames 5 --rounds 2 > $OUT/ab_ref.log 2>&1 || { tail -3 $OUT/ab_ref.log; exit 1; }
cat $OUT/ab_ref.log
