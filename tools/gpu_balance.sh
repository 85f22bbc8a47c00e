#!/bin/bash
# tools/block_balance.py for c2 (N = 2/4/8) and c4 (N = 8) on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-balance}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python3 -u tools/block_balance.py --config c2 --ns 2,4,8 --frames 20 --rounds 3 > "$OUT/c2.log" 2>&1 || { echo c2 failed; tail -5 "$OUT/c2.log"; exit 1; }
tail -8 "$OUT/c2.log"
timeout -k 10 500 python3 -u tools/block_balance.py --config c4 --ns 8 --frames 2 --rounds 1 > "$OUT/c4.log" 2>&1 || { echo c4 failed; tail -5 "$OUT/c4.log"; exit 1; }
tail -8 "$OUT/c4.log"
