#!/bin/bash
# Row blocks of the 8-way split on one GPU (what one rank of an N = 8 run renders): c2 135 rows (megakernel), c4 270
# rows (wavefront), through tools/ab.py --rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-blocks}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/ab.py --config c2 --rows 135 --frames 20 --rounds 3 --variants "kernel=0" > "$OUT/c2_135.log" 2>&1 || { echo c2 failed; tail -3 "$OUT/c2_135.log"; exit 1; }
cat "$OUT/c2_135.log"
timeout -k 10 400 python3 tools/ab.py --config c4 --rows 270 --frames 3 --rounds 2 --variants "kernel=2" > "$OUT/c4_270.log" 2>&1 || { echo c4 failed; tail -3 "$OUT/c4_270.log"; exit 1; }
cat "$OUT/c4_270.log"
