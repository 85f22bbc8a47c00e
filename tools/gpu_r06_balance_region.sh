#!/bin/bash
# Round 6: the N-way split's balance with region timing (frame overlap where its auto rule applies).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_balance_region}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; cat "$OUT/$name.log" | cut -c1-220; [ $rc -eq 0 ] || exit 1; }
run balance_c2 300 python3 tools/block_balance.py --config c2 --ns 2,4,8 --stripes 0,8 --frames 60
run balance_c3 300 python3 tools/block_balance.py --config c3 --ns 2,4,8 --stripes 0,8
run balance_c4 900 python3 tools/block_balance.py --config c4 --ns 8 --stripes 0,8 --frames 8 --rounds 2
echo SESSION_DONE
