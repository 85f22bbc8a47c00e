#!/bin/bash
# Round 6 closing session, part B: the wavefront configs' counter passes and bench lines (tools/gpu_r06_final.sh with
# c3 and c4), then the 8-way split's balance on the final build (blocks against 8-row stripes) for c2, c3 and c4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_final_b} CONFIGS="c3 c4" TESTS=0 bash tools/gpu_r06_final.sh || exit 1
OUT=gpurun_out/${TAG:-r06_final_b}
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep "N=" "$OUT/$name.log" | cut -c1-220; [ $rc -eq 0 ] || exit 1; }
run balance_c3 300 python3 tools/block_balance.py --config c3 --ns 2,4,8 --stripes 0,8
run balance_c2 300 python3 tools/block_balance.py --config c2 --ns 2,4,8 --stripes 0,8
run balance_c4 900 python3 tools/block_balance.py --config c4 --ns 8 --stripes 0,8 --frames 8 --rounds 2
echo SESSION_B_DONE
