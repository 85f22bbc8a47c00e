#!/bin/bash
# Round 6: the path-persistent trace's shading-batch threshold (WCPT_OPTION_WF_REFILL, which the persistent trace reads
# as "shade once this many lanes wait") on c3 8-way blocks and 8-row stripes, interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_sweep2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep "N=" "$OUT/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit 1; }
for r in 1 2 3; do
  for f in 8 12 16 20; do
    run c3_refill${f}_$r 300 python3 tools/block_balance.py --config c3 --ns 8 --stripes 0,8 --skip-full --wf-refill $f
  done
done
echo SESSION_DONE
