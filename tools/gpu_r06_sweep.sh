#!/bin/bash
# Round 6: the c3 8-way interleaved split (stripes of 8 rows) under the path-persistent trace's knobs: pipelines
# (WCPT_OPTION_WF_PIPES) and the shading-batch / refill threshold (WCPT_OPTION_WF_REFILL).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_sweep}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep "N=" "$OUT/$name.log" | cut -c1-220; [ $rc -eq 0 ] || exit 1; }
for r in 1 2; do
  run c3_default_$r 300 python3 tools/block_balance.py --config c3 --ns 8 --stripes 0,8 --skip-full
  run c3_pipes2_$r 300 python3 tools/block_balance.py --config c3 --ns 8 --stripes 8 --skip-full --wf-pipes 2
  run c3_refill12_$r 300 python3 tools/block_balance.py --config c3 --ns 8 --stripes 8 --skip-full --wf-refill 12
  run c3_refill32_$r 300 python3 tools/block_balance.py --config c3 --ns 8 --stripes 8 --skip-full --wf-refill 32
done
run c3_n4_persist 300 python3 tools/block_balance.py --config c3 --ns 4 --stripes 0,8 --skip-full --wf-persist 1
echo SESSION_DONE
