#!/bin/bash
# Round 6: the full GPU suite on the current build, then the N-way split's balance with contiguous blocks against
# interleaved row stripes (tools/block_balance.py --stripes) on c3 and c4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_tests}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BALANCE:-1}" = 1 ]; then
  run balance_c3 600 python3 tools/block_balance.py --config c3 --ns 4,8 --stripes 0,8,16,32
  run balance_c4 900 python3 tools/block_balance.py --config c4 --ns 8 --stripes 0,8,16 --frames 8 --rounds 2
  run balance_c2 300 python3 tools/block_balance.py --config c2 --ns 8 --stripes 0,8
fi
echo SESSION_DONE
