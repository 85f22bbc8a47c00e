#!/bin/bash
# Round 5 final-build session, part 1: GPU tests + smoke on the final build, then the counter passes bench.py prices
# its rooflines from (tools/gpu_sq.sh) for every bench line of the round, moving-camera lines included.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05_final}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
TAG=$TAG/sq CONFIGS="${CONFIGS:-c2 ref c3 c4 c2_orbit ref_orbit}" bash tools/gpu_sq.sh || exit 1
echo SESSION_DONE
