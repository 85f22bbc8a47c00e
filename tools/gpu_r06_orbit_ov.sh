#!/bin/bash
# Round 6: frame overlap with a moving camera (per-pipe primary-ray records): GPU tests, then orbit bench lines off/on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_orbit_ov}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "=== tests $(date +%T)"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
line() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"
}
for r in 1 2; do
  for cfg in c2 ref; do
    for ov in 0 1; do line ${cfg}_orbit_ov${ov}_$r --config $cfg --camera orbit --frame-overlap $ov; done
  done
  line c2_still_$r --config c2
done
echo SESSION_DONE
