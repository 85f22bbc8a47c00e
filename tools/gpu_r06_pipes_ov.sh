#!/bin/bash
# Round 6: wavefront pipeline count with the frame overlap on (bench lines, interleaved rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_pipes_ov}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
line() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"
}
for r in 1 2; do
  for k in 2 3 4; do line c3_k${k}_$r --config c3 --wf-pipes $k --steps 100 --warmup 20; done
done
for k in 2 3 4; do line c4_k${k} --config c4 --wf-pipes $k --steps 12 --warmup 3; done
echo SESSION_DONE
