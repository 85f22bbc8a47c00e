#!/bin/bash
# Round 6: c3's wavefront knobs re-swept under the frame overlap (runtime options, bench lines, interleaved rounds).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_c3_knobs_ov}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
line() {
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --config c3 --steps 100 --warmup 20 "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'])"
}
for r in 1 2; do
  line base_$r
  for rf in 12 16 24 32; do line refill${rf}_$r --wf-refill $rf; done
  line fetch0_$r --wf-fetch 0
  line fetch1_$r --wf-fetch 1
done
echo SESSION_DONE
