#!/bin/bash
# Round 6: the driver's short bench window (--steps 20 --warmup 5), repeated, frame overlap off and on alternately.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_s20}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for r in 1 2 3 4 5 6; do
  for ov in 1 0; do
    n=c2_ov${ov}_$r
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup ${WARMUP:-5} --frame-overlap $ov > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['kernel_ms_avg'])"
  done
done
echo SESSION_DONE
