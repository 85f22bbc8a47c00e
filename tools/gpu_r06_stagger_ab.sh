#!/bin/bash
# Round 6: fork stagger A/B (the default library against variants/stagger.so), bench lines with the driver's short
# window (--steps 20 --warmup 5) and the default one, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_stagger_ab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
line() {
  local n=$1 lib=$2; shift 2
  WCPT_LIBRARY=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"
}
BASE=$PWD/wc-path-tracer_amd/libwcpt.so; VAR=$PWD/wc-path-tracer_amd/variants/${VARIANT:-stagger}.so
for r in 1 2 3; do
  for cfg in c2 ref; do
    line ${cfg}_base_s20_$r $BASE --config $cfg --steps 20 --warmup 5
    line ${cfg}_stag_s20_$r $VAR --config $cfg --steps 20 --warmup 5
  done
done
for r in 1 2; do
  for cfg in c2 ref; do
    line ${cfg}_base_s200_$r $BASE --config $cfg
    line ${cfg}_stag_s200_$r $VAR --config $cfg
  done
done
echo SESSION_DONE
