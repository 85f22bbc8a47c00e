#!/bin/bash
# Round 6: frame overlap (WCPT_OPTION_FRAME_OVERLAP): its GPU tests, then bench lines with it off and on, interleaved
# rounds: c2 / ref with the still and the orbiting camera, c3, and (once) c4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_overlap_ab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "=== tests $(date +%T)"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_overlap.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1; rc=$?
echo "rc=$rc"; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit 1
line() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'], d['kernel_ms_avg'])"
}
for r in ${ROUNDS:-1 2}; do
  for cfg in c2 ref; do
    for cam in still orbit; do
      for ov in 0 1; do line ${cfg}_${cam}_ov${ov}_$r --config $cfg --camera $cam --frame-overlap $ov; done
    done
  done
  for ov in 0 1; do line c3_ov${ov}_$r --config c3 --frame-overlap $ov --steps 100 --warmup 20; done
done
for ov in 0 1; do line c4_ov${ov} --config c4 --frame-overlap $ov --steps 12 --warmup 3; done
echo SESSION_DONE
