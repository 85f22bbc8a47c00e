#!/bin/bash
# Round 6: the driver's short bench window (--steps 20 --warmup 5) on the pre-overlap library (variants/pre_overlap.so,
# build 2859da8aaec7) against the current one, and the current one with more warmup frames.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_s20b}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
line() {
  local n=$1 lib=$2; shift 2
  WCPT_LIBRARY=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -3 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['kernel_ms_avg'], d['build_id'])"
}
CUR=$PWD/wc-path-tracer_amd/libwcpt.so; OLD=$PWD/wc-path-tracer_amd/variants/pre_overlap.so
for r in 1 2 3; do
  line old_s20_$r $OLD --steps 20 --warmup 5
  line cur_ov0_s20_$r $CUR --steps 20 --warmup 5 --frame-overlap 0
  line cur_s20_$r $CUR --steps 20 --warmup 5
  line cur_ov0_s20_w100_$r $CUR --steps 20 --warmup 100 --frame-overlap 0
  line cur_s100_w5_$r $CUR --steps 100 --warmup 5 --frame-overlap 0
done
echo SESSION_DONE
