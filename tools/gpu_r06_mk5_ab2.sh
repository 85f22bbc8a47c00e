#!/bin/bash
# Round 6: the megakernel at 5 waves/SIMD (variants/mk5.so, WCPT_MK_WAVES=5) against the default, under the frame
# overlap: still and moving camera lines and the one-round 8-way block, interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_mk5_ab2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
BASE=$PWD/wc-path-tracer_amd/libwcpt.so; VAR=$PWD/wc-path-tracer_amd/variants/mk5.so
line() {
  local n=$1 lib=$2; shift 2
  WCPT_LIBRARY=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" || { echo "$n failed"; tail -5 "$OUT/$n.err"; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['ms_per_step'], d['value'])"
}
blk() {
  local n=$1 lib=$2; shift 2
  WCPT_LIBRARY=$lib timeout -k 10 300 python3 tools/block_balance.py "$@" > "$OUT/$n.log" 2>&1 || { echo "$n failed"; tail -5 "$OUT/$n.log"; exit 1; }
  echo "$n $(grep 'N=' "$OUT/$n.log" | cut -c1-160)"
}
for r in 1 2 3; do
  for cfg in c2 ref; do
    line ${cfg}_orbit_base_$r $BASE --config $cfg --camera orbit
    line ${cfg}_orbit_mk5_$r $VAR --config $cfg --camera orbit
    line ${cfg}_base_$r $BASE --config $cfg
    line ${cfg}_mk5_$r $VAR --config $cfg
  done
  blk c2_n8_base_$r $BASE --config c2 --ns 8 --skip-full --frames 60
  blk c2_n8_mk5_$r $VAR --config c2 --ns 8 --skip-full --frames 60
done
echo SESSION_DONE
