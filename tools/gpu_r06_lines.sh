#!/bin/bash
# Round 6: the closing bench lines only (no counter passes: the committed profiles of the same build price them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_lines}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit 1; }
for c in ${CONFIGS:-c2 ref c2_orbit ref_orbit c3 c4}; do
  base=${c%_orbit}; CAM=""; [ "$base" != "$c" ] && CAM="--camera orbit"
  CPU="--no-cpu-baseline"; [ "$c" = c2 ] && CPU=""
  EXTRA=""; [ "$c" = c4 ] && EXTRA="--steps 20 --warmup 3"
  run bench_$c 900 python3 -u bench.py --config $base $CAM $CPU $EXTRA
done
run bench_c2_driver_cmd 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
echo SESSION_DONE
