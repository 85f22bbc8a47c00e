#!/bin/bash
# Round 6 closing session (one call per config set): on the final build, optionally the GPU tests and smoke(), then
# the counter passes bench.py prices its rooflines from (tools/gpu_sq.sh: the bench line's own command under
# rocprofv3 --kernel-trace --stats, FETCH/WRITE and the SQ / VALU-mix passes), summarised on the box
# (tools/profile_summaries.py) and put in the box's profiles/, then the bench lines of the same configs, which price
# their rooflines from those summaries. Everything the host needs comes back under gpurun_out/$TAG.
#   TAG=r06_final_a CONFIGS="c2 ref c2_orbit ref_orbit" TESTS=1 bash tools/gpu_r06_final.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_final}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit 1; }
CFGS="${CONFIGS:-c2 ref c3 c4 c2_orbit ref_orbit}"
if [ "${TESTS:-0}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
TAG=$TAG/sq CONFIGS="$CFGS" bash tools/gpu_sq.sh || exit 1
S=$OUT/summaries; mkdir -p "$S"
cp "$OUT/sq/build_id" "$S/build_id"
python3 tools/profile_summaries.py "$OUT/sq" --configs $CFGS --out "$S" --source "round 6 final build ($TAG)" || exit 1
for c in c3 c4; do
  PF=2; [ $c = c3 ] && PF=3
  case " $CFGS " in *" $c "*) python3 tools/traffic_split.py "$OUT/sq/sq_$c" --per-frame $PF --json "$S/traffic_split_$c.json" > "$S/traffic_split_$c.log" || exit 1;; esac
done
for c in $CFGS; do
  f=$(find "$OUT/sq/prof_$c" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$S/${c}_kernel_stats.csv"
  cp "$OUT/sq/prof_$c.log" "$S/prof_$c.log" 2>/dev/null
done
rm -rf "$OUT"/sq/sq_* "$OUT"/sq/prof_*
cp $S/sq_*.json $S/valu_mix_*.json $S/pmc_traffic_*.json profiles/ || exit 1
for c in $CFGS; do
  base=${c%_orbit}; CAM=""; [ "$base" != "$c" ] && CAM="--camera orbit"
  CPU="--no-cpu-baseline"; [ "$c" = c2 ] && CPU=""
  EXTRA=""; [ "$c" = c4 ] && EXTRA="--steps 20 --warmup 3"
  run bench_$c 900 python3 -u bench.py --config $base $CAM $CPU $EXTRA
done
du -sh "$OUT"
echo SESSION_DONE
