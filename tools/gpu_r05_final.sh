#!/bin/bash
# Round 5 final-build session, part 1: GPU tests + smoke on the final build, then the counter passes bench.py prices
# its rooflines from (tools/gpu_sq.sh) for every bench line of the round, moving-camera lines included.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05_final}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
CFGS="${CONFIGS:-c2 ref c3 c4 c2_orbit ref_orbit}"
TAG=$TAG/sq CONFIGS="$CFGS" bash tools/gpu_sq.sh || exit 1
# summarise on the box and drop the raw per-dispatch CSVs (gpurun copies back at most 64 MiB)
S=$OUT/summaries; mkdir -p "$S"
cp "$OUT/sq/build_id" "$S/build_id"
python3 tools/profile_summaries.py "$OUT/sq" --configs $CFGS --out "$S" --source "round 5 final build ($TAG)" || exit 1
for c in c3 c4; do
  PF=2; [ $c = c3 ] && PF=3  # wavefront pipelines per frame (tools/profile_summaries.py PIPES)
  case " $CFGS " in *" $c "*) python3 tools/traffic_split.py "$OUT/sq/sq_$c" --per-frame $PF --json "$S/traffic_split_$c.json" > "$S/traffic_split_$c.log" || exit 1;; esac
done
for c in $CFGS; do
  f=$(find "$OUT/sq/prof_$c" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cp "$f" "$S/${c}_kernel_stats.csv"
  cp "$OUT/sq/prof_$c.log" "$S/prof_$c.log" 2>/dev/null
done
rm -rf "$OUT"/sq/sq_* "$OUT"/sq/prof_*
du -sh "$OUT"
echo SESSION_DONE
