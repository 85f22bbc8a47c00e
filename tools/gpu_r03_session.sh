#!/bin/bash
# One measurement session: the GPU tests, smoke(), then tools/gpu_r03_measure.sh over c2 / c3 / ref (bench line,
# rocprof kernel stats, FETCH/WRITE and SQ passes) and the c4 bench line. TAG names the output directory.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
echo "=== smoke $(date +%T)"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; tail -5 "$OUT/smoke.log"; exit 1; }
tail -2 "$OUT/smoke.log"
TAG=$TAG CEILINGS=0 CONFIGS="${CONFIGS:-c2 c3 ref}" bash tools/gpu_r03_measure.sh || exit 1
echo "=== bench_c4 $(date +%T)"
timeout -k 10 600 python3 -u bench.py --config c4 --no-cpu-baseline > "$OUT/bench_c4.log" 2>&1 || { echo c4 failed; exit 1; }
tail -1 "$OUT/bench_c4.log" | cut -c1-300
echo SESSION_DONE
