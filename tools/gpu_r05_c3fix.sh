#!/bin/bash
# Re-take the c3 counter passes with the per-frame divisor of the 3 automatic pipelines, put the summaries in this box's
# profiles/, then the c3 bench line priced from them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05_c3fix}
TAG=$TAG/final TESTS=0 CONFIGS=c3 bash tools/gpu_r05_final.sh || exit 1
S=gpurun_out/$TAG/final/summaries
cp $S/sq_c3.json $S/valu_mix_c3.json $S/pmc_traffic_c3.json profiles/ || exit 1
mkdir -p gpurun_out/$TAG/session
timeout -k 10 600 python3 -u bench.py --config c3 --no-cpu-baseline > gpurun_out/$TAG/session/bench_c3.log 2>&1 || exit 1
tail -n 1 gpurun_out/$TAG/session/bench_c3.log | cut -c1-300
echo ALL_SESSIONS_DONE
