#!/bin/bash
# Round-2 closing measurements after a wavefront-only change: GPU tests + smoke, c3 bench/rocprof/PMC, c4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02i}
CONFIGS=c3 TAG=$TAG bash tools/gpu_r02.sh || exit 1
timeout -k 10 600 python3 bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/$TAG/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/$TAG/bench_c4.log | cut -c1-300
echo R02I_DONE
