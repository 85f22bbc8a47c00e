#!/bin/bash
# Round-2 closing measurements: GPU tests + smoke, bench/rocprof/PMC for c2 and c3, SQ passes for c2, c4 bench,
# row-block balance and the emulated N=8 step. Every GPU step has its own limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02e}
TAG=$TAG bash tools/gpu_r02.sh || exit 1
TAG=sq_$TAG CONFIGS=c2 bash tools/gpu_sq_r02.sh || exit 1
timeout -k 10 600 python3 bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/$TAG/bench_c4.log 2>&1 || exit 1
tail -1 gpurun_out/$TAG/bench_c4.log | cut -c1-300
timeout -k 10 300 python3 tools/block_balance.py --config c2 > gpurun_out/$TAG/balance_c2.log 2>&1 || exit 1
timeout -k 10 300 python3 tools/step_emulate.py --config c2 --ns 8 --steps 300 --warmup 20 > gpurun_out/$TAG/step_c2_n8.log 2>&1 || exit 1
tail -4 gpurun_out/$TAG/balance_c2.log; grep N= gpurun_out/$TAG/step_c2_n8.log
echo R02E_DONE
