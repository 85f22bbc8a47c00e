#!/bin/bash
# Round-2 GPU session: GPU parity tests, smoke, then bench + rocprof stats + FETCH/WRITE PMC passes per config.
# Every GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r02}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 \
    || { tail -10 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
[ "${SKIP_BENCH:-0}" = 1 ] && { echo ALL_DONE; exit 0; }
CONFIGS=${CONFIGS:-c2 c3} TAG=$TAG bash tools/gpu_bench.sh || exit 1
echo ALL_DONE
