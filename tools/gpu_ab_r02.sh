#!/bin/bash
# Round-2 A/B: GPU parity tests on the in-tree library, then alternating bench runs of variant builds.
# LIBS / CONFIGS / ROUNDS as tools/gpu_libab.sh. Every GPU step has its own limit; failures end the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-ab}; mkdir -p gpurun_out/$TAG
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
TAG=$TAG bash tools/gpu_libab.sh || exit 1
