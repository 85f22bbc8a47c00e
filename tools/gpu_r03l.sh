#!/bin/bash
# wf_trace micro-optimisations: buffer-resource child-pair loads and the full-rate 24-bit multiply, A/B on c3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03l}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wavefront or pipelines or c3 or multi_draw or deeper or boundary" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=${TAG:-r03l} LIBS="base0 rsrconly mul24only cur" CONFIGS="c3" ROUNDS=3 STEPS=60 bash tools/gpu_libab.sh
