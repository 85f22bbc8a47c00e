#!/bin/bash
# Parity subset on the in-tree library, then an A/B of library variants against it on c3.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-variantab}; mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "frame_parity or c3_full_frame or wavefront or random_scenes or edge_inputs or multi_draw or deeper or c4_bands or reference_init" \
  > "$OUT/pytest_subset.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_subset.log"; [ $rc -ne 0 ] && exit $rc
TAG=${TAG:-variantab} LIBS="${LIBS:-geo1 cur}" CONFIGS="${CONFIGS:-c3}" ROUNDS=${ROUNDS:-2} bash tools/gpu_libab.sh
