#!/bin/bash
# Round 6 A/B: the wavefront queue counters zeroed by the previous frame's ray generation (in-tree, WCPT_WF_CTR_PARITY)
# against a memset per pipeline and frame (variant noparity) on c3 / c4; the megakernel's software-pipelined pair
# records (variant pf, WCPT_PAIR_PREFETCH) against the in-tree build on c2 / ref. GPU suite on the in-tree build first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_ab2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -20 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
WCPT_LIBRARY=wc-path-tracer_amd/variants/pf.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "frame or full or c2 or primary or pair" > "$OUT/pytest_pf.log" 2>&1 || { tail -20 "$OUT/pytest_pf.log"; exit 1; }
tail -1 "$OUT/pytest_pf.log"
TAG=$TAG/wf LIBS="noparity cur" CONFIGS="c3" ROUNDS=3 STEPS=100 bash tools/gpu_libab.sh || exit 1
TAG=$TAG/c4 LIBS="noparity cur" CONFIGS="c4" ROUNDS=2 STEPS=10 BENCH_ARGS="--warmup 2" bash tools/gpu_libab.sh || exit 1
TAG=$TAG/mk LIBS="pf cur" CONFIGS="c2 ref" ROUNDS=3 STEPS=200 bash tools/gpu_libab.sh || exit 1
echo SESSION_DONE
