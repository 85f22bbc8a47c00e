#!/bin/bash
# Round-3 e: is the c3 trace VALU-bound once both pipelines share the SIMDs? SQ passes with one pipeline (the trace
# alone at 8 waves/SIMD) and pipes 1/2 timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03e}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 200 python3 tools/ab.py --config c3 --variants "kernel=2,pipes=1" "kernel=2,pipes=2" --frames 4 --rounds 2 > $OUT/ab_pipes.log 2>&1 || { tail -3 $OUT/ab_pipes.log; exit 1; }
cat $OUT/ab_pipes.log
TAG=${TAG:-r03e} CONFIGS="c3" BENCH_ARGS="--wf-pipes 1" bash tools/gpu_pmc_passes.sh \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
