#!/bin/bash
# Round-3 d: SIMD efficiency and SQ passes of the reference Init scene on the megakernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03d}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python3 tools/diag.py --config ref --kernel 0 > $OUT/diag_ref.log 2>&1 || { tail -5 $OUT/diag_ref.log; exit 1; }
tail -30 $OUT/diag_ref.log
TAG=${TAG:-r03d} CONFIGS="ref" bash tools/gpu_pmc_passes.sh \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM" \
  "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
