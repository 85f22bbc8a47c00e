#!/bin/bash
# SQ/TCC counter passes (one rocprofv3 --pmc run each, --kernel-trace only) for c2 (megakernel) and c3 (wavefront).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-sq}
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
for cfg in ${CONFIGS:-c2 c3}; do
  n=0
  for P in "$P1" "$P2" "$P3"; do
    n=$((n+1))
    PMC="$P" TAG=${TAG}_$cfg N=$n T=120 BENCH_ARGS="--config $cfg" bash tools/pmc_one.sh || exit 1
  done
done
echo SQ_DONE
