#!/bin/bash
# L2 hit rate + SQ issue/wait breakdown of the dominant kernels (separate --pmc passes, kernel trace only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
n=1
for cfg in ${CONFIGS:-c3 c2}; do
  for pmc in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES"; do
    PMC="$pmc" TAG=${TAG:-cache}_$cfg N=$n BENCH_ARGS="--config $cfg ${EXTRA:-}" bash tools/pmc_one.sh || exit 1
    n=$((n+1))
  done
done
echo ALL_DONE
