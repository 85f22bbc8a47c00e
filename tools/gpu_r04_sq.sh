#!/bin/bash
# Round 4: kernel stats + SQ counter passes (issue, stalls, instruction/scalar cache, VALU mix) of the benched build for
# CONFIGS (default c2). One rocprofv3 --pmc pass per counter set, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04_sq}; mkdir -p "$OUT"; export TMPDIR=/tmp
B="--no-cpu-baseline --steps 2 --warmup 1"
for cfg in ${CONFIGS:-c2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o $cfg -- python3 bench.py --config $cfg --no-cpu-baseline --steps 20 --warmup 5 > "$OUT/prof_$cfg.log" 2>&1 || { echo "prof $cfg failed"; tail -3 "$OUT/prof_$cfg.log"; exit 1; }
  tail -1 "$OUT/prof_$cfg.log" | cut -c1-300
  n=0
  for P in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
           "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQC_DCACHE_MISSES SQC_DCACHE_HITS"; do
    n=$((n+1))
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/sq_$cfg/p$n" -o run -- python3 bench.py --config $cfg $B > "$OUT/sq${n}_$cfg.log" 2>&1 || { echo "pass $n $cfg failed"; tail -3 "$OUT/sq${n}_$cfg.log"; exit 1; }
    echo "pass $n $cfg ok"
  done
done
echo ALL_DONE
