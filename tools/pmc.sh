#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only with --kernel-trace; no sys/runtime traces).
# Usage: TAG=name BENCH_ARGS="--config c3" bash tools/pmc.sh ; then python tools/pmc_summary.py gpurun_out/<TAG>/pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 3 --warmup 1 ${BENCH_ARGS:-}"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; if [ $rc -ne 1 ]; then echo ABORT; exit $rc; fi; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
LIST
echo PMC_DONE
