#!/bin/bash
# Memory-pipeline PMC passes for the dominant kernel. Usage: TAG=x BENCH_ARGS="--config c3 --kernel 2" bash tools/pmc_mem.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmcmem}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-}"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "=== pass $i: $counters"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- python3 bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?; echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; if [ $rc -ne 1 ]; then echo ABORT; exit $rc; fi; fi
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
TD_TD_BUSY_sum TD_TC_STALL_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE
TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_THRASHING_STALL_sum
TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE
WRITE_SIZE
LIST
echo PMC_DONE
