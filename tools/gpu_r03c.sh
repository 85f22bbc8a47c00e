#!/bin/bash
# Round-3 c: reference scene on the wavefront kernel, and load-path counters of c3 / c2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03c}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 120 python3 -u bench.py --config ref --kernel 2 --no-cpu-baseline > $OUT/bench_ref_wf.log 2>&1 || exit 1
tail -c 600 $OUT/bench_ref_wf.log | head -c 300; echo
TAG=${TAG:-r03c} CONFIGS="c3 c2 ref" bash tools/gpu_pmc_passes.sh \
  "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
  "TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCP_TA_ADDR_STALL_CYCLES_sum TCP_TOTAL_ACCESSES_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum"
