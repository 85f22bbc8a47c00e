#!/bin/bash
# The counter passes bench.py's roofline is priced from, on the library that is loaded (its wcpt_build_id is recorded in
# $OUT/build_id): kernel stats, FETCH_SIZE and WRITE_SIZE (HBM traffic), the SQ issue/stall sets and the VALU class mix,
# for CONFIGS (default "c2 ref c3 c4"; a "_orbit" suffix runs the config with the moving camera, bench.py --camera
# orbit). One rocprofv3 --pmc pass per counter set, each under its own time limit. Summarise with
# tools/profile_summaries.py on the host. EXTRA_PASSES=1 adds the instruction/scalar-cache passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sq}; mkdir -p "$OUT"; export TMPDIR=/tmp
python3 -c "import sys; sys.path.insert(0, 'wc-path-tracer_amd'); import wcpt; print(wcpt.build_id())" > "$OUT/build_id" || exit 1
for cfg in ${CONFIGS:-c2 ref c3 c4}; do
  base=${cfg%_orbit}; CAM=""; [ "$base" != "$cfg" ] && CAM="--camera orbit"
  # the moving camera's passes skip the untimed settle phase: its frames repeat the first camera position (bench.py
  # renders frame 0 for --settle-ms), which would otherwise make up most of the dispatches the counters average over
  SETTLE=""; [ -n "$CAM" ] && SETTLE="--settle-ms 0 --steps 6 --warmup 0"
  B="--config $base $CAM --no-cpu-baseline --steps 2 --warmup 1 $SETTLE"
  [ "$cfg" = c4 ] && B="--config $cfg --no-cpu-baseline --steps 1 --warmup 0 --settle-ms 0"
  # the kernel-stats run is the bench line's own command (tools/gpu_r05_session.sh: default steps and warmup, c4 20 + 3),
  # so the rocprof average covers the same frames under the same sustained load as the bench's HIP events
  PB=""; [ "$cfg" = c4 ] && PB="--steps 20 --warmup 3"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o $cfg -- python3 bench.py --config $base $CAM --no-cpu-baseline $PB > "$OUT/prof_$cfg.log" 2>&1 || { echo "prof $cfg failed"; tail -3 "$OUT/prof_$cfg.log"; exit 1; }
  echo "prof $cfg ok"
  n=0
  PASSES=("FETCH_SIZE" "WRITE_SIZE" \
          "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES" \
          "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM" \
          "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
          "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
          "SQ_INSTS_VALU SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32")
  [ "${EXTRA_PASSES:-0}" = 1 ] && PASSES+=("SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES" "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQC_DCACHE_MISSES SQC_DCACHE_HITS")
  for P in "${PASSES[@]}"; do
    n=$((n+1))
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/sq_$cfg/p$n" -o run -- python3 bench.py $B > "$OUT/sq${n}_$cfg.log" 2>&1 || { echo "pass $n $cfg failed"; tail -3 "$OUT/sq${n}_$cfg.log"; exit 1; }
    echo "pass $n $cfg ok"
  done
done
echo ALL_DONE
