#!/bin/bash
# Round-3 measurement session on one MI355X: GPU tests, the bench line per config, rocprofv3 kernel stats, the HBM
# (FETCH_SIZE / WRITE_SIZE) and SQ counter passes, and the two ceilings the roofline is priced against
# (tools/valu_peak, tools/gather_bench). Every GPU step has its own time limit; the first failure ends the script.
#   TAG=r03a [TESTS=1] [CONFIGS="c2 c3 ref"] bash tools/gpu_r03_measure.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-600; return $rc; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1
fi
if [ "${CEILINGS:-1}" = 1 ]; then
  run valu_peak 120 ./tools/valu_peak || exit 1
  run gather_ceiling 180 ./tools/gather_bench 64 4096 9216 16384 24576 524288 || exit 1
fi
for cfg in ${CONFIGS:-c2 c3}; do
  extra=""; [ "$cfg" != "c2" ] && extra="--no-cpu-baseline"
  run bench_$cfg 600 python3 -u bench.py --config $cfg $extra || exit 1
  [ "${PROF:-1}" = 1 ] || continue
  run prof_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o $cfg -- python3 bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 2 || exit 1
  run pmcf_$cfg 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$cfg/p1" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit 1
  run pmcw_$cfg 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$cfg/p2" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit 1
  n=0
  for P in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM" \
           "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
    n=$((n+1))
    run sq${n}_$cfg 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/sq_$cfg/p$n" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit 1
  done
done
echo ALL_DONE
