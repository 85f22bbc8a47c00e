#!/bin/bash
# Issue-stall counters of a config's render (instruction fetch, scalar cache, SALU/SMEM cycles), one --pmc pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sqstall}; mkdir -p "$OUT"; export TMPDIR=/tmp
n=0
for P in "SQ_IFETCH SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INST_CYCLES_SMEM SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_WAVE_CYCLES" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS" "SQC_DCACHE_MISSES SQC_DCACHE_HITS"; do
  n=$((n+1))
  for cfg in ${CONFIGS:-c2}; do
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/$cfg/p$n" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/${cfg}_p$n.log" 2>&1 || { echo "pass $n $cfg failed"; tail -3 "$OUT/${cfg}_p$n.log"; exit 1; }
    echo "pass $n $cfg ok"
  done
done
echo ALL_DONE
