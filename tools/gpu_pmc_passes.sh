#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, --kernel-trace only) of bench.py for the configs in CONFIGS.
#   TAG=x CONFIGS="c3 c2" bash tools/gpu_pmc_passes.sh "PASS1 counters" "PASS2 counters" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmcx}; mkdir -p "$OUT"; export TMPDIR=/tmp
for cfg in ${CONFIGS:-c3}; do
  n=0
  for P in "$@"; do
    n=$((n+1))
    echo "=== $cfg pass $n: $P"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/$cfg/p$n" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$OUT/${cfg}_p$n.log" 2>&1
    rc=$?; echo "rc=$rc"; [ $rc -ne 0 ] && { tail -3 "$OUT/${cfg}_p$n.log"; exit $rc; }
  done
done
echo PMC_DONE
