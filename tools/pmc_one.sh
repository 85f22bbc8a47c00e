#!/bin/bash
# One rocprofv3 --pmc pass: PMC="counters" TAG=x N=k BENCH_ARGS=... bash tools/pmc_one.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc1}/pmc; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 ${T:-150} rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d "$OUT/p${N:-1}" -o run -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 ${BENCH_ARGS:-} > "$OUT/p${N:-1}.log" 2>&1
rc=$?; echo "pass ${N:-1} rc=$rc"; [ $rc -ne 0 ] && tail -3 "$OUT/p${N:-1}.log"; exit $rc
