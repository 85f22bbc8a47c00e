#!/bin/bash
# Round bench session: for each config, bench (with CPU baseline for the default one), rocprofv3 kernel stats,
# and FETCH/WRITE PMC passes for the dominant kernel. GPU steps chained: any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bench}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-400; return $rc; }
for cfg in ${CONFIGS:-c2 c3}; do
  extra=""; [ "$cfg" != "c2" ] && extra="--no-cpu-baseline"
  run bench_$cfg 600 python3 bench.py --config $cfg $extra || exit 1
  run prof_$cfg 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$cfg" -o $cfg -- python3 bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 2 || exit 1
  run pmcf_$cfg 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_$cfg/p1" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit 1
  run pmcw_$cfg 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_$cfg/p2" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 || exit 1
done
echo ALL_DONE
