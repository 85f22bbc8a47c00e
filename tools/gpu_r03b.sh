#!/bin/bash
# Round-3 b: the new deep-stack tests, the reference-scene and c4 bench lines, and the counter list for c3 analysis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03b}; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-600; return $rc; }
run pytest_new 300 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "deeper_than or reference_init or group" || exit 1
run bench_ref 300 python3 -u bench.py --config ref || exit 1
run prof_ref 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_ref" -o ref -- python3 bench.py --config ref --no-cpu-baseline --steps 10 --warmup 2 || exit 1
run bench_c4 600 python3 -u bench.py --config c4 --steps 3 --warmup 1 --cpu-seconds 20 || exit 1
run counters 120 rocprofv3 -L || exit 1
echo ALL_DONE
