#!/bin/bash
# Round 4: the reworked multi-rank group on one GPU (COPY-transport rehearsals, overlap, failure atomicity), the
# group-of-one bench against the round-3 context path, and the moving-camera mode. TAG names the output directory.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04_group}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; tail -c 700 "$OUT/$name.log"; echo; [ $rc -eq 0 ] || { echo "$name failed rc=$rc"; exit 1; }; }
run pytest_multi 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py ${PYTEST_K:+-k "$PYTEST_K"}
run bench_c2_g1 300 python3 -u bench.py --no-cpu-baseline
run bench_c2_g3copy 300 python3 -u bench.py --no-cpu-baseline --gpus 3 --devices 0,0,0 --transport copy --verify --steps 50 --warmup 10
run bench_c2_g2copy_display 300 python3 -u bench.py --no-cpu-baseline --gpus 2 --devices 0,0 --transport copy --gather display --verify --steps 50 --warmup 10
run bench_c2_g2copy_inline 300 python3 -u bench.py --no-cpu-baseline --gpus 2 --devices 0,0 --transport copy --no-overlap --verify --steps 50 --warmup 10
run bench_c2_orbit 300 python3 -u bench.py --no-cpu-baseline --camera orbit
echo SESSION_DONE
