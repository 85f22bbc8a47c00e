#!/bin/bash
# Round 6: the bounded group sync (a peer that skips a frame -> DEVICE_LOST, not a hang), the plain
# `bench.py --gpus N` spawner (one fresh process per rank) rehearsed on one GPU over RCCL's socket transport, with
# contiguous row blocks and with interleaved row stripes (RCCL staging + scatter), and the new GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_group}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-600; [ $rc -eq 0 ] || exit 1; }
run fault_probe 170 python3 tools/group_fault_probe.py --ranks 2 --timeout-ms 3000 --json "$OUT/fault_probe.json"
for n in ${RANKS:-2 4}; do
  run spawn_c2_n$n 240 python3 bench.py --gpus $n --rccl-rehearsal --verify --steps 50 --warmup 10 --no-cpu-baseline --watchdog-s 150
done
run spawn_c2_n4_stripe8 240 python3 bench.py --gpus 4 --rccl-rehearsal --row-stripe 8 --verify --steps 50 --warmup 10 --no-cpu-baseline --watchdog-s 150
run spawn_c2_n3_stripe8_display 240 python3 bench.py --gpus 3 --rccl-rehearsal --row-stripe 8 --gather display --verify --steps 30 --warmup 5 --no-cpu-baseline --watchdog-s 150
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_stripes 600 python3 -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread -k "stripe or direct or n_ranks"
fi
echo SESSION_DONE
