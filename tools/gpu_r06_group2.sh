#!/bin/bash
# Round 6: 8 spawned ranks on one GPU (RCCL over sockets) with row blocks and with row stripes, and a 4-rank c3 frame
# (wavefront kernel, path-persistent trace on its blocks) over the same path, each presented frame verified.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_group2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-300; [ $rc -eq 0 ] || exit 1; }
run spawn_c2_n8 300 python3 bench.py --gpus 8 --rccl-rehearsal --verify --steps 40 --warmup 10 --no-cpu-baseline --watchdog-s 200
run spawn_c2_n8_stripe8 300 python3 bench.py --gpus 8 --rccl-rehearsal --row-stripe 8 --verify --steps 40 --warmup 10 --no-cpu-baseline --watchdog-s 200
run spawn_c3_n4_stripe8 300 python3 bench.py --gpus 4 --config c3 --rccl-rehearsal --row-stripe 8 --verify --steps 10 --warmup 3 --no-cpu-baseline --watchdog-s 200
run onepro_c2_n4_copy_stripe8 300 python3 bench.py --gpus 4 --one-process --transport copy --devices 0,0,0,0 --row-stripe 8 --verify --steps 40 --warmup 10 --no-cpu-baseline
echo SESSION_DONE
