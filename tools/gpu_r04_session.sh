#!/bin/bash
# Round 4 session: GPU tests, smoke, bench lines (c2 with the CPU baseline, ref, c3, c4; still and orbiting camera),
# N-rank group rehearsals on one GPU (COPY transport, verified bit-exact) and the torch.distributed rehearsal path.
# Every GPU step has its own time limit; the first failure ends the script. TAG names the output directory.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 1 "$OUT/$name.log" | cut -c1-400; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${BENCH:-1}" = 1 ]; then
  run bench_c2 600 python3 -u bench.py
  run bench_ref 300 python3 -u bench.py --config ref --no-cpu-baseline
  run bench_c2_orbit 300 python3 -u bench.py --camera orbit --no-cpu-baseline
  run bench_ref_orbit 300 python3 -u bench.py --config ref --camera orbit --no-cpu-baseline
  run bench_c3 600 python3 -u bench.py --config c3 --no-cpu-baseline
  [ "${C4:-1}" = 1 ] && run bench_c4 900 python3 -u bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 3
fi
if [ "${GROUP:-1}" = 1 ]; then
  run group_c2_g4copy 300 python3 -u bench.py --no-cpu-baseline --gpus 4 --devices 0,0,0,0 --transport copy --verify --steps 50 --warmup 10
  run group_c3_g3copy 300 python3 -u bench.py --config c3 --no-cpu-baseline --gpus 3 --devices 0,0,0 --transport copy --verify --gather display --steps 10 --warmup 3
  run torch_gloo_c2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --dist-backend gloo --verify --steps 20 --warmup 5 --watchdog-s 120
fi
if [ "${BALANCE:-1}" = 1 ]; then
  run balance_c2 300 python3 -u tools/block_balance.py --config c2 --ns 2,4,8
  run balance_c3 300 python3 -u tools/block_balance.py --config c3 --ns 2,4,8
fi
echo SESSION_DONE
