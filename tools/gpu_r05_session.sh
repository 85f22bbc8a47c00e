#!/bin/bash
# Round 5 session. Steps chosen by env flags; every GPU step has its own time limit and the first failure ends the
# script. TAG names the output directory under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-700; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "${HOST:-0}" = 1 ]; then
  run api_probe 120 tools/host_api_probe 4096
  run group_probe 300 python3 -u tools/host_group_probe.py --ranks 1 2 4 8 --steps 2000
  WCPT_LIBRARY=$PWD/wc-path-tracer_amd/libwcpt_gt.so run group_probe_timers 300 python3 -u tools/host_group_probe.py --ranks 1 8 --steps 2000 --threads 0
fi
if [ "${BENCH:-0}" = 1 ]; then
  run bench_c2 600 python3 -u bench.py
  [ "${BENCH_ALL:-0}" = 1 ] && run bench_ref 300 python3 -u bench.py --config ref --no-cpu-baseline
  [ "${BENCH_ALL:-0}" = 1 ] && run bench_c3 600 python3 -u bench.py --config c3 --no-cpu-baseline
  [ "${C4:-0}" = 1 ] && run bench_c4 900 python3 -u bench.py --config c4 --no-cpu-baseline --steps 20 --warmup 3
  [ "${BENCH_ALL:-0}" = 1 ] && run bench_c2_orbit 300 python3 -u bench.py --camera orbit --no-cpu-baseline
  [ "${BENCH_ALL:-0}" = 1 ] && run bench_ref_orbit 300 python3 -u bench.py --config ref --camera orbit --no-cpu-baseline
fi
if [ "${KTRACE:-0}" = 1 ]; then
  # every dispatch of a c3 135-row block (the N = 8 share) and of the full frame: per-launch durations and how the
  # pipelines' launches overlap (tools/ktrace_summary.py)
  run ktrace_c3_block 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_c3_block" -o kt -- python3 tools/block_balance.py --config c3 --ns 8 --first --frames 10 --rounds 1
fi
if [ "${BALANCE:-0}" = 1 ]; then
  run balance_c2 300 python3 -u tools/block_balance.py --config c2 --ns 2,4,8
  run balance_c3 300 python3 -u tools/block_balance.py --config c3 --ns 2,4,8
  [ "${C4:-0}" = 1 ] && run balance_c4 900 python3 -u tools/block_balance.py --config c4 --ns 8 --frames 6 --rounds 2
fi
if [ "${GROUP:-0}" = 1 ]; then
  run group_c2_g8copy 300 python3 -u bench.py --no-cpu-baseline --gpus 8 --devices 0,0,0,0,0,0,0,0 --transport copy --verify --steps 50 --warmup 10
  run group_c2_g8direct 300 python3 -u bench.py --no-cpu-baseline --gpus 8 --devices 0,0,0,0,0,0,0,0 --transport direct --verify --steps 50 --warmup 10
  run group_c2_g8copy_thr 300 python3 -u bench.py --no-cpu-baseline --gpus 8 --devices 0,0,0,0,0,0,0,0 --transport copy --group-threads 1 --verify --steps 50 --warmup 10
  run rccl_rehearsal_c2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 bench.py --rccl-rehearsal --verify --steps 20 --warmup 5 --watchdog-s 150
  run rccl_rehearsal_c2_n4 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29641 bench.py --rccl-rehearsal --verify --steps 20 --warmup 5 --watchdog-s 150
fi
echo SESSION_DONE
