set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_v9.log 2>&1 || { tail -30 gpurun_out/pytest_v9.log; exit 1; }
tail -1 gpurun_out/pytest_v9.log
TAG=v9 bash tools/gpu_bench.sh || exit 1
timeout -k 10 600 python3 bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/v9/bench_c4.log 2>&1 || { tail -5 gpurun_out/v9/bench_c4.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/v9/bench_c4.log
echo ALL_DONE
