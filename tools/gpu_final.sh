set -o pipefail
mkdir -p gpurun_out/v10
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_v10.log 2>&1 || { tail -30 gpurun_out/pytest_v10.log; exit 1; }
tail -1 gpurun_out/pytest_v10.log
CONFIGS=c3 TAG=v10 bash tools/gpu_bench.sh || exit 1
timeout -k 10 600 python3 bench.py --config c4 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/v10/bench_c4.log 2>&1 || { tail -5 gpurun_out/v10/bench_c4.log; exit 1; }
timeout -k 10 600 python3 bench.py --config c3 --bvh sah --no-cpu-baseline > gpurun_out/v10/bench_c3_sah.log 2>&1 || { tail -5 gpurun_out/v10/bench_c3_sah.log; exit 1; }
timeout -k 10 600 python3 bench.py --config c4 --bvh sah --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/v10/bench_c4_sah.log 2>&1 || { tail -5 gpurun_out/v10/bench_c4_sah.log; exit 1; }
for f in bench_c4 bench_c3_sah bench_c4_sah; do echo "$f: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' gpurun_out/v10/$f.log | tr '\n' ' ')"; done
echo ALL_DONE
