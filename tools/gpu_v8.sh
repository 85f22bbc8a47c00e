set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_v8.log 2>&1 || { tail -30 gpurun_out/pytest_v8.log; exit 1; }
tail -1 gpurun_out/pytest_v8.log
TAG=v8 bash tools/gpu_bench.sh || exit 1
AB_TORCH_FIRST=1 timeout -k 10 400 python3 tools/ab.py --config c4 --rows 270 --frames 2 --rounds 2 --variants kernel=2 kernel=2,pipes=2 kernel=2,pipes=3 2>&1 | grep -v amdgpu.ids | sed "s/^/c4 rows 270: /" || exit 1
echo ALL_DONE
