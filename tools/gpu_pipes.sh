set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "pipelines" --timeout 300 --timeout-method thread > gpurun_out/pytest_pipes.log 2>&1 || { tail -30 gpurun_out/pytest_pipes.log; exit 1; }
tail -1 gpurun_out/pytest_pipes.log
for r in 0 135; do
AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c3 --rows $r --frames 5 --rounds 3 --variants kernel=2 kernel=2,pipes=2 kernel=2,pipes=3 kernel=2,pipes=4 2>&1 | grep -v amdgpu.ids | sed "s/^/rows $r: /" || exit 1
done
echo ALL_DONE
