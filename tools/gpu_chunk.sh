set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "wavefront or pipelines or random or WAVEFRONT or rows" --timeout 300 --timeout-method thread > gpurun_out/pytest_chunk.log 2>&1 || { tail -30 gpurun_out/pytest_chunk.log; exit 1; }
tail -1 gpurun_out/pytest_chunk.log
AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c2 --rows 8 --frames 5 --rounds 2 --variants kernel=2 2>&1 | grep -v amdgpu.ids | sed "s/^/rows 8: /" || exit 1
for r in 135 0; do
AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c3 --rows $r --frames 5 --rounds 3 --variants kernel=2 kernel=2,pipes=2 kernel=2,pipes=3 kernel=0 2>&1 | grep -v amdgpu.ids | sed "s/^/rows $r: /" || exit 1
done
LIBS="chunk128 chunk256 cur" CONFIGS=c3 ROUNDS=2 STEPS=20 bash tools/gpu_libab.sh 2>&1 | grep -v amdgpu.ids || exit 1
