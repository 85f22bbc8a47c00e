set -u
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s5.log 2>&1 || { tail -30 gpurun_out/pytest_s5.log; exit 1; }
tail -1 gpurun_out/pytest_s5.log
for r in 135 270 0; do
AB_TORCH_FIRST=1 timeout -k 10 200 python3 tools/ab.py --config c2 --rows $r --frames 20 --rounds 3 --variants stack=0 stack=1 stack=0,order=0 stack=1,order=0 2>&1 | grep -v amdgpu.ids | sed "s/^/rows $r: /" || exit 1
done
echo ALL_DONE
