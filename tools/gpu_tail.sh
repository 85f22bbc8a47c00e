set -o pipefail
for cfg in c2 c3; do for r in 8 0; do
AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config $cfg --rows $r --frames 5 --rounds 2 --variants kernel=2 kernel=0 2>&1 | grep -v amdgpu.ids | sed "s/^/rows $r: /" || exit 1
done; done
mkdir -p gpurun_out/tail && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tail -o c2 -- python3 tools/ab.py --config c2 --rows 8 --frames 3 --rounds 1 --variants kernel=2 > gpurun_out/tail/log 2>&1
echo ALL_DONE
