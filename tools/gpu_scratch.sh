set -o pipefail
AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c2 --rows 8 --frames 5 --rounds 2 --variants kernel=2 2>&1 | grep -v amdgpu.ids | sed "s/^/default: /" || exit 1
HSA_SCRATCH_SINGLE_LIMIT=4000000000 AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c2 --rows 8 --frames 5 --rounds 2 --variants kernel=2 2>&1 | grep -v amdgpu.ids | sed "s/^/limit4G: /" || exit 1
HSA_SCRATCH_SINGLE_LIMIT=4000000000 AB_TORCH_FIRST=1 timeout -k 10 300 python3 tools/ab.py --config c3 --rows 0 --frames 5 --rounds 2 --variants kernel=2 kernel=2,pipes=2 2>&1 | grep -v amdgpu.ids | sed "s/^/limit4G: /" || exit 1
echo ALL_DONE
