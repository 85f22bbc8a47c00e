set -o pipefail
timeout -k 10 300 python3 tools/block_balance.py --config c3 --frames 4 --rounds 2 --ns 2,4,8,16,32,64 --first 2>&1 | grep -v amdgpu.ids
mkdir -p gpurun_out/sweep && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sweep -o c3 -- python3 tools/block_balance.py --config c3 --frames 2 --rounds 1 --ns 8,64 --first > gpurun_out/sweep/log 2>&1
