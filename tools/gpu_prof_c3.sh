set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/profc3
cd /tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profc3/kt -o c3 -- python3 bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/profc3/bench.log 2>&1
echo rc=$?
