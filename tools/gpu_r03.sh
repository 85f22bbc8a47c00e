# Round-3 GPU check: the -m gpu suite, then (if green) the default bench line. Usage: bash tools/gpu_r03.sh <tag>
set -o pipefail
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 200 --warmup 100 > $out/bench_c2.log 2>&1
