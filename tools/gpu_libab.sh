#!/bin/bash
# A/B of whole library builds (variants/NAME.so from tools/ab_build.sh vs the in-tree libwcpt.so), alternating
# runs of bench.py in separate processes. Usage: LIBS="base cur" CONFIGS="c2 c3" ROUNDS=2 bash tools/gpu_libab.sh
# ("cur" = the in-tree library). Optional TESTS=1 runs pytest -m gpu on the in-tree library first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-libab}; mkdir -p "$OUT"; export TMPDIR=/tmp
if [ "${TESTS:-0}" = "1" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -n 5 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && { echo "pytest rc=$rc"; exit $rc; }
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${CONFIGS:-c2}; do
    for lib in ${LIBS:-base cur}; do
      if [ "$lib" = "cur" ]; then unset WCPT_LIBRARY; else export WCPT_LIBRARY="wc-path-tracer_amd/variants/$lib.so"; fi
      timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline --steps ${STEPS:-30} ${BENCH_ARGS:-} \
        > "$OUT/${cfg}_${lib}_$r.log" 2>&1 || { echo "bench $cfg $lib failed"; tail -5 "$OUT/${cfg}_${lib}_$r.log"; exit 1; }
      python3 - "$OUT/${cfg}_${lib}_$r.log" "$cfg" "$lib" <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
j = json.loads(line)
print(f"{sys.argv[2]} {sys.argv[3]:>10}: {j['ms_per_step']:.4f} ms/frame  {j['value']:.1f} Mray/s  kernel {j['kernel_ms_avg']:.4f} ms")
PY
    done
  done
done
echo ALL_DONE
