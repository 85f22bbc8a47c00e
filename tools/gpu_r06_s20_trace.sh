#!/bin/bash
# Round 6: kernel traces of the driver's short bench window (--steps 20 --warmup 5) with the frame overlap off and on.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_s20_trace}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for ov in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_ov$ov" -o kt -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 --frame-overlap $ov > "$OUT/bench_ov$ov.log" 2>&1 || { tail -3 "$OUT/bench_ov$ov.log"; exit 1; }
  tail -1 "$OUT/bench_ov$ov.log" | cut -c1-120 | head -1
  python3 -c "import json; d=json.loads(open('$OUT/bench_ov$ov.log').read().strip().splitlines()[-1]); print('ov$ov', d['ms_per_step'])"
  python3 tools/launch_durations.py "$OUT/kt_ov$ov" --last 200 > "$OUT/durations_ov$ov.log" || exit 1
  f=$(find "$OUT/kt_ov$ov" -name "*kernel_trace.csv" | head -1); cp "$f" "$OUT/kernel_trace_ov$ov.csv"; rm -rf "$OUT/kt_ov$ov"
done
echo SESSION_DONE
