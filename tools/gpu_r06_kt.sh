#!/bin/bash
# Round 6: kernel trace of a short bench (CONFIG, default c3) (per-pipeline timeline, tools/ktrace_summary.py) and the device-idle gaps
# between its launches (tools/frame_gaps.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIG=${CONFIG:-c3}; OUT=gpurun_out/${TAG:-r06_kt}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/kt_$CONFIG" -o kt -- python3 bench.py --config $CONFIG --no-cpu-baseline --steps ${STEPS:-12} --warmup 3 --settle-ms 50 > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 1; }
python3 tools/ktrace_summary.py "$OUT/kt_$CONFIG" --pipes 3 > "$OUT/summary.log" 2>&1 || echo "(no pipeline summary for $CONFIG)"
python3 tools/frame_gaps.py "$OUT/kt_$CONFIG" > "$OUT/gaps.log" || exit 1
head -45 "$OUT/summary.log"; head -40 "$OUT/gaps.log"
f=$(find "$OUT/kt_$CONFIG" -name "*kernel_trace.csv" | head -1); cp "$f" "$OUT/kernel_trace.csv"; rm -rf "$OUT/kt_$CONFIG"
echo DONE
