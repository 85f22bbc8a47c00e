#!/bin/bash
# Row-block A/B of library variants: tools/ab.py on the first ROWS rows (an N-way split's block) per variant library.
# Usage: LIBS="base cur" CONFIG=c2 ROWS=135 bash tools/gpu_rows_ab.sh   ("cur" = the in-tree library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-rowsab}; mkdir -p "$OUT"
for lib in ${LIBS:-base cur}; do
  if [ "$lib" = "cur" ]; then unset WCPT_LIBRARY; else export WCPT_LIBRARY="wc-path-tracer_amd/variants/$lib.so"; fi
  timeout -k 10 200 python3 tools/ab.py --config ${CONFIG:-c2} --rows ${ROWS:-135} --variants kernel=${KERNEL:-0} \
      --frames ${FRAMES:-20} --rounds ${ROUNDS:-3} > "$OUT/${lib}.log" 2>&1 || { echo "$lib failed"; tail -5 "$OUT/${lib}.log"; exit 1; }
  echo "$lib: $(tail -1 "$OUT/${lib}.log")"
done
