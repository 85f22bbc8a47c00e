#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-diag}; mkdir -p "$OUT"
for cfg in ${CONFIGS:-c2 c3}; do
  for k in ${KERNELS:-0}; do
    timeout -k 10 300 python3 tools/diag.py --config $cfg --kernel $k > "$OUT/diag_${cfg}_k$k.log" 2>&1; rc=$?
    cat "$OUT/diag_${cfg}_k$k.log" | tail -40
    if [ $rc -ne 0 ]; then echo "rc=$rc"; exit $rc; fi
  done
done
