#!/bin/bash
# c3 trace: share of the waves' time spent after the queue drained (DIAG build timers), one pipeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03m}; mkdir -p $OUT
timeout -k 10 300 python3 tools/diag.py --config c3 --kernel 2 > $OUT/diag_c3.log 2>&1 || { tail -5 $OUT/diag_c3.log; exit 1; }
tail -22 $OUT/diag_c3.log
