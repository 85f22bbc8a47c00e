#!/bin/bash
# Round 6: frame-to-frame overlap headroom (tools/stream_overlap.py): K contexts rendering round-robin against one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_overlap}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; cut -c1-200 "$OUT/$name.log"; [ $rc -eq 0 ] || exit 1; }
run c2 200 python3 tools/stream_overlap.py --config c2 --contexts 1,2,3,1 --frames 120
run ref 200 python3 tools/stream_overlap.py --config ref --contexts 1,2,1 --frames 60
run c3 300 python3 tools/stream_overlap.py --config c3 --contexts 1,2,1 --frames 30
echo SESSION_DONE
