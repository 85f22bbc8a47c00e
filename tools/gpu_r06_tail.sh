#!/bin/bash
# Round 6: the per-frame fixed cost (launch gap + last-round tail) of c2 / c3 / c4 from a height sweep
# (tools/launch_tail.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_tail}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; cat "$OUT/$name.log" | cut -c1-200; [ $rc -eq 0 ] || exit 1; }
run c2 200 python3 tools/launch_tail.py --config c2 --heights 540,1080,1620,2160,4320
run ref 200 python3 tools/launch_tail.py --config ref --heights 540,1080,2160
run c3 300 python3 tools/launch_tail.py --config c3 --heights 540,1080,2160 --frames 12
echo SESSION_DONE
