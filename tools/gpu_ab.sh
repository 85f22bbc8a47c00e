#!/bin/bash
# GPU tests + A/B of kernel variants. Usage: TAG=x AB="--config c3 --variants stack=0 stack=1" bash tools/gpu_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n 30 "$OUT/$name.log"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo ABORT; exit $rc; fi; }
if [ "${TESTS:-1}" = "1" ]; then step pytest_gpu 900 python3 -m pytest tests -m gpu -x -q; fi
step ab 600 python3 tools/ab.py ${AB:-}
if [ -n "${AB2:-}" ]; then step ab2 600 python3 tools/ab.py ${AB2}; fi
echo ALL_DONE
