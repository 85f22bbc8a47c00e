#!/bin/bash
# One GPU session: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel trace. Each GPU step has its own time
# limit; a crash/timeout (exit status other than 0 or 1) ends the script without starting further GPU work.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python3 -m pytest tests -m gpu -x -q
step bench 600 python3 bench.py ${BENCH_ARGS:-}
if [ "${PROF:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-}
fi
echo ALL_DONE
