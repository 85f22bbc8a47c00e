#!/bin/bash
# Round 6: frame overlap through a plain context and a one-rank group (tools/overlap_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_overlap_ab2}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for cfg in ${CONFIGS:-c2 ref}; do
  echo "=== $cfg $(date +%T)"
  timeout -k 10 300 python3 tools/overlap_ab.py --config $cfg ${ARGS:-} > "$OUT/$cfg.log" 2>&1 || { tail -5 "$OUT/$cfg.log"; exit 1; }
  grep median "$OUT/$cfg.log"
done
echo SESSION_DONE
