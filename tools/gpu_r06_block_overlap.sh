#!/bin/bash
# Round 6: the frame overlap forced on row blocks (one context, region timing): what a group sender could gain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r06_block_overlap}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for spec in "c2 8,0" "c2 8,7" "c2 4,0" "c2 2,0" "ref 8,0" "c3 8,0" "c3 4,0"; do
  set -- $spec
  n=${1}_$(echo $2 | tr , _)
  echo "=== $n $(date +%T)"
  timeout -k 10 300 python3 tools/overlap_ab.py --config $1 --modes ctx --values ${VALUES:-0,2} --block $2 --frames 300 > "$OUT/$n.log" 2>&1 || { tail -5 "$OUT/$n.log"; exit 1; }
  grep median "$OUT/$n.log"
done
echo SESSION_DONE
