set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03r; mkdir -p $OUT
export WCPT_LIBRARY=wc-path-tracer_amd/variants/tiletrace.so
for args in "--config c2" "--config c2 --rows 135" "--config ref" "--config c2 --rows 270"; do
  timeout -k 10 300 python3 tools/tile_trace.py $args >> $OUT/tile_trace.log 2>&1 || { tail -5 $OUT/tile_trace.log; exit 1; }
  tail -1 $OUT/tile_trace.log
done
