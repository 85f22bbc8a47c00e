set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03k; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wavefront or pipelines or c3 or c4 or multi_draw" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
TAG=r03k LIBS="together cur" CONFIGS="c3" ROUNDS=3 STEPS=60 bash tools/gpu_libab.sh
