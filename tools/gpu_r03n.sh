#!/bin/bash
# Long-first wavefront queue order: parity tests, then thresholds on c3 / c4 block / ref (wavefront).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03n}; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "wavefront or pipelines or c3 or multi_draw or deeper or boundary or long_first" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python3 tools/ab.py --config c3 --variants "kernel=2,lf=0" "kernel=2,lf=64" "kernel=2,lf=128" "kernel=2,lf=256" "kernel=2,lf=512" --frames 5 --rounds 3 > $OUT/ab_c3.log 2>&1 || { tail -3 $OUT/ab_c3.log; exit 1; }
cat $OUT/ab_c3.log
timeout -k 10 400 python3 tools/ab.py --config c4 --rows 270 --variants "kernel=2,lf=0" "kernel=2,lf=128" "kernel=2,lf=256" --frames 2 --rounds 2 > $OUT/ab_c4.log 2>&1 || { tail -3 $OUT/ab_c4.log; exit 1; }
cat $OUT/ab_c4.log
