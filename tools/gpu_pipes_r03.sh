set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 300 python3 tools/ab.py --config c3 --variants "kernel=2,pipes=2" "kernel=2,pipes=3" "kernel=2,pipes=4" --frames 5 --rounds 3 > $OUT/ab_c3.log 2>&1 || { tail -3 $OUT/ab_c3.log; exit 1; }
cat $OUT/ab_c3.log
timeout -k 10 300 python3 tools/ab.py --config c4 --rows 270 --variants "kernel=2,pipes=2" "kernel=2,pipes=3" --frames 2 --rounds 2 > $OUT/ab_c4.log 2>&1 || { tail -3 $OUT/ab_c4.log; exit 1; }
cat $OUT/ab_c4.log
