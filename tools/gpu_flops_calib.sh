#!/bin/bash
# Calibrate SQ_INSTS_VALU_FLOPS_FP32 against known instruction streams (tools/valu_peak: v_add/v_mul/v_fma and their
# packed forms, full exec) and collect the same pass on c2, to split c2's FP32 add/mul/fma counts into packed and
# single instructions. One --pmc pass per program, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-flops_calib}; mkdir -p "$OUT"; export TMPDIR=/tmp
P="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_THREAD_CYCLES_VALU"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/peak" -o run -- ./tools/valu_peak > "$OUT/peak.log" 2>&1 || { echo "peak pass failed"; tail -3 "$OUT/peak.log"; exit 1; }
echo "peak ok"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/c2" -o run -- python3 bench.py --config c2 --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/c2.log" 2>&1 || { echo "c2 pass failed"; tail -3 "$OUT/c2.log"; exit 1; }
echo "c2 ok"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d "$OUT/ref" -o run -- python3 bench.py --config ref --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/ref.log" 2>&1 || { echo "ref pass failed"; tail -3 "$OUT/ref.log"; exit 1; }
echo ALL_DONE
