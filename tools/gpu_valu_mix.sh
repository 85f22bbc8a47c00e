#!/bin/bash
# VALU instruction-class rates (tools/valu_peak) and the VALU class mix of each config's dominant kernel (one --pmc pass
# of 8 SQ counters), for the mix-weighted VALU ceiling of bench.py's roofline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-valumix}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 180 ./tools/valu_peak > "$OUT/valu_peak.log" 2>&1 || { echo valu_peak failed; exit 1; }
tail -7 "$OUT/valu_peak.log"
for cfg in ${CONFIGS:-c2 ref c3}; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT \
    --output-format csv -d "$OUT/mix_$cfg" -o run -- python3 bench.py --config $cfg --no-cpu-baseline --steps 2 --warmup 1 > "$OUT/mix_$cfg.log" 2>&1 || { echo "mix $cfg failed"; tail -3 "$OUT/mix_$cfg.log"; exit 1; }
  echo "mix $cfg ok"
done
echo ALL_DONE
