# Kernel timeline of the emulated N-way step (tools/step_emulate.py) for one split.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-emu}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/prof -o emu -- python3 tools/step_emulate.py --ns ${NS:-8} --steps 50 --warmup 5 > $OUT/log 2>&1 || { tail $OUT/log; exit 1; }
grep "^N=" $OUT/log
echo ALL_DONE
