#!/bin/bash
# Round 5 A/B session: GPU tests (in-tree library), the parity tests on a variant library, interleaved bench A/B of
# variants against the in-tree build (tools/gpu_libab.sh), and the c3 135-row block at 1-4 wavefront pipelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r05_ab}; OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; tail -n 3 "$OUT/$name.log" | cut -c1-500; [ $rc -eq 0 ] || exit 1; }
if [ "${TESTS:-1}" = 1 ]; then
  run pytest_gpu 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
for v in ${VARIANT_TESTS:-}; do
  WCPT_LIBRARY=$PWD/wc-path-tracer_amd/variants/$v.so run pytest_gpu_$v 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread
done
if [ -n "${LIBS:-}" ]; then
  TAG=$TAG/libab run libab 1200 bash tools/gpu_libab.sh
fi
for r in $(seq 1 ${BLOCK_ROUNDS:-0}); do
  for v in ${BLOCK_VARIANTS:-}; do
    if [ "$v" = cur ]; then unset WCPT_LIBRARY; else export WCPT_LIBRARY=$PWD/wc-path-tracer_amd/variants/$v.so; fi
    run block_${BLOCK_CONFIG:-c2}_${v}_$r 300 python3 -u tools/block_balance.py --config ${BLOCK_CONFIG:-c2} --ns ${BLOCK_NS:-8} --skip-full
    unset WCPT_LIBRARY
  done
done
if [ "${PIPES:-0}" = 1 ]; then
  for p in 1 2 3 4; do
    run c3_block_pipes$p 300 python3 -u tools/block_balance.py --config c3 --ns 8 --skip-full --wf-pipes $p
  done
  run c3_block_mk 300 python3 -u tools/block_balance.py --config c3 --ns 8 --skip-full --kernel 0
fi
for r in $(seq 1 ${EVENT_ROUNDS:-0}); do
  for ev in live after; do
    if [ $ev = after ]; then A=--events-after; else A=; fi
    run events_c2_${ev}_$r 300 python3 -u bench.py --config ${EVENT_CONFIG:-c2} --no-cpu-baseline --steps 200 $A
  done
done
for r in $(seq 1 ${REFILL_ROUNDS:-0}); do
  for cfg in ${REFILL_CONFIGS:-c3}; do
    for f in ${REFILLS:-8 12 16}; do
      run refill_${cfg}_${f}_$r 300 python3 -u bench.py --config $cfg --no-cpu-baseline --steps ${REFILL_STEPS:-30} --wf-refill $f
    done
  done
done
for r in $(seq 1 ${FETCH_ROUNDS:-0}); do
  for f in 0 1; do
    for cfg in ${FETCH_CONFIGS:-c3 c4}; do
      run fetch_${cfg}_${f}_$r 300 python3 -u bench.py --config $cfg --no-cpu-baseline --steps ${FETCH_STEPS:-30} --wf-fetch $f ${FETCH_ARGS:-}
    done
    for cfg in ${FETCH_BLOCKS:-}; do
      run fetchblock_${cfg}_${f}_$r 300 python3 -u tools/block_balance.py --config $cfg --ns 8 --skip-full --wf-fetch $f
    done
  done
done
for r in $(seq 1 ${PIPEB_ROUNDS:-0}); do
  for pp in ${PIPEBS:-2 3}; do
    for cfg in ${PIPEB_CONFIGS:-c3 c4}; do
      run pipes_${cfg}_${pp}_$r 300 python3 -u bench.py --config $cfg --no-cpu-baseline --steps ${PIPEB_STEPS:-30} --wf-pipes $pp
    done
  done
done
for r in $(seq 1 ${PERSIST_ROUNDS:-0}); do
  for f in 0 -1; do
    for cfg in ${PERSIST_BLOCKS:-c3}; do
      run persistblock_${cfg}_${f}_$r 300 python3 -u tools/block_balance.py --config $cfg --ns ${PERSIST_NS:-8} --skip-full --wf-persist $f
    done
  done
done
echo SESSION_DONE
