set -u
# GPU session: pytest -m gpu, the emulated N-way step (tools/step_emulate.py), gloo rehearsals of the N>1 bench
# path with --verify (bit-exact gathered frame), the default bench, and the step variants at N=8.

export TMPDIR=/tmp
OUT=gpurun_out/s4; mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 200 python3 -u tools/step_emulate.py --steps 100 2>&1 | grep "^N=" || exit 1
for be in gloo gloo-host; do
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --config c2 --steps 4 --warmup 2 --dist-backend $be --verify > $OUT/n2_$be.log 2>&1 || { tail -20 $OUT/n2_$be.log; exit 1; }
grep -o '"verified": [a-z]*' $OUT/n2_$be.log
done
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 3 --config c1 --steps 4 --warmup 2 --dist-backend gloo --gather rgba --no-overlap --verify > $OUT/n3.log 2>&1 || { tail -20 $OUT/n3.log; exit 1; }
grep -o '"verified": [a-z]*' $OUT/n3.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $OUT/bench.log


for v in gather streamwait inline; do
timeout -k 10 200 python3 -u tools/step_emulate.py --ns 8 --steps 200 --variant $v 2>&1 | grep "^N=" | sed "s/^/$v: /" || exit 1
done

echo ALL_DONE
