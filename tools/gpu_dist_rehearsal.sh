#!/bin/bash
# Rehearse bench.py's N>1 path on a one-GPU box: 2 and 3 ranks share cuda:0 over the gloo backend (RCCL refuses
# duplicate devices), with device tensors (the stream/event path of the RCCL run) and host-staged, overlapped and
# not; --verify checks the gathered row blocks against a full-frame render bit-for-bit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-dist}; mkdir -p "$OUT"
run() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -n 3 | cut -c1-600; return $rc; }
run n1_c1 300 python3 bench.py --config c1 --steps 4 --warmup 2 --no-cpu-baseline --verify || exit 1
for n in 2 3; do
  for be in gloo gloo-host; do
    run n${n}_c1_$be 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29500 + n)) bench.py --gpus $n --config c1 --steps 4 --warmup 2 --dist-backend $be --verify || exit 1
    run n${n}_c1_${be}_noov 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
        --master-port $((29510 + n)) bench.py --gpus $n --config c1 --steps 4 --warmup 2 --dist-backend $be --verify --no-overlap || exit 1
  done
done
run n2_c1_rgba 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29520 bench.py --gpus 2 --config c1 --steps 4 --warmup 2 --dist-backend gloo --gather rgba --verify || exit 1
run n2_c1_display 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29521 bench.py --gpus 2 --config c1 --steps 4 --warmup 2 --dist-backend gloo --gather display --verify || exit 1
run n3_c2_display_host 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 \
    --master-port 29522 bench.py --gpus 3 --config c2 --steps 4 --warmup 2 --dist-backend gloo-host --gather display --verify || exit 1
run n2_c2 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29510 bench.py --gpus 2 --config c2 --steps 5 --warmup 2 --dist-backend gloo --verify || exit 1
run n2_c3 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29530 bench.py --gpus 2 --config c3 --steps 3 --warmup 1 --dist-backend gloo --verify || exit 1
run n2_c4 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29540 bench.py --gpus 2 --config c4 --steps 2 --warmup 1 --dist-backend gloo --verify || exit 1
echo ALL_DONE
