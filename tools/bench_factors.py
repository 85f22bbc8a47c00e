"""Which part of bench.py's N=1 setup changes the c2 render time: the torch stream, the torch-allocated external
image, or neither (one factor at a time, same process, interleaved rounds)."""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]
import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402

name, W, H, spp, bounces, _ = bench.CONFIGS["c2"]
s = wscene.generate(name)
ctx = wcpt.Context(0)
dev = wcpt.DeviceScene(ctx, s)
ctx.create_screen(W, H)
tstream = torch.cuda.Stream()
shard = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(3, 23)]
res = {}
for r in range(4):
    for ts in (0, 1):
        for ext in (0, 1):
            ctx.set_stream(tstream.cuda_stream if ts else None)
            ctx.set_external_image(shard.data_ptr() if ext else 0, shard.numel() * 4)
            ctx.profile_begin()
            for sd in sds:
                ctx.render(sd, *dev.addresses())
            ms, n = ctx.profile_end()
            ctx.sync()
            if r:
                res.setdefault((ts, ext), []).append(ms / n)
for k, v in res.items():
    print(f"torch_stream={k[0]} external_image={k[1]}: {statistics.median(v):.4f} ms ({', '.join(f'{x:.4f}' for x in v)})")
