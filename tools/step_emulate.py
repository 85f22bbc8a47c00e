"""Per-step cost of bench.py's N>1 step on ONE GPU: rank 0's row block of an N-way split, rendered and handed to a
world-size-1 RCCL gather (the same stream/event/staging machinery as bench.py), so the host overhead of the N>1
step and the render time of one block are measured without the 8-GPU node. The xGMI transfer itself is not
emulated (a size-1 gather copies locally).

    python tools/step_emulate.py [--config c2] [--steps 200] [--warmup 10]

Prints one line per N in {1, 2, 4, 8}: render-only ms/step, overlapped render+gather ms/step, kernel ms.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
from wcpt.dist import row_block  # noqa: E402
from bench import CONFIGS, DEFAULT_KERNEL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--order", type=int, default=None, help="WCPT_OPTION_MK_TILE_ORDER")
    ap.add_argument("--ns", default="1,2,4,8", help="row-block splits to emulate")
    ap.add_argument("--variant", default="gather", choices=["gather", "events", "copy", "inline", "streamwait", "nowait"],
                    help="gather: bench.py's step (RCCL gather on a communication stream, 3 payload buffers, the host "
                         "waits for a buffer's previous gather); streamwait: 2 buffers, the render stream waits instead; "
                         "nowait: no reuse ordering (unsafe; cost probe); events: only the event hand-off; copy: a "
                         "device copy instead of the collective; inline: the gather on the render stream")
    args = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    name, W, H, spp, bounces, _ = CONFIGS[args.config]
    scene = wscene.generate(name)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = wcpt.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_kernel(DEFAULT_KERNEL[args.config])
    if args.order is not None:
        ctx.set_option(wcpt._lib.OPTION_MK_TILE_ORDER, args.order)
    dev = wcpt.DeviceScene(ctx, scene)
    ctx.create_screen(W, H)
    sd = scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)
    addrs = dev.addresses()
    for n in [int(x) for x in args.ns.split(",")]:
        y0, rows = row_block(H, n, 0)
        ctx.set_row_range(y0, rows)
        shard = torch.zeros((-(-H // n), W, 4), dtype=torch.float32, device="cuda")
        ctx.set_external_image(shard.data_ptr(), shard.numel() * 4)
        comm = torch.cuda.Stream()
        nb = 2 if args.variant in ("streamwait", "nowait") else 3
        payload = [torch.empty((shard.shape[0], W, 3), dtype=torch.float32, device="cuda") for _ in range(nb)]
        gathered = [[torch.empty_like(payload[0])] for _ in range(nb)]
        ready = [torch.cuda.Event() for _ in range(nb)]
        done = [torch.cuda.Event() for _ in range(nb)]
        used = [False] * nb

        def step(f, gather):  # bench.py's N>1 step (overlapped, kernel-written RGB payload)
            sd["renderedFramesCount"] = f
            if not gather:
                ctx.set_gather_output(0, 0)
                ctx.render(sd, *addrs)
                return
            i = f % nb
            if args.variant == "streamwait":
                if used[i] and not done[i].query():
                    stream.wait_event(done[i])
            elif args.variant != "nowait" and used[i]:
                done[i].synchronize()  # the host blocks instead of the render stream (the host runs ahead)
            ctx.set_gather_output(payload[i].data_ptr(), payload[i].numel() * 4, 3)
            ctx.render(sd, *addrs)
            if args.variant == "inline":
                dist.gather(payload[i], gathered[i], dst=0)
                return
            ready[i].record(stream)
            with torch.cuda.stream(comm):
                comm.wait_event(ready[i])
                if args.variant in ("gather", "streamwait", "nowait"):
                    dist.gather(payload[i], gathered[i], dst=0)
                elif args.variant == "copy":
                    gathered[i][0].copy_(payload[i], non_blocking=True)
                done[i].record(comm)
            used[i] = True

        res = {}
        for gather in (False, True):
            for f in range(args.warmup):
                step(f, gather)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                step(args.warmup + k, gather)
            t_host = time.perf_counter() - t0
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            # kernel time in a separate pass, as bench.py at N > 1 (per-launch events are kept out of timed steps)
            ctx.set_gather_output(0, 0)
            ctx.profile_begin()
            for k in range(args.steps):
                sd["renderedFramesCount"] = args.warmup + k
                ctx.render(sd, *addrs)
            kms, launches = ctx.profile_end()
            res[gather] = (el / args.steps * 1e3, t_host / args.steps * 1e3, kms / max(1, launches))
        print(f"N={n} rows={rows}: render-only {res[False][0]:.4f} ms/step (host {res[False][1]:.4f}), "
              f"render+gather {res[True][0]:.4f} ms/step (host {res[True][1]:.4f}), kernel {res[False][2]:.4f} ms",
              flush=True)
        ctx.set_gather_output(0, 0)
        ctx.set_external_image(0, 0)
    dev.free()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
