"""Host cost of each call in bench.py's N>1 step (overlapped gather), on ONE GPU with a world-size-1 RCCL group.

    python tools/host_step_probe.py [--config c2] [--rows 135] [--steps 300]

Prints the mean host microseconds per step of every call (event waits, the ctypes render, event records, the
stream switch, the collective) and the step period, so the N>1 step's host budget can be compared with the
render time of one row block.
"""
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
from bench import CONFIGS, DEFAULT_KERNEL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rows", type=int, default=135)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--profile", action="store_true", help="per-launch profiling events on (as bench.py's timed region)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", "1")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    name, W, H, spp, bounces, _ = CONFIGS[a.config]
    scene = wscene.generate(name)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    ctx = wcpt.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_kernel(DEFAULT_KERNEL[a.config])
    dev = wcpt.DeviceScene(ctx, scene)
    ctx.create_screen(W, H)
    ctx.set_row_range(0, a.rows)
    shard = torch.zeros((a.rows, W, 4), dtype=torch.float32, device="cuda")
    ctx.set_external_image(shard.data_ptr(), shard.numel() * 4)
    sd = scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)
    addrs = dev.addresses()
    comm = torch.cuda.Stream()
    nb = 3
    payload = [torch.empty((a.rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nb)]
    gathered = [[torch.empty_like(payload[0])] for _ in range(nb)]
    ready = [torch.cuda.Event() for _ in range(nb)]
    done = [torch.cuda.Event() for _ in range(nb)]
    used = [False] * nb
    names = ["done.sync", "set_output", "render", "ready.record", "stream+wait", "gather", "done.record"]
    acc = [0.0] * len(names)
    pc = time.perf_counter_ns

    def step(f, timed):
        sd["renderedFramesCount"] = f
        i = f % nb
        t = [pc()]
        if used[i]:
            done[i].synchronize()
        t.append(pc())
        ctx.set_gather_output(payload[i].data_ptr(), payload[i].numel() * 4, 3)
        t.append(pc())
        ctx.render(sd, *addrs)
        t.append(pc())
        ready[i].record(stream)
        t.append(pc())
        with torch.cuda.stream(comm):
            comm.wait_event(ready[i])
            t.append(pc())
            dist.gather(payload[i], gathered[i], dst=0)
            t.append(pc())
            done[i].record(comm)
        t.append(pc())
        used[i] = True
        if timed:
            for k in range(len(names)):
                acc[k] += t[k + 1] - t[k]

    for f in range(20):
        step(f, False)
    torch.cuda.synchronize()
    if a.profile:
        ctx.profile_begin()
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(20 + k, True)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / a.steps * 1e6
    if a.profile:
        ctx.profile_end()
    print(f"{a.config} rows={a.rows} profile={int(a.profile)}: step period {el:.1f} us; host us/step: " +
          ", ".join(f"{n} {v / a.steps / 1e3:.1f}" for n, v in zip(names, acc)), flush=True)
    ctx.set_gather_output(0, 0)
    ctx.set_external_image(0, 0)
    dev.free()
    ctx.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
