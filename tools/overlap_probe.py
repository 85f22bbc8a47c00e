"""Does a long-running collective-like kernel on the communication stream overlap the N>1 row-block render?

    python tools/overlap_probe.py [--rows 135] [--us 60] [--blocks 16]

bench.py's N>1 step with the RCCL gather replaced by a stand-in kernel (tools/spin_kernel.hip: `--blocks` workgroups
of 256 threads that stay resident for `--us` microseconds, like RCCL's transfer kernel while 7 x 3.1 MB arrive over
xGMI). Prints the step period with no stand-in, with it, and with the render stream restricted by a CU mask that
leaves `--reserve` CUs to the communication stream.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
from bench import CONFIGS, DEFAULT_KERNEL  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rows", type=int, default=135)
    ap.add_argument("--us", type=float, default=60.0)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--reserve", default="8,16", help="CUs kept out of the render stream's mask (comma list)")
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    so = os.path.join(ROOT, "tools", "libspin.so")
    if not os.path.exists(so):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", "-o", so,
                        os.path.join(ROOT, "tools", "spin_kernel.hip")], check=True)
    torch.cuda.set_device(0)
    spin = C.CDLL(so)
    spin.spin_launch.argtypes = [C.c_void_p, C.c_int, C.c_longlong, C.c_void_p]
    spin.masked_stream_create.argtypes = [C.POINTER(C.c_void_p), C.c_uint32, C.POINTER(C.c_uint32)]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    name, W, H, spp, bounces, _ = CONFIGS[a.config]
    scene = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(DEFAULT_KERNEL[a.config])
    dev = wcpt.DeviceScene(ctx, scene)
    ctx.create_screen(W, H)
    ctx.set_row_range(0, a.rows)
    shard = torch.zeros((a.rows, W, 4), dtype=torch.float32, device="cuda")
    ctx.set_external_image(shard.data_ptr(), shard.numel() * 4)
    sd = scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)
    addrs = dev.addresses()
    sink = torch.zeros(256, device="cuda")
    ticks = int(a.us * 100)  # s_memrealtime: 100 MHz

    def run(render_stream, with_spin):
        torch.cuda.set_stream(render_stream)
        ctx.set_stream(render_stream.cuda_stream)
        comm = torch.cuda.Stream()
        nb = 3
        payload = [torch.empty((a.rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nb)]
        ready = [torch.cuda.Event() for _ in range(nb)]
        done = [torch.cuda.Event() for _ in range(nb)]
        used = [False] * nb

        def step(f):
            sd["renderedFramesCount"] = f
            i = f % nb
            if used[i]:
                done[i].synchronize()
            ctx.set_gather_output(payload[i].data_ptr(), payload[i].numel() * 4, 3)
            ctx.render(sd, *addrs)
            ready[i].record(render_stream)
            comm.wait_event(ready[i])
            if with_spin:
                spin.spin_launch(C.c_void_p(comm.cuda_stream), a.blocks, ticks, C.c_void_p(sink.data_ptr()))
            done[i].record(comm)
            used[i] = True

        for f in range(20):
            step(f)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(a.steps):
            step(20 + k)
        torch.cuda.synchronize()
        ctx.set_gather_output(0, 0)
        return (time.perf_counter() - t0) / a.steps * 1e6

    plain = torch.cuda.Stream()
    res = {"render only": run(plain, False), f"+ stand-in ({a.blocks} x {a.us:.0f} us)": run(plain, True)}
    for r in [int(x) for x in a.reserve.split(",") if x]:
        words = (cus + 31) // 32
        bits = [1] * cus
        # keep CUs out of the mask spread over the device (every cus/r-th CU)
        for j in range(r):
            bits[(j * cus) // r] = 0
        mask = (C.c_uint32 * words)(*[sum(bits[w * 32 + b] << b for b in range(32) if w * 32 + b < cus) for w in range(words)])
        h = C.c_void_p()
        rc = spin.masked_stream_create(C.byref(h), words, mask)
        if rc != 0:
            print(f"hipExtStreamCreateWithCUMask failed: {rc}")
            continue
        ms = torch.cuda.ExternalStream(h.value)
        res[f"render masked -{r} CUs"] = run(ms, False)
        res[f"render masked -{r} CUs + stand-in"] = run(ms, True)
    print(f"{a.config} rows={a.rows} ({cus} CUs): " + "; ".join(f"{k} {v:.1f} us/step" for k, v in res.items()), flush=True)
    ctx.set_external_image(0, 0)
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
