"""Per-frame fixed cost of a bench config: the frame rendered at several heights (same width, scene, kernel and
options as bench.py), timed with HIP events on the context stream, and the line t(H) = fixed + per_row * H fitted
through the medians. `fixed` is what one render costs whatever its size -- the launch gap and the tail of the last
round of waves (megakernel), or the per-bounce launch tails and the pipelines' join (wavefront): the part of a frame
that overlapping consecutive frames could recover.

    python tools/launch_tail.py [--config c2] [--heights 540,1080,2160,4320] [--frames 20] [--rounds 3]
"""
import argparse
import os
import statistics
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--heights", default="540,1080,2160,4320")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--wf-pipes", type=int, default=0)
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(bench.DEFAULT_KERNEL[a.config])
    if a.wf_pipes:
        ctx.set_option(wcpt._lib.OPTION_WF_PIPES, a.wf_pipes)
    dev = wcpt.DeviceScene(ctx, s)
    hs = [int(x) for x in a.heights.split(",")]
    res = []
    for h in hs:
        ctx.create_screen(W, h)
        sds = [s.scene_data(W, h, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]
        for sd in sds[:3]:
            ctx.render(sd, *dev.addresses())
        out = []
        for _ in range(a.rounds):
            ctx.profile_begin()
            for sd in sds:
                ctx.render(sd, *dev.addresses())
            ms, n = ctx.profile_end()
            ctx.sync()
            out.append(ms / n)
        t = statistics.median(out)
        res.append(t)
        print(f"{a.config} {W}x{h}: {t:.4f} ms/frame, {W * h * spp / t / 1e3:.1f} Mray/s (primary)", flush=True)
    slope, fixed = np.polyfit(np.asarray(hs, float), np.asarray(res), 1)
    for h, t in zip(hs, res):
        print(f"  H={h}: fixed {fixed:.4f} ms = {fixed / t * 100:.1f} % of the frame; fit residual "
              f"{(t - fixed - slope * h) * 1e3:+.1f} us")
    print(f"{a.config}: {desc}; fit t = {fixed:.4f} ms + {slope * 1e3:.4f} us/row", flush=True)
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
