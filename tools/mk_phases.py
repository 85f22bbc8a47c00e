"""Megakernel phase shares from the tools-only timer build (pt_device.h phase_mark, -DWCPT_MK_TIMERS=1).

    bash tools/ab_build.sh timers "-DWCPT_MK_TIMERS=1"
    WCPT_LIBRARY=wc-path-tracer_amd/variants/timers.so python tools/mk_phases.py --config c2 [--frames 5]

Prints, per phase, the share of the waves' s_memtime ticks (summed over waves and frames).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402

PHASES = ("primary", "spheres", "bvh_steps", "leaf_tests", "hit_resolve", "shade", "store")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=5)
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
    dev = wcpt.DeviceScene(ctx, s)
    ctx.create_screen(W, H)
    tot = [0] * len(PHASES)
    for f in range(a.frames + 1):
        ctx.render(s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f), *dev.addresses())
        ctx.sync()
        t = ctx.read_diagnostics()
        if f > 0:  # frame 0 warms up
            tot = [x + y for x, y in zip(tot, t[:len(PHASES)])]
    all_ = sum(tot) or 1
    print(a.config, json.dumps({p: round(v / all_, 4) for p, v in zip(PHASES, tot)}, indent=1))
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
