"""How much of a frame a following frame could overlap: K independent contexts (each its own stream, screen and
scene copy) render the same bench config round-robin, and the per-frame time of the whole batch (host clock between
two synchronisations) is compared with one context. With one context consecutive renders serialise on its stream
(launch gap + the last round of waves / the pipelines' join); with K their launches overlap, so the difference is
the per-frame cost that letting frame k + 1 start under frame k's tail could recover.

    python tools/stream_overlap.py [--config c2] [--contexts 1,2,3] [--frames 60] [--rounds 5]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--contexts", default="1,2,3")
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ks = [int(x) for x in a.contexts.split(",")]
    ctxs, devs = [], []
    for _ in range(max(ks)):
        c = wcpt.Context(0)
        c.set_kernel(bench.DEFAULT_KERNEL[a.config])
        devs.append(wcpt.DeviceScene(c, s))
        c.create_screen(W, H)
        ctxs.append(c)
    sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]
    print(f"{a.config}: {desc}", flush=True)
    base = None
    for k in ks:
        for j in range(k):
            for sd in sds[:3]:
                ctxs[j].render(sd, *devs[j].addresses())
        for j in range(k):
            ctxs[j].sync()
        out = []
        for _ in range(a.rounds):
            t0 = time.perf_counter()
            for f, sd in enumerate(sds):
                j = f % k
                ctxs[j].render(sd, *devs[j].addresses())
            for j in range(k):
                ctxs[j].sync()
            out.append((time.perf_counter() - t0) * 1e3 / len(sds))
        t = statistics.median(out)
        base = base or t
        print(f"contexts {k}: {t:.4f} ms/frame ({' '.join(f'{x:.4f}' for x in out)}), {base / t:.3f}x of one",
              flush=True)
    for c, d in zip(ctxs, devs):
        d.free()
        c.close()


if __name__ == "__main__":
    main()
