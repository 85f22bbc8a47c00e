"""A/B kernel variants in one process (interleaved, n rounds) on a bench config.

    python tools/ab.py --config c3 --variants "kernel=0" "kernel=2" "kernel=2,deindex=1" [--frames 5 --rounds 3]

Each variant is a comma list of option=value: stack=<0|1>, kernel=<0|2>, order=<0|1|2>, pipes=<1..4>, deindex=<0|1> (mesh re-laid out in
BVH leaf order with identity indices: same triangles, same results, soup-like locality). Prints the median
ms/frame (HIP events on the context stream) and Mray/s.
"""
import argparse
import os

if os.environ.get("AB_TORCH_FIRST"):  # bench.py's load order: libwcpt then binds to torch's HIP runtime
    import torch  # noqa: F401
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import numpy as np  # noqa: E402
import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402  (CONFIGS)


def parse(spec):
    return dict(kv.split("=") for kv in filter(None, spec.split(",")))


def deindexed(s):
    import copy
    d = copy.copy(s)
    d.meshes = []
    for m in s.meshes:
        pos = np.ascontiguousarray(m.positions[m.indices])
        d.meshes.append(wscene.HostBVH(pos, np.arange(m.indices.size, dtype=np.uint32), m.nodes))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--variants", nargs="+", default=["kernel=0"])
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--rows", type=int, default=0, help="render rows [0, rows) only (a row block of an N-way split)")
    ap.add_argument("--check", action="store_true", help="compare the variants' last images bit for bit")
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    scenes = {"0": wcpt.DeviceScene(ctx, s)}
    if any(parse(v).get("deindex") == "1" for v in a.variants):
        scenes["1"] = wcpt.DeviceScene(ctx, deindexed(s))
    ctx.create_screen(W, H)
    if a.rows:
        ctx.set_row_range(0, a.rows)
    sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]
    segs = sum(ctx.render_counters(sd, *scenes["0"].addresses())["segments"] for sd in sds)
    res = {v: [] for v in a.variants}
    imgs = {}
    for r in range(a.rounds + 1):
        for v in a.variants:
            o = parse(v)
            ctx.set_option(wcpt._lib.OPTION_STACK, int(o.get("stack", 1)))
            ctx.set_kernel(int(o.get("kernel", 0)))
            ctx.set_option(wcpt._lib.OPTION_SORT_RAYS, int(o.get("sort", 0)))
            ctx.set_option(wcpt._lib.OPTION_WF_STACK, int(o.get("lds", 10)))
            ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, int(o.get("pairs", -1)))
            ctx.set_option(wcpt._lib.OPTION_PACKED_REFS, int(o.get("refs", 1)))
            ctx.set_option(wcpt._lib.OPTION_WF_REFILL, int(o.get("refill", wcpt._lib.DEFAULT_WF_REFILL)))
            ctx.set_option(wcpt._lib.OPTION_MK_TILE_ORDER, int(o.get("order", 2)))
            ctx.set_option(wcpt._lib.OPTION_WF_PIPES, int(o.get("pipes", wcpt._lib.DEFAULT_WF_PIPES)))
            dev = scenes[o.get("deindex", "0")]
            ctx.profile_begin()
            for sd in sds:
                ctx.render(sd, *dev.addresses())
            ms, n = ctx.profile_end()
            ctx.sync()
            if r > 0:
                res[v].append(ms / n)
            if a.check and r == a.rounds:
                imgs[v] = ctx.readback(a.rows or H).view(np.uint32).copy()
    print(f"{a.config}: {desc}; {segs / a.frames:.0f} segments/frame")
    for v, t in res.items():
        m = statistics.median(t)
        print(f"  {v:30s} {m:8.3f} ms/frame  {segs / a.frames / m / 1e3:9.1f} Mray/s   (runs {', '.join(f'{x:.3f}' for x in t)})")
    if imgs:
        first = next(iter(imgs.values()))
        for v, im in imgs.items():
            print(f"  image of {v}: {'bit-identical to' if np.array_equal(im, first) else 'DIFFERS from'} "
                  f"{a.variants[0]} ({int((im != first).any(axis=-1).sum())} pixels differ)")
    for d in scenes.values():
        d.free()
    ctx.close()


if __name__ == "__main__":
    main()
