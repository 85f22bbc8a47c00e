"""Frame overlap (WCPT_OPTION_FRAME_OVERLAP) A/B on one GPU: a bench config rendered through a plain context and
through a one-rank group (its communication stream on or off: GROUP_OPTION_OVERLAP), with the frame overlap off and
on, interleaved rounds; ms/frame from the host clock between two synchronisations.

    python tools/overlap_ab.py [--config c2] [--frames 200] [--rounds 3] [--modes ctx,group,group-inline]
        [--values 0,1] [--block N,r]    (--block: one rank's row block of an N-way split, ctx mode)
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

T = wcpt._lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="ctx,group,group-inline")
    ap.add_argument("--values", default="0,1")
    ap.add_argument("--block", default=None, help="N,r: render only rank r's row block of an N-way split (ctx mode)")
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]
    print(f"{a.config}: {desc}", flush=True)
    res = {}
    for r in range(a.rounds):
        for mode in a.modes.split(","):
            for ov in [int(v) for v in a.values.split(",")]:
                g = None
                if mode == "ctx":
                    ctx = wcpt.Context(0)
                else:
                    g = wcpt.Group([0], root=0)
                    g.set_option(T.GROUP_OPTION_OVERLAP, 0 if mode == "group-inline" else 1)
                    ctx = g.context(0)
                ctx.set_kernel(bench.DEFAULT_KERNEL[a.config])
                ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
                dev = wcpt.DeviceScene(ctx, s)
                if g:
                    g.create_screen(W, H)
                    addr = [[x] for x in dev.addresses()]
                    render, sync = (lambda sd: g.render(sd, *addr)), g.sync
                else:
                    ctx.create_screen(W, H)
                    if a.block:
                        from wcpt.dist import row_block
                        n, rk = (int(x) for x in a.block.split(","))
                        ctx.set_row_range(*row_block(H, n, rk))
                    render, sync = (lambda sd: ctx.render(sd, *dev.addresses())), ctx.sync
                for sd in sds[:20]:
                    render(sd)
                sync()
                t0 = time.perf_counter()
                for sd in sds:
                    render(sd)
                sync()
                ms = (time.perf_counter() - t0) * 1e3 / len(sds)
                res.setdefault((mode, ov), []).append(ms)
                print(f"round {r} {mode:12s} overlap {ov}: {ms:.4f} ms/frame", flush=True)
                dev.free()
                if g:
                    g.close()
                else:
                    ctx.close()
    for (mode, ov), v in sorted(res.items()):
        print(f"{mode:12s} overlap {ov}: median {statistics.median(v):.4f} ms/frame ({' '.join(f'{x:.4f}' for x in v)})")


if __name__ == "__main__":
    main()
