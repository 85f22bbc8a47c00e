"""Megakernel traversal-stack status per build mode on a bench config (render / count / diag x stack kind x record
format): reports whether the frame set WCPT_ERROR_STACK_OVERFLOW and, for the render, compares the image with the
wavefront render of the same frame (bit-exact expected).

    python tools/stack_probe.py --config c3 [--rows 1080]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import numpy as np  # noqa: E402
import wcpt  # noqa: E402
from wcpt import _lib  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rows", type=int, default=0)
    a = ap.parse_args()
    name, W, H, spp, bounces, _ = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    dev = wcpt.DeviceScene(ctx, s)
    ctx.create_screen(W, H)
    rows = a.rows or H
    ctx.set_row_range(0, rows)
    sd = s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)
    ctx.set_kernel(wcpt.KERNEL_WAVEFRONT)
    ctx.render(sd, *dev.addresses())
    ctx.sync()
    ref = ctx.readback(rows)
    ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
    for pairs in (1, 0):
        ctx.set_option(_lib.OPTION_PAIR_RECORDS, pairs)
        for stack in (0, 1):
            ctx.set_option(_lib.OPTION_STACK, stack)
            tag = f"pairs={pairs} stack={stack}"
            try:
                ctx.render(sd, *dev.addresses())
                ctx.sync()
                img = ctx.readback(rows)
                print(f"{tag} render: ok, equal to wavefront: {np.array_equal(img, ref)}", flush=True)
            except wcpt.WcptError as e:
                print(f"{tag} render: {e}", flush=True)
            for diag in (False, True):
                try:
                    c = ctx.render_counters(sd, *dev.addresses(), diagnostics=diag)
                    print(f"{tag} {'diag' if diag else 'count'}: ok segments {c['segments']}", flush=True)
                except wcpt.WcptError as e:
                    print(f"{tag} {'diag' if diag else 'count'}: {e}", flush=True)
    ctx.set_option(_lib.OPTION_PAIR_RECORDS, -1)


if __name__ == "__main__":
    main()
