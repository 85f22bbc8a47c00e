"""Per-tile timing of the megakernel (tools-only build with -DWCPT_MK_TILE_TRACE=1) and A/B of a cost-ordered tile
list against the built-in order.

    bash tools/ab_build.sh tiletrace "-DWCPT_MK_TILE_TRACE=1"
    WCPT_LIBRARY=wc-path-tracer_amd/variants/tiletrace.so python tools/tile_trace.py --config c2 [--rows 135]

The build writes, per block, its tile, s_memrealtime start/end (100 MHz) and HW_ID/XCC_ID into the gather payload
buffer, and renders tile order[b] for block b when that buffer starts with an explicit order. Prints the launch's
busy profile (share of the span during which fewer than half the waves are still running) and the median frame time
of: the built-in order, longest-first (LPT) by last frames' tile times, and for one-round launches a serpentine order
that gives each SIMD (blocks b, b + S, b + 2S, ... share one, tools/dispatch_probe.hip) one tile of each cost band.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import numpy as np  # noqa: E402
import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    rows = a.rows or H
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
    dev = wcpt.DeviceScene(ctx, s)
    ctx.create_screen(W, H)
    if a.rows:
        ctx.set_row_range(0, rows)
    tilesX, tilesY = (W + 7) // 8, (rows + 7) // 8
    T = tilesX * tilesY
    head = (T + 3) & ~3
    nbytes = max(W * rows * 16, head * 4 + T * 32)
    buf = ctx.buffer_alloc(nbytes)
    addr = ctx.buffer_address(buf)
    ctx.set_gather_output(addr, nbytes, 4)
    sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]

    def set_order(order):
        o = np.full(head, 0xFFFFFFFF, np.uint32)
        if order is not None:
            o[:T] = order
        ctx.buffer_upload(buf, o)

    def trace_frame(sd):
        ctx.render(sd, *dev.addresses())
        ctx.sync()
        raw = np.frombuffer(ctx.buffer_download(buf, T * 32, head * 4), np.uint32).reshape(T, 8)
        t0 = raw[:, 1].astype(np.uint64) | (raw[:, 2].astype(np.uint64) << 32)
        t1 = raw[:, 3].astype(np.uint64) | (raw[:, 4].astype(np.uint64) << 32)
        return raw[:, 0].copy(), t0, t1, raw[:, 5].copy(), raw[:, 6].copy()

    # tile costs (realtime ticks) averaged over frames, built-in order
    set_order(None)
    cost = np.zeros(T)
    for sd in sds[:8]:
        tile, t0, t1, hw, xcc = trace_frame(sd)
        cost[tile] += (t1 - t0).astype(np.float64)
    cost /= 8
    span = float(t1.max() - t0.min())
    starts, ends = (t0 - t0.min()).astype(np.float64), (t1 - t0.min()).astype(np.float64)
    grid = np.linspace(0, span, 400)
    active = np.array([np.sum((starts <= g) & (ends > g)) for g in grid])
    peak = active.max()
    half_tail = float(np.mean(active < 0.5 * peak))
    out = {"config": a.config, "rows": rows, "tiles": int(T), "span_us": round(span / 100.0, 2),
           "tile_cost_us": {"mean": round(cost.mean() / 100, 2), "cv": round(cost.std() / cost.mean(), 3),
                            "max": round(cost.max() / 100, 2)},
           "share_of_span_below_half_the_peak_waves": round(half_tail, 3)}

    lpt = np.argsort(-cost, kind="stable").astype(np.uint32)
    S = a.simds
    serp = np.empty(T, np.uint32)
    for b in range(T):
        k, i = divmod(b, S)
        r = k * S + (i if k % 2 == 0 else min(S, T - k * S) - 1 - i)
        serp[b] = lpt[r]
    variants = {"builtin": None, "lpt": lpt, "serpentine": serp}
    res = {k: [] for k in variants}
    for r in range(a.rounds + 1):
        for k, order in variants.items():
            set_order(order)
            ctx.profile_begin()
            for sd in sds:
                ctx.render(sd, *dev.addresses())
            ms, n = ctx.profile_end()
            ctx.sync()
            if r:
                res[k].append(ms / n)
    out["ms_per_frame"] = {k: round(statistics.median(v), 4) for k, v in res.items()}
    print(json.dumps(out))
    ctx.set_gather_output(0, 0)
    ctx.buffer_free(buf)
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
