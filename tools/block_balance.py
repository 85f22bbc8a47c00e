"""Load balance of the N-way row-block split on ONE GPU: every rank's block of a bench config rendered in turn
(same kernel, options and progressive frames as bench.py), timed with HIP events on the context stream, on the
system HIP runtime that bench.py binds (torch is not imported).

    python tools/block_balance.py [--config c2] [--ns 2,4,8] [--frames 20] [--rounds 3] [--stripes 0,8]

--stripes: the split's stripe sizes to time (0 = contiguous row blocks; S = interleaved stripes of S rows,
wcpt_set_row_stripes, rank r taking the stripes r, r + N, ...).

Per N prints each block's median ms/frame, the max (what the N-GPU step waits for), the mean, and
full-frame / N (perfect split). max / (full / N) is the load-balance + tail loss of the split. Each block's frames are
timed as one region (WCPT_OPTION_PROFILE_REGION, as bench.py times its steps), so the frame overlap applies where its
auto rule does (full frames, 2- and 4-way blocks; --per-render-events restores the round-5 timing, one event pair per
render, under which the overlap is off).
"""
import argparse
import os

import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]

import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
from wcpt.dist import row_stripes  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--ns", default="2,4,8")
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--first", action="store_true", help="rank 0's block only (a size sweep)")
    ap.add_argument("--kernel", type=int, default=-1, help="WCPT_KERNEL_* (default: bench.py's for the config)")
    ap.add_argument("--wf-pipes", type=int, default=0, help="WCPT_OPTION_WF_PIPES (0: the library default)")
    ap.add_argument("--wf-fetch", type=int, default=-1, help="WCPT_OPTION_WF_FETCH (-1: auto)")
    ap.add_argument("--wf-persist", type=int, default=-1, help="WCPT_OPTION_WF_PERSIST (-1: auto)")
    ap.add_argument("--wf-refill", type=int, default=0, help="WCPT_OPTION_WF_REFILL (0: the library default)")
    ap.add_argument("--skip-full", action="store_true", help="do not time the full frame (full/N columns then 0)")
    ap.add_argument("--stripes", default="0", help="stripe sizes: 0 = contiguous row blocks, S = interleaved stripes")
    ap.add_argument("--per-render-events", action="store_true", help="one event pair per render (no frame overlap)")
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(bench.DEFAULT_KERNEL[a.config] if a.kernel < 0 else a.kernel)
    if a.wf_pipes:
        ctx.set_option(wcpt._lib.OPTION_WF_PIPES, a.wf_pipes)
    ctx.set_option(wcpt._lib.OPTION_WF_FETCH, a.wf_fetch)
    ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, a.wf_persist)
    if a.wf_refill:
        ctx.set_option(wcpt._lib.OPTION_WF_REFILL, a.wf_refill)
    ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 0 if a.per_render_events else 1)
    dev = wcpt.DeviceScene(ctx, s)
    ctx.create_screen(W, H)
    sds = [s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f) for f in range(a.frames)]

    def timed(y0, rows, stripe=0, period=0):
        ctx.set_row_stripes(y0, rows, stripe, period)
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
        return statistics.median(out)

    full = 0.0 if a.skip_full else timed(0, H)
    stripes = [int(x) for x in a.stripes.split(",")]
    print(f"{a.config}: {desc}; kernel {bench.DEFAULT_KERNEL[a.config] if a.kernel < 0 else a.kernel}; "
          f"wf pipes {a.wf_pipes or 'default'}; full frame {full:.4f} ms", flush=True)
    for n in [int(x) for x in a.ns.split(",")]:
        for st in stripes:
            t = [timed(*row_stripes(H, n, r, st), st, st * n) for r in range(1 if a.first else n)]
            mx, mean = max(t), sum(t) / len(t)
            ratio = f"{mx / (full / n):.2f}" if full else "-"
            kind = f"stripes {st}" if st else "blocks"
            print(f"N={n} {kind}: {' '.join(f'{x:.4f}' for x in t)} | max {mx:.4f} mean {mean:.4f} full/N "
                  f"{full / n:.4f} | max/(full/N) {ratio} max/mean {mx / mean:.2f} | speed-up {full / mx if full else 0:.2f}x",
                  flush=True)
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
