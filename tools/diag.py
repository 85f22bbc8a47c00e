"""SIMD-efficiency and trace-loop phase diagnostics of the instrumented (DIAG) kernels.

    python tools/diag.py --config c3 [--kernel 0|2] [--size WxH] [--stack 0|1]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--kernel", type=int, default=0)
    ap.add_argument("--stack", type=int, default=0)
    ap.add_argument("--size", default=None, help="WxH override")
    a = ap.parse_args()
    name, W, H, spp, bounces, desc = bench.CONFIGS[a.config]
    if a.size:
        W, H = map(int, a.size.split("x"))
    s = wscene.generate(name)
    ctx = wcpt.Context(0)
    ctx.set_kernel(a.kernel)
    ctx.set_option(wcpt._lib.OPTION_STACK, a.stack)
    dev = wcpt.DeviceScene(ctx, s)
    ctx.create_screen(W, H)
    c = ctx.render_counters(s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0), *dev.addresses(),
                            diagnostics=True)
    out = dict(c)
    for ph in ("interior", "triangle", "segment"):
        w, l = c[f"wave_{ph}_steps"], c[f"lane_{ph}_steps"]
        out[f"simd_eff_{ph}"] = round(l / (64.0 * w), 4) if w else None
    out["per_segment"] = {k: round(c[k] / c["segments"], 3) for k in ("interior_visits", "triangle_tests",
                                                                       "node_pops", "sphere_tests")}
    if a.kernel == 2:
        t = ctx.read_diagnostics()
        tot = sum(t[:5]) or 1
        out["trace_phase_share"] = {k: round(v / tot, 4) for k, v in
                                    zip(("fetch", "leaf", "interior", "pop", "epilogue"), t[:5])}
        out["trace_waves"], out["trace_iterations"] = t[5], t[6]
        out["trace_tail_share"] = round(t[7] / tot, 4)   # wave-time after the wave found the queue empty
        if t[6]:
            out["trace_cycles_per_iteration"] = round(tot / t[6], 1)
            out["trace_iterations_per_wave"] = round(t[6] / max(1, t[5]), 1)
    print(a.config, "kernel", a.kernel, json.dumps(out, indent=1))
    dev.free()
    ctx.close()


if __name__ == "__main__":
    main()
