"""Host cost of one group step (wcpt_group_render through bench.py's GroupBench path) on a frame so small that the GPU
work is negligible: the rate the host can issue frames at. At 8 ranks a c2 block renders in ~0.07 ms; the host's
per-step cost must stay well below that for the scaling run to stay GPU-bound.

    python tools/host_group_probe.py [--ranks 1 2 4] [--steps 2000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), ROOT]
import bench  # noqa: E402
import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402

bench.wcpt = wcpt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    s = wscene.generate("cornell")
    W, H = 8, 8
    for n in a.ranks:
        for overlap in (1, 0):
            args = bench.parse_args(["--gpus", str(n), "--devices", ",".join(["0"] * n), "--transport", "copy"]
                                    + ([] if overlap else ["--no-overlap"]))
            args.kernel = 0
            topo = bench.resolve_topology(args, {})
            drv = bench.GroupBench(args, topo, s, W, max(H, n))
            sd = s.scene_data(W, max(H, n), max_bounce=1, frame=0)
            for _ in range(50):
                drv.render(sd)
            drv.sync()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                drv.render(sd)
            t1 = time.perf_counter()
            drv.sync()
            t2 = time.perf_counter()
            print(f"ranks {n} overlap {overlap}: host {1e6 * (t1 - t0) / a.steps:.1f} us/step issue, "
                  f"{1e6 * (t2 - t0) / a.steps:.1f} us/step with the drain", flush=True)
            drv.close()


if __name__ == "__main__":
    main()
