"""Host cost of one group step (wcpt_group_render through bench.py's GroupBench path) on a frame so small that the GPU
work is negligible: the rate the host can issue frames at. At 8 ranks a c2 block renders in ~0.07 ms; the host's
per-step cost must stay well below that for the scaling run to stay GPU-bound.

    python tools/host_group_probe.py [--ranks 1 2 4 8] [--steps 2000]

With WCPT_LIBRARY pointing at a build made with EXTRA=-DWCPT_GROUP_TIMERS=1 the group prints, when destroyed, the
host time of each plan step kind per frame (stderr, "group_timers ...").
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
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--threads", type=int, nargs="+", default=[0, 1],
                    help="WCPT_GROUP_OPTION_THREADS values to measure (0: the caller's thread issues every rank)")
    ap.add_argument("--overlap", type=int, nargs="+", default=[1, 0])
    a = ap.parse_args()
    s = wscene.generate("cornell")
    W, H = 8, 8
    cases = [(n, t, o) for n in a.ranks for t in (a.threads if n > 1 else [0]) for o in a.overlap]
    for n, threads, overlap in cases:
        args = bench.parse_args(["--gpus", str(n), "--devices", ",".join(["0"] * n), "--transport", "copy",
                                 "--group-threads", str(threads)] + ([] if overlap else ["--no-overlap"]))
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
        print(f"ranks {n} issue_threads {drv.info()['issue_threads']} overlap {overlap}: host "
              f"{1e6 * (t1 - t0) / a.steps:.1f} us/step issue, {1e6 * (t2 - t0) / a.steps:.1f} us/step with the drain",
              flush=True)
        drv.close()

if __name__ == "__main__":
    main()
