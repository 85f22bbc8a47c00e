"""Host cost of one group step (wcpt_group_render through bench.py's GroupBench path) on a frame so small that the GPU
work is negligible: the rate the host can issue frames at. At 8 ranks a c2 block renders in ~0.07 ms; the host's
per-step cost must stay well below that for the scaling run to stay GPU-bound. Every rank is on device 0 here (COPY or
DIRECT transport), so the device runs all ranks' launches and a sustained run is paced by it: the host's own cost is
taken over short bursts after a drain.

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
    ap.add_argument("--transports", nargs="+", default=["copy", "direct"])
    ap.add_argument("--burst", type=int, default=16,
                    help="steps issued back to back after a drain for the host-issue figure: short enough that the "
                         "device queues never fill (one GPU runs all ranks' work here, so a long run is paced by the "
                         "device and the host's own cost is hidden)")
    a = ap.parse_args()
    s = wscene.generate("cornell")
    W, H = 8, 8
    cases = [(n, x, t, o) for n in a.ranks for x in (a.transports if n > 1 else ["copy"])
             for t in (a.threads if n > 1 else [0]) for o in (a.overlap if x != "direct" and n > 1 else [1])]
    for n, transport, threads, overlap in cases:
        args = bench.parse_args(["--gpus", str(n), "--devices", ",".join(["0"] * n), "--transport", transport,
                                 "--group-threads", str(threads)] + ([] if overlap else ["--no-overlap"]))
        args.kernel = 0
        topo = bench.resolve_topology(args, {})
        drv = bench.GroupBench(args, topo, s, W, max(H, n))
        sd = s.scene_data(W, max(H, n), max_bounce=1, frame=0)
        for _ in range(50):
            drv.render(sd)
        drv.sync()
        issue = 0.0
        done = 0
        while done < a.steps:
            drv.sync()
            t0 = time.perf_counter()
            for _ in range(a.burst):
                drv.render(sd)
            issue += time.perf_counter() - t0
            done += a.burst
        drv.sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            drv.render(sd)
        drv.sync()
        t2 = time.perf_counter()
        print(f"ranks {n} transport {transport} issue_threads {drv.info()['issue_threads']} overlap {overlap}: host "
              f"{1e6 * issue / done:.1f} us/step issue (bursts of {a.burst}), {1e6 * (t2 - t0) / a.steps:.1f} us/step "
              f"sustained with the drain", flush=True)
        drv.close()

if __name__ == "__main__":
    main()
