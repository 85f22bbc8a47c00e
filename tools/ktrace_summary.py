"""Per-launch timeline of wavefront frames from a rocprofv3 --kernel-trace CSV (tools/gpu_r05_session.sh KTRACE=1).

    python tools/ktrace_summary.py gpurun_out/<tag>/kt_c3_block

Frames are cut at each render-mode wf_init (one per pipeline), grouped by wf_init's grid size (a full frame and a row
block differ), and for each group the median frame span and, per pipeline (queue) and position in the chain, the
median duration of each launch (trace, shade) are printed: how much of a block's time each bounce's trace takes, and
whether the two pipelines' chains overlap.
"""
import argparse
import csv
import glob
import os
import re
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--pipes", type=int, default=2, help="wavefront pipelines per frame (one wf_init each)")
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:
        raise SystemExit(f"no kernel_trace.csv under {a.dir}")
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    qkey = "Queue_Id" if "Queue_Id" in rows[0] else ("Stream_Id" if "Stream_Id" in rows[0] else None)
    gkey = next((k for k in ("Grid_Size", "Grid_Size_X", "Grid_X") if k in rows[0]), None)

    def short(name):
        m = re.search(r"(wf_\w+|pt_\w+|build_\w+|scan_\w+|fill_\w+)<([^>]*)>", name)
        return f"{m.group(1)}<{m.group(2)}>" if m else re.sub(r"\(.*", "", name)[:40]

    frames = []
    cur = None
    for r in rows:
        n = short(r["Kernel_Name"])
        if n.startswith("wf_init<false"):
            if cur is None or len(cur["inits"]) >= a.pipes:
                cur = {"k": [], "inits": [], "grid": r.get(gkey, "?") if gkey else "?"}
                frames.append(cur)
            cur["inits"].append(r)
        if cur is None or "<true" in n:
            continue
        cur["k"].append((n, r.get(qkey, "0") if qkey else "0", int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    groups = defaultdict(list)
    for fr in frames:
        if fr["k"]:
            groups[fr["grid"]].append(fr)
    for grid, frs in groups.items():
        spans = [(max(e for *_, e in f["k"]) - min(s for *_, s, _ in f["k"])) / 1e6 for f in frs]
        print(f"wf_init grid {grid}: {len(frs)} frames, median span {statistics.median(spans):.4f} ms")
        per = defaultdict(list)
        for f in frs:
            t0 = min(s for *_, s, _ in f["k"])
            pos = defaultdict(int)
            for n, q, s, e in f["k"]:
                key = (q, n.split("<")[0], pos[(q, n.split("<")[0])])
                pos[(q, n.split("<")[0])] += 1
                per[key].append(((s - t0) / 1e6, (e - s) / 1e6))
        for key in sorted(per):
            v = per[key]
            print(f"  queue {key[0]} {key[1]:10s} #{key[2]}: start {statistics.median(x for x, _ in v):.4f} ms, "
                  f"duration {statistics.median(d for _, d in v):.4f} ms")


if __name__ == "__main__":
    main()
