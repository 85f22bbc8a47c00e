"""Per-launch durations of a kernel in a rocprofv3 --kernel-trace CSV, in dispatch order, with the idle gap before each
launch: shows whether the first frames after an idle host sync run slower than the steady ones.

    python tools/launch_durations.py <dir with *kernel_trace.csv> [--kernel pt_megakernel<false] [--last 40]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="pt_megakernel<false")
    ap.add_argument("--last", type=int, default=40)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if a.kernel in r["Kernel_Name"]]
    prev_end = None
    out = []
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
        out.append((s, (e - s) / 1e3, gap, r.get("Queue_Id", ""), r.get("Grid_Size_X", "")))
        prev_end = e if prev_end is None else max(prev_end, e)
    t0 = out[-a.last][0] if len(out) >= a.last else out[0][0]
    for s, d, g, q, grid in out[-a.last:]:
        print(f"t {(s - t0) / 1e3:10.1f} us  dur {d:8.1f} us  gap {g:8.1f} us  queue {q} grid {grid}")


if __name__ == "__main__":
    main()
