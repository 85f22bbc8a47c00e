"""Idle gaps of the whole device in a rocprofv3 --kernel-trace CSV: the union of every queue's kernel intervals, and
each gap longer than --min-us with the kernel that ends it (tools/gpu_r06_kt.sh). Shows whether a frame boundary
leaves the GPU idle (host issue, a copy between frames) or the frame is one continuous stretch of kernels.

    python tools/frame_gaps.py <kernel_trace.csv dir> [--min-us 5]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-us", type=float, default=5.0)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(a.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cur_e = int(rows[0]["End_Timestamp"])
    gaps = []
    for r in rows[1:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > cur_e:
            gaps.append((s - cur_e, r["Kernel_Name"][:50]))
        cur_e = max(cur_e, e)
    big = [g for g in gaps if g[0] > a.min_us * 1e3]
    span = (cur_e - int(rows[0]["Start_Timestamp"])) / 1e6
    print(f"{len(rows)} kernels over {span:.2f} ms; {len(big)} device-idle gaps > {a.min_us} us, "
          f"{sum(g for g, _ in big) / 1e6:.3f} ms in all")
    for g, n in big[:80]:
        print(f"{g / 1e3:9.1f} us before {n}")


if __name__ == "__main__":
    main()
