"""HBM traffic of a frame split by kernel, from the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_sq.sh (one --pmc pass
each, every dispatch of the run recorded with its kernel name).

    python tools/traffic_split.py gpurun_out/<tag>/sq_c3 [--frame-kernel "wf_init<false" --per-frame 2] [--json out]

Per kernel (template arguments folded into the name): dispatches per frame, FETCH_SIZE x 2 + WRITE_SIZE bytes per frame
(the gfx950 correction of MI355X_MICROARCH.md, as tools/pmc_summary.py applies it), and the share of the frame. Each
counter comes from its own run, whose untimed settle phase renders its own number of frames, so each is divided by the
frames of the pass that collected it (dispatches of --frame-kernel / --per-frame).
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frame-kernel", default="wf_init<false")
    ap.add_argument("--per-frame", type=int, default=2)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    vals = defaultdict(lambda: defaultdict(float))   # counter -> kernel -> sum
    disp = defaultdict(lambda: defaultdict(int))     # counter -> kernel -> dispatches
    for f in glob.glob(os.path.join(a.dir, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            c = row["Counter_Name"]
            if c not in ("FETCH_SIZE", "WRITE_SIZE"):
                continue
            name = row.get("Kernel_Name", "")
            full = name
            key = re.sub(r"\(.*", "", name)
            key = re.sub(r"^.*::", "", key) if "<" not in key else key
            vals[c][full] += float(row["Counter_Value"])
            disp[c][full] += 1
    if not vals:
        raise SystemExit(f"no FETCH_SIZE / WRITE_SIZE passes under {a.dir}")
    frames = {c: sum(n for k, n in disp[c].items() if a.frame_kernel in k) / a.per_frame for c in disp}
    kernels = sorted(set(vals["FETCH_SIZE"]) | set(vals["WRITE_SIZE"]))
    rows = []
    for k in kernels:
        fetch = vals["FETCH_SIZE"].get(k, 0.0) / max(frames.get("FETCH_SIZE", 0), 1e-9)
        write = vals["WRITE_SIZE"].get(k, 0.0) / max(frames.get("WRITE_SIZE", 0), 1e-9)
        short = re.sub(r"\(.*", "", k)
        short = re.sub(r"void ", "", short)
        rows.append({"kernel": short, "dispatches_per_frame": round(disp["FETCH_SIZE"].get(k, 0) /
                                                                     max(frames.get("FETCH_SIZE", 0), 1e-9), 2),
                     "fetch_bytes_per_frame": int(2 * fetch * 1024), "write_bytes_per_frame": int(write * 1024),
                     "hbm_bytes_per_frame": int((2 * fetch + write) * 1024)})
    total = sum(r["hbm_bytes_per_frame"] for r in rows)
    for r in sorted(rows, key=lambda r: -r["hbm_bytes_per_frame"]):
        r["share"] = round(r["hbm_bytes_per_frame"] / max(total, 1), 4)
        if r["hbm_bytes_per_frame"] > 0.001 * total:
            print(f"{r['hbm_bytes_per_frame'] / 1e9:8.3f} GB/frame  {100 * r['share']:5.1f} %  "
                  f"(fetch {r['fetch_bytes_per_frame'] / 1e9:.3f}, write {r['write_bytes_per_frame'] / 1e9:.3f}; "
                  f"{r['dispatches_per_frame']:.1f} dispatches/frame)  {r['kernel'][:90]}")
    print(f"{total / 1e9:8.3f} GB/frame total ({frames} frames per pass)")
    if a.json:
        json.dump({"frames_per_pass": frames, "total_hbm_bytes_per_frame": total, "kernels": rows},
                  open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
