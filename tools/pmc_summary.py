"""Aggregate rocprofv3 --pmc CSVs (tools/pmc.sh) per kernel: mean counter value per dispatch.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc [--kernel pt_megakernel<false] [--json out.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half the bytes of wide
coalesced reads on gfx950, so traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes; our reads are 16-byte
per-lane gathers, an access width the guide leaves uncalibrated (stated wherever the number is used).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

from sq_summary import grid_size


def load(d, grids=None):
    per = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            per[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
            if grids is not None:
                grids[name][row["Counter_Name"]] += grid_size(row)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="pt_megakernel<false")
    ap.add_argument("--json", default=None)
    ap.add_argument("--build-id", default=None, help="wcpt_build_id() of the library the passes measured")
    ap.add_argument("--config", default=None)
    ap.add_argument("--camera", default="still", help="bench.py --camera of the passes (still | orbit)")
    ap.add_argument("--kernel-id", type=int, default=0)
    ap.add_argument("--per-frame", type=int, default=2,
                    help="dispatches of --frame-kernel per frame (wavefront: one wf_init per pipeline; "
                         "WCPT_OPTION_WF_PIPES defaults to 2)")
    ap.add_argument("--frame-kernel", default=None,
                    help="whole-frame mode (wavefront: several kernels per frame): --kernel is a comma list of "
                         "kernel filters whose counters are SUMMED over all their dispatches and divided by the "
                         "dispatch count of this kernel (one per frame, e.g. 'wf_init<false')")
    ap.add_argument("--frame-grid", type=int, default=0,
                    help="work-items of --kernel per frame: per-FRAME counters, the dispatches' sums scaled by frame "
                         "grid / dispatched grid (a megakernel frame under the frame overlap is two launches)")
    a = ap.parse_args()
    grids = defaultdict(lambda: defaultdict(float)) if a.frame_grid else None
    per = load(a.dir, grids)
    out = {}
    if a.frame_kernel:
        # frames per counter: each counter comes from its own --pmc pass (a separate run, whose untimed settle phase
        # renders its own number of frames), so every counter is divided by the frames of the pass that collected it
        frames = defaultdict(int)
        for n, c in per.items():
            if a.frame_kernel in n:
                for ctr, vals in c.items():
                    frames[ctr] += len(vals)
        if not frames:
            raise SystemExit(f"no dispatches of {a.frame_kernel} in {a.dir}")
        filters = a.kernel.split(",")
        for name, ctrs in per.items():
            if not any(f in name for f in filters):
                continue
            for c, vals in ctrs.items():
                out[c] = out.get(c, 0.0) + sum(vals) / (frames[c] / a.per_frame)
        if not out:
            raise SystemExit(f"no dispatches of {a.kernel} in {a.dir}")
    elif a.frame_grid:
        tot, gr = defaultdict(float), defaultdict(float)
        for name, ctrs in per.items():
            if a.kernel not in name:
                continue
            for c, vals in ctrs.items():
                tot[c] += sum(vals)
                gr[c] += grids[name][c]
        out = {c: tot[c] * a.frame_grid / gr[c] for c in tot}
    else:
        for name, ctrs in per.items():
            if a.kernel not in name:
                continue
            for c, vals in ctrs.items():
                out[c] = sum(vals) / len(vals)
    if not out:
        raise SystemExit(f"no dispatches of {a.kernel} in {a.dir}")
    d = dict(out)
    if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
        key = "hbm_bytes_per_frame" if (a.frame_kernel or a.frame_grid) else "hbm_bytes_per_launch"
        d[key] = int((2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024)
    if "SQ_ACTIVE_INST_VALU" in out and "SQ_THREAD_CYCLES_VALU" in out and out["SQ_ACTIVE_INST_VALU"]:
        d["valu_lane_utilization"] = out["SQ_THREAD_CYCLES_VALU"] / (64.0 * out["SQ_ACTIVE_INST_VALU"])
    if "SQ_WAVE_CYCLES" in out and out["SQ_WAVE_CYCLES"]:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in out:
                d[k + "_frac"] = out[k] / out["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
        d["l2_hit_rate"] = out["TCC_HIT_sum"] / max(1.0, out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
    if a.config:
        d["config"] = a.config
        d["camera"] = a.camera
        d["kernel"] = a.kernel_id
    d["kernel_name_filter"] = a.kernel
    if a.build_id:
        d["build_id"] = a.build_id
    print(json.dumps(d, indent=1))
    if a.json:
        json.dump(d, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
