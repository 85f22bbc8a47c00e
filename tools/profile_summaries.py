"""Turn a tools/gpu_sq.sh session (gpurun_out/<tag>) into the profile summaries bench.py prices its roofline from:
profiles/sq_<cfg>.json, valu_mix_<cfg>.json, pmc_traffic_<cfg>.json, each stamped with the build id the session
measured (bench.py refuses a profile of another build) and the kernel time from the session's own kernel stats.
A "_orbit" config (c2_orbit, ref_orbit) is the base config with the moving camera (bench.py --camera orbit); its
summaries carry "camera": "orbit".

    python tools/profile_summaries.py gpurun_out/<tag> [--configs c2 ref c3 c4 c2_orbit] [--out profiles] [--source ..]
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# per config: (kernel id, dominant-kernel filter, launches of it per frame, bound, resource, whole-frame PMC filters)
SPEC = {
    "c2": (0, "pt_megakernel<false", 1.0, "valu_issue",
           "VALU issue (SQ_INSTS_VALU x 2 cycles over the SIMD cycles of the launch; the mix-weighted ceiling in "
           "profiles/valu_mix_c2.json)", None),
    "ref": (0, "pt_megakernel<false", 1.0, "valu_issue",
            "VALU issue, with lane utilisation ~0.55: divergent waves (camera inside the mushroom, leaves of 1-43 "
            "triangles)", None),
    "c3": (2, "wf_trace<false", 1.0, "memory_latency",
           "latency of dependent node fetches (waves parked on memory, SQ_WAIT_ANY share of wave cycles) and the loop "
           "control between them", "wf_trace<false,wf_shade<false,wf_init<false"),
    "c4": (2, "wf_trace<false", 130.0, "memory_latency",
           "latency of dependent node fetches (waves parked on memory, SQ_WAIT_ANY share of wave cycles) and the loop "
           "control between them", "wf_trace<false,wf_shade<false,wf_init<false"),
}
MIX = ("ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32", "INT32", "INT64", "CVT")
# megakernel work-items per frame (8x8 tiles x 64 lanes of the 1920x1080 frame): under the frame overlap
# (WCPT_OPTION_FRAME_OVERLAP) a frame is two launches of half the tiles (and one around each re-sort), so the megakernel
# summaries count per frame by grid and time the frame as the union of its launches' intervals (frame_ms)
FRAME_GRID = {"c2": 240 * 135 * 64, "ref": 240 * 135 * 64}
# wavefront pipelines per frame (one wf_init each: the per-frame divisor of the PMC passes). The library picks them by
# queue length (WCPT_OPTION_WF_PIPES 0): 3 for the 1080p atrium (2.1 M paths, 4 per resident trace lane), 2 at 4K
PIPES = {"c3": 3, "c4": 2}


def kernel_ms(d, cfg, filt):
    for f in glob.glob(os.path.join(d, f"prof_{cfg}", "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if filt in row["Name"]:
                return float(row["AverageNs"]) / 1e6
    raise SystemExit(f"{cfg}: no {filt} in the kernel stats")


def frame_ms(d, cfg, filt, frame_grid):
    """A frame's time from the session's kernel trace: the union of the kernel's launch intervals over the frames
    they hold (work-items dispatched / work-items per frame). Launches of consecutive frames overlap under the frame
    overlap, so neither a launch's duration nor their sum is a frame's time."""
    iv, work = [], 0.0
    for f in glob.glob(os.path.join(d, f"prof_{cfg}", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if filt in row["Kernel_Name"]:
                iv.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
                work += float(row["Grid_Size_X"]) * float(row.get("Grid_Size_Y") or 1) * float(row.get("Grid_Size_Z") or 1)
    if not iv:
        raise SystemExit(f"{cfg}: no {filt} in the kernel trace")
    iv.sort()
    busy, s0, e0 = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > e0:
            busy += e0 - s0
            s0, e0 = s, e
        else:
            e0 = max(e0, e)
    busy += e0 - s0
    return busy / 1e6 / (work / frame_grid)


def counters(d, cfg, filt):
    per = defaultdict(list)
    for f in glob.glob(os.path.join(d, f"sq_{cfg}", "p*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if filt in row.get("Kernel_Name", ""):
                per[row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--configs", nargs="+", default=["c2", "ref", "c3", "c4"])
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles"))
    ap.add_argument("--source", default=None)
    a = ap.parse_args()
    build = open(os.path.join(a.dir, "build_id")).read().strip()
    tag = os.path.basename(os.path.normpath(a.dir))
    for cfg in a.configs:
        base = cfg[:-len("_orbit")] if cfg.endswith("_orbit") else cfg
        camera = "orbit" if base != cfg else "still"
        kid, filt, lpf, bound, resource, frame_filters = SPEC[base]
        fg = FRAME_GRID.get(base, 0)
        if fg:
            ms = frame_ms(a.dir, cfg, filt, fg)
            src = (a.source or tag) + f" (tools/gpu_sq.sh; {filt.split('<')[0]} {ms:.4f} ms per frame: the union of " \
                                      f"its launch intervals in the session's kernel trace over the frames they hold; " \
                                      f"camera {camera})"
        else:
            ms = kernel_ms(a.dir, cfg, filt)
            src = (a.source or tag) + f" (tools/gpu_sq.sh; {filt.split('<')[0]} {ms:.4f} ms avg from " \
                                      f"the session's kernel stats; camera {camera})"
        py = sys.executable
        subprocess.run([py, os.path.join(ROOT, "tools", "sq_summary.py"), os.path.join(a.dir, f"sq_{cfg}"), "--kernel",
                        filt, "--ms", str(ms), "--launches-per-frame", str(lpf), "--config", base, "--camera", camera, "--kernel-id",
                        str(kid), "--bound", bound, "--resource", resource, "--source", src, "--build-id", build,
                        "--json", os.path.join(a.out, f"sq_{cfg}.json")] + (["--frame-grid", str(fg)] if fg else []),
                       check=True, stdout=subprocess.DEVNULL)
        pm = [py, os.path.join(ROOT, "tools", "pmc_summary.py"), os.path.join(a.dir, f"sq_{cfg}"), "--config", base,
              "--camera", camera,
              "--kernel-id", str(kid), "--build-id", build, "--json", os.path.join(a.out, f"pmc_traffic_{cfg}.json")]
        pm += (["--kernel", frame_filters, "--frame-kernel", "wf_init<false", "--per-frame", str(PIPES[base])]
               if frame_filters else ["--kernel", filt] + (["--frame-grid", str(fg)] if fg else []))
        subprocess.run(pm, check=True, stdout=subprocess.DEVNULL)
        m, n = counters(a.dir, cfg, filt)
        tot = m.get("SQ_INSTS_VALU")
        frac = {c: m[f"SQ_INSTS_VALU_{c}"] / tot for c in MIX if f"SQ_INSTS_VALU_{c}" in m}
        packed_note = ""
        if "SQ_INSTS_VALU_FLOPS_FP32" in m and {"ADD_F32", "MUL_F32", "FMA_F32", "TRANS_F32"} <= set(frac):
            # packed add/mul: FLOPS_FP32 counts FLOPs per lane of each wave-instruction and a packed instruction once
            # in its class (profiles/valu_flops_calibration.json), so the surplus over ADD + MUL + 2 FMA + TRANS is the
            # packed adds and multiplies (a packed FMA would add 2: counted as one packed add/mul pair, an upper bound)
            am = frac["ADD_F32"] + frac["MUL_F32"]
            surplus = m["SQ_INSTS_VALU_FLOPS_FP32"] / tot - (am + 2 * frac["FMA_F32"] + frac["TRANS_F32"])
            pk = min(max(surplus, 0.0), am)
            if am > 0:
                for c in ("ADD", "MUL"):
                    share = pk * frac[f"{c}_F32"] / am
                    frac[f"PK_{c}_F32"] = share
                    frac[f"{c}_F32"] -= share
            packed_note = (f"; PK_ADD_F32 / PK_MUL_F32 = the packed forms, from SQ_INSTS_VALU_FLOPS_FP32 "
                           f"({m['SQ_INSTS_VALU_FLOPS_FP32'] / tot:.3f} FLOPs per lane per VALU instruction: surplus "
                           f"{surplus:.3f} over one per add/mul/transcendental and two per FMA)")
        frac["other"] = 1.0 - sum(frac.values())
        json.dump({"config": base, "camera": camera, "kernel": kid, "kernel_name_filter": filt, "dispatches": n.get("SQ_INSTS_VALU_ADD_F32"),
                   "SQ_INSTS_VALU_per_launch": tot, "class_fraction": {k: round(v, 4) for k, v in frac.items()},
                   "build_id": build,
                   "source": src + "; one --pmc pass of SQ_INSTS_VALU and its classes; other = the remainder (moves, "
                                   "selects, compares, min/max, bit ops)" + packed_note},
                  open(os.path.join(a.out, f"valu_mix_{cfg}.json"), "w"), indent=1)
        print(f"{cfg}: build {build}, {filt} {ms:.4f} ms, summaries written")


if __name__ == "__main__":
    main()
