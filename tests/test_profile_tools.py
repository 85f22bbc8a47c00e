"""The profile summaries bench.py prices its megakernel rooflines from, on synthetic rocprofv3 CSVs (CPU): under the
frame overlap a frame is two launches of half the tiles (and one around each re-sort), so the counters are normalised
per frame by grid (tools/sq_summary.py, tools/pmc_summary.py --frame-grid) and a frame's time is the union of the
launch intervals over the frames they hold (tools/profile_summaries.py frame_ms)."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import profile_summaries  # noqa: E402

FRAME = 240 * 135 * 64
K = "void wcpt::dev::pt_megakernel<false, false, 1, true, true, false>(...)"


def _counter_csv(path, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, ["Dispatch_Id", "Grid_Size", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, (grid, name, ctr, val) in enumerate(rows):
            w.writerow({"Dispatch_Id": i, "Grid_Size": grid, "Kernel_Name": name, "Counter_Name": ctr,
                        "Counter_Value": val})


def test_counters_per_frame_by_grid(tmp_path):
    # one whole-frame launch (before the first sort) and two frames of two half launches: 3 frames' work in all
    half = FRAME // 2
    rows = [(FRAME, K, "SQ_INSTS_VALU", 1000.0)] + [(half, K, "SQ_INSTS_VALU", 500.0)] * 4 + \
           [(4096, "split_tiles(...)", "SQ_INSTS_VALU", 7.0)]
    _counter_csv(str(tmp_path / "sq" / "p0" / "run_counter_collection.csv"), rows)
    out = tmp_path / "sq.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(tmp_path / "sq"), "--kernel",
                    "pt_megakernel<false", "--ms", "0.35", "--frame-grid", str(FRAME), "--json", str(out)],
                   check=True, stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    assert d["counters_per_launch"]["SQ_INSTS_VALU"] == 1000.0 and d["launches_per_frame"] == 1.0
    # without --frame-grid: the mean per dispatch (the round-5 form, one launch per frame)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sq_summary.py"), str(tmp_path / "sq"), "--kernel",
                    "pt_megakernel<false", "--ms", "0.35", "--json", str(out)], check=True, stdout=subprocess.DEVNULL)
    assert json.load(open(out))["counters_per_launch"]["SQ_INSTS_VALU"] == 600.0


def test_hbm_bytes_per_frame_by_grid(tmp_path):
    half = FRAME // 2
    rows = []
    for g, fs, ws in ((FRAME, 100.0, 40.0), (half, 50.0, 20.0), (half, 50.0, 20.0)):
        rows += [(g, K, "FETCH_SIZE", fs), (g, K, "WRITE_SIZE", ws)]
    _counter_csv(str(tmp_path / "pm" / "p0" / "run_counter_collection.csv"), rows)
    out = tmp_path / "pm.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), str(tmp_path / "pm"), "--kernel",
                    "pt_megakernel<false", "--frame-grid", str(FRAME), "--json", str(out)],
                   check=True, stdout=subprocess.DEVNULL)
    d = json.load(open(out))
    assert d["hbm_bytes_per_frame"] == int((2 * 100 + 40) * 1024) and "hbm_bytes_per_launch" not in d


def test_frame_ms_is_the_union_over_frames(tmp_path):
    d = tmp_path / "prof_c2" / "x"
    os.makedirs(d)
    half = FRAME // 2
    # frame A: one launch 0-350 us; frames B, C: pipes overlapping (B0 400-740, B1 410-760, C0 740-1080, C1 760-1100)
    trace = [(0, 350, FRAME), (400, 740, half), (410, 760, half), (740, 1080, half), (760, 1100, half),
             (1200, 1210, 1024)]
    with open(d / "kt_kernel_trace.csv", "w", newline="") as f:
        w = csv.DictWriter(f, ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y",
                               "Grid_Size_Z"])
        w.writeheader()
        for i, (s, e, g) in enumerate(trace):
            w.writerow({"Kernel_Name": K if i < 5 else "split_tiles(...)", "Start_Timestamp": s * 1000,
                        "End_Timestamp": e * 1000, "Grid_Size_X": g, "Grid_Size_Y": 1, "Grid_Size_Z": 1})
    ms = profile_summaries.frame_ms(str(tmp_path), "c2", "pt_megakernel<false", FRAME)
    assert abs(ms - (350 + 700) / 3 / 1000) < 1e-9
