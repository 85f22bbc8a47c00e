"""bench.py — Mray/s + ms/frame of the MI355X path-tracing compute path (BASELINE.json metric).

Default workload (N=1): BASELINE.json configs[1] = Cornell box (34 triangles + 4 spheres), 1920x1080, 1 spp,
maxBounceCount 4, progressive frames (renderedFramesCount = 0, 1, 2, ...). A "step" is one frame: one render of the
whole frame (with N ranks: each rank renders its row block, SURVEY.md §8(e), and the blocks are gathered to the root
over RCCL). Rays = ray segments = Intersect() calls, counted exactly by the instrumented kernel for the very frames
that were timed (untimed re-run).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|ref] [--camera still|orbit]
                    [--row-stripe S] [--one-process] [--transport rccl|copy|direct] [--devices 0,1,..] [--verify]
                    [--rccl-rehearsal] [--no-cpu-baseline]

Prints one JSON line on rank 0 (its "launch" field names how the ranks were started). Every mode drives the
product's C ABI (include/wcpt.h wcpt_group_*) on the system HIP runtime (/opt/rocm), as the Jai host would; torch is
not imported:
  - --gpus 1 (the default): a group of one, which renders exactly as a single context.
  - under a launcher (torchrun: WORLD_SIZE = N): this process is rank RANK of a one-process-per-GPU group on device
    LOCAL_RANK (wcpt_group_create_rank, ncclCommInitRank); the 128-byte RCCL id, barriers and the max-over-ranks time
    go through a TCP rendezvous (wcpt.rdzv, MASTER_ADDR:MASTER_PORT+1). --gpus, if given, must equal WORLD_SIZE.
  - plain `python bench.py --gpus N` (N > 1, no launcher): before anything touches a GPU, this process spawns N fresh
    rank processes with torchrun's environment (spawn_ranks; never an exec) and waits for them: the same
    one-process-per-GPU path as under torchrun.
  - --one-process (or --transport copy|direct, or --devices): one process, one host thread, a group over devices
    0..N-1 (wcpt_group_create_ex; RCCL ncclCommInitAll, or the COPY / DIRECT transports). Its RCCL form over several
    GPUs has never run on hardware, and its line says "unrehearsed".
  - --dist-backend gloo | gloo-host | torch-nccl under torchrun: the torch.distributed gather of rounds 1-3 (torch
    imported first, so libwcpt binds torch's bundled HIP runtime): N-rank rehearsals on one GPU.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd")]

import numpy as np  # noqa: E402

wcpt = None  # libwcpt.so's binding, imported in main() once the process knows which HIP runtime it binds

CONFIGS = {
    # name: (scene, width, height, spp, maxBounceCount, description)
    "c1": ("cornell", 256, 256, 1, 1, "Cornell box (34 tris), 256x256, 1 spp, 1 bounce"),
    "c2": ("cornell", 1920, 1080, 1, 4, "Cornell box (34 tris), 1920x1080, 1 spp, 4 bounces"),
    "c3": ("atrium", 1920, 1080, 1, 4, "Sponza-scale atrium OBJ (262k tris), 1920x1080, 1 spp, 4 bounces"),
    "c4": ("atrium", 3840, 2160, 16, 4, "Sponza-scale atrium OBJ (262k tris), 3840x2160, 16 spp, 4 bounces"),
    # the reference's own Init scene (PathTracingRenderer.jai:219-243,322-339: mushroom.obj + 4 spheres, editor start
    # camera inside the mushroom's box) at the headline size with its default maxBounceCount 3 (:119)
    "ref": ("reference_init", 1920, 1080, 1, 3, "Reference Init scene (mushroom.obj + 4 spheres), 1920x1080, 1 spp, "
                                                "maxBounceCount 3"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
BASELINE_METRIC = "Mray/s + ms/frame at 1920×1080 1spp; achieved HBM GB/s vs peak"  # BASELINE.json "metric"
# rays = ray segments (Intersect() calls), counted exactly by the instrumented kernel
# Measured best kernel per workload: the megakernel (WCPT_KERNEL_MEGAKERNEL = 0) wins on the
# coherent, L1-resident Cornell box; the wavefront variant (WCPT_KERNEL_WAVEFRONT = 2) on the 262k-triangle atrium.
KERNEL_MEGAKERNEL, KERNEL_WAVEFRONT = 0, 2
DEFAULT_KERNEL = {"c1": KERNEL_MEGAKERNEL, "c2": KERNEL_MEGAKERNEL, "c3": KERNEL_WAVEFRONT, "c4": KERNEL_WAVEFRONT,
                  "ref": KERNEL_MEGAKERNEL}
# VALU issue ceiling (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs at the 2.4 GHz peak engine clock; a wave64 VALU
# instruction issues over 2 cycles on the 32-lane SIMD (tools/valu_peak.hip measures the rates: profiles/r03_valu_peak*.log)
SIMDS = 1024
CLOCK_GHZ = 2.4
CYCLES_PER_VALU = 2
VALU_PEAK_GINSTR = SIMDS * CLOCK_GHZ / CYCLES_PER_VALU  # spec: 1,228.8 G wave64 VALU instructions/s
# the gathered frame's wire format (wcpt.h WCPT_PAYLOAD_*) and its bytes per pixel
GATHER_FORMATS = {"rgb": (3, 12), "rgba": (4, 16), "display": (8, 4)}
# --camera orbit: the editor's camera while the user strafes (D / A at 4.0 * deltaTime, editor.jai:91,105-112) and drags
# with the right mouse button (yaw, editor.jai:138-143), at 60 frames/s, turning back every ORBIT_HALF_PERIOD frames so
# the camera stays in the scene (0.8 units of travel each way: the Cornell box spans [-1, 1]); every such frame resets
# renderedFramesCount to 0 (editor.jai:149-150)
ORBIT_DT = 1.0 / 60.0
ORBIT_YAW_DEG = 0.5
ORBIT_HALF_PERIOD = 12


def algorithmic_bytes(c: dict) -> int:
    """B_seg = 20*S + sum_draw[32*N_pop + 64*N_interior + 48*N_tri] + 60*[hit] + 28*N_draw,
    plus 164 (SceneData) + 32 (image read-modify-write) per pixel."""
    return (20 * c["sphere_tests"] + 32 * c["node_pops"] + 64 * c["interior_visits"] + 48 * c["triangle_tests"]
            + 60 * c["hits"] + 28 * c["draw_fetches"] + (164 + 32) * c["pixels"])


STALE_PROFILES: list = []  # profiles refused because they were measured on another build (reported in the line)


def _profile_key(args) -> str:
    """The profiles/ file key of a bench line: its config, with "_orbit" for the moving camera (its own SQ / PMC passes,
    since the frames differ: no image read, primary records rebuilt every frame)."""
    return args.config + ("_orbit" if getattr(args, "camera", "still") == "orbit" else "")


def _profile_json(path, args):
    """A committed profile summary (profiles/*.json) when it was measured on this config, kernel, camera and build: a
    profile that records another build id (wcpt_build_id of the library it measured) is refused, not reused."""
    if not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None
    build = getattr(args, "build_id", None)
    if build is not None and pm.get("build_id") != build:
        STALE_PROFILES.append(f"{os.path.basename(path)}: build {pm.get('build_id')} != loaded {build}")
        return None
    if (pm.get("config") == args.config and pm.get("kernel") == args.kernel and args.bvh == "midpoint" and
            getattr(args, "camera", "still") == pm.get("camera", "still")):
        return pm
    return None


def roofline(args, tot, render_s, frame_s, devices=1, ranks=1) -> dict:
    """The dominant kernel against the ceiling of the resource that binds it, measured per render.

    Multi-rank lines price the whole frame's work against the devices it ran on: with one rank per GPU, the slowest
    rank's block time against `devices` x each per-GPU ceiling; in a rehearsal (several ranks sharing a GPU, whose
    block renders overlap on it), the frame time against the shared devices' ceilings.

    valu_issue (megakernel; c2): SQ_INSTS_VALU wave-instructions per render from the committed SQ counter pass
      (profiles/sq_<config>.json) over the live render time, against the spec issue rate (1024 SIMDs x 2.4 GHz, one
      wave64 instruction per 2 cycles); measured_ceiling = the rate the kernel's VALU instruction mix could reach
      (profiles/valu_mix_<config>.json x profiles/valu_ceiling.json).
    memory_latency (wavefront trace; c3): dependent scene-line visits (one 64-B child pair per interior visit, one
      triangle record per test) per second of the frame, against the best rate of dependent random line visits the
      cache hierarchy sustains at 8 waves/SIMD (L2-resident chain, tools/gather_bench.hip, profiles/gather_ceiling.json).
    Beside it: the HBM bytes the PMC counters measured (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction), the only
      true HBM load, and under not_a_roofline the SURVEY 8(d) algorithmic bytes, which price every scene fetch at HBM
      cost although these scenes are served from L1/L2/MALL."""
    steps = max(1, args.steps)
    devices = max(1, int(devices))
    if ranks > devices:
        render_s = frame_s  # ranks share a device: their block times overlap there and do not add up to its busy time
    alg_bytes = algorithmic_bytes(tot) / steps
    # SURVEY 8(d)'s bytes price every scene fetch at HBM cost, but these scenes are served from L1/L2/MALL, so their
    # rate exceeds the HBM peak: kept for reference, outside the roofline head (every frac there is physical, <= 1)
    r = {"not_a_roofline": {"algorithmic_bytes_per_render": int(alg_bytes),
                            "algorithmic_gbs": round(alg_bytes / render_s / 1e9, 1),
                            "note": "cache-served: SURVEY 8(d) bytes priced at HBM cost; the scene stays in "
                                    "L1/L2/MALL, so this is not an HBM rate"}}
    key = _profile_key(args)
    pm = _profile_json(args.pmc_json or os.path.join(ROOT, "profiles", f"pmc_traffic_{key}.json"), args)
    traffic = None if pm is None else pm.get("hbm_bytes_per_launch", pm.get("hbm_bytes_per_frame"))
    r["traffic"] = traffic
    if traffic is not None:
        r["hbm_measured_gbs"] = round(traffic / render_s / 1e9, 2)
        r["hbm_measured_frac"] = round(traffic / render_s / 1e9 / (HBM_PEAK_GBS * devices), 4)
    sq = _profile_json(os.path.join(ROOT, "profiles", f"sq_{key}.json"), args)
    bound = None if sq is None else sq.get("bound")
    if bound == "valu_issue":
        valu = sq["counters_per_launch"]["SQ_INSTS_VALU"] * sq.get("launches_per_frame", 1.0)
        achieved = valu / render_s / 1e9
        head = {"bound": "valu_issue", "achieved": round(achieved, 1), "peak": VALU_PEAK_GINSTR * devices,
                "unit": "G wave64 VALU instructions/s", "frac": round(achieved / (VALU_PEAK_GINSTR * devices), 3),
                "source": f"SQ_INSTS_VALU {valu:.4g}/render ({sq.get('source', 'profiles')}) over the live render "
                          f"time; peak {SIMDS} SIMDs x {CLOCK_GHZ} GHz / {CYCLES_PER_VALU} cycles"}
        ceil = _valu_mix_ceiling(key, getattr(args, "build_id", None))
        if ceil:
            # what this kernel's VALU mix can reach: each instruction class at the fastest rate measured for an
            # instruction of that class (tools/valu_peak.hip; v_add/v_mul/v_mov issue about twice as fast as v_fma)
            head["measured_ceiling"] = round(ceil * devices, 1)
            head["measured_frac"] = round(achieved / (ceil * devices), 3)
    elif bound == "memory_latency":
        ceil = _gather_ceiling()
        # the line visits the kernels execute: with samples > 1 every sample after the first shades its primary
        # segment from sample 0's Intersect record (the same ray), so those traversals are counted by the reference's
        # work (COUNT build) but never run, and are taken out here
        reused = tot.get("reused_primary_lines", 0)
        lines = (tot["interior_visits"] + tot["triangle_tests"] - reused) / steps
        achieved = lines / frame_s / 1e9
        head = {"bound": "memory_latency", "achieved": round(achieved, 2), "peak": round(ceil * devices, 2),
                "unit": "G dependent line-visits/s", "frac": round(achieved / (ceil * devices), 3),
                "source": "interior visits + triangle tests executed per frame over the frame time (the reference's "
                          "counts less the primary traversals of samples after the first, which reuse sample 0's "
                          "record); peak: dependent random 64-B line visits at 8 waves/SIMD from an L2-resident "
                          "table (profiles/gather_ceiling.json)"}
        if reused:
            head["reused_primary_lines_per_frame"] = int(reused / steps)
    else:
        head = {"bound": "unprofiled", "achieved": None, "peak": None, "unit": None, "frac": None,
                "source": f"no SQ counter pass of this build committed for {key} "
                          f"(profiles/sq_{key}.json)"}
    if devices > 1:
        head["devices"] = devices  # every peak above is the sum over these GPUs
    if STALE_PROFILES:
        head["stale_profiles_refused"] = sorted(set(STALE_PROFILES))
    if sq is not None:
        head["binding"] = {k: sq[k] for k in ("resource", "valu_issue_share", "wave_cycle_split", "l2_hit_rate",
                                              "lane_utilisation_valu") if k in sq}
    head.update(r)
    return head


def _json_field(name: str, key: str):
    try:
        return float(json.load(open(os.path.join(ROOT, "profiles", name)))[key])
    except (OSError, ValueError, KeyError, TypeError):
        return None


def _valu_mix_ceiling(config: str, build=None):
    """Mix-weighted VALU ceiling (G wave64 instructions/s) of the config's dominant kernel: 1 / sum(f_c / R_c) over the
    instruction classes c of profiles/valu_mix_<config>.json (fractions f_c of SQ_INSTS_VALU) with the class rates R_c
    of profiles/valu_ceiling.json."""
    try:
        rates = json.load(open(os.path.join(ROOT, "profiles", "valu_ceiling.json")))["class_gwave_instr_per_s"]
        mj = json.load(open(os.path.join(ROOT, "profiles", f"valu_mix_{config}.json")))
        if build is not None and mj.get("build_id") != build:
            STALE_PROFILES.append(f"valu_mix_{config}.json: build {mj.get('build_id')} != loaded {build}")
            return None
        mix = mj["class_fraction"]
        t = sum(f / float(rates[c]) for c, f in mix.items() if f > 0)
        return round(1.0 / t, 1) if t > 0 else None
    except (OSError, ValueError, KeyError, TypeError, ZeroDivisionError):
        return None


def _gather_ceiling() -> float:
    v = _json_field("gather_ceiling.json", "l2_resident_chain_glines_per_s")
    return v if v else 207.4  # profiles/r03_gather_ceiling.log (4 MiB, L2-resident)


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _native_oracle() -> tuple[str, str]:
    """BASELINE.md:21's CPU build of the oracle: pt_oracle.c at -O3 -march=native -ffp-contract=off, compiled here on
    the host that runs the bench (-march=native must target THIS CPU, so it cannot be prebuilt in the build container).
    The test oracle (oracle/liboracle.so, -O2) is unchanged. Returns (library path, flags); falls back to the test
    build if no C compiler is available."""
    import subprocess
    import tempfile
    import atexit
    import shutil
    flags = "-O3 -march=native -ffp-contract=off -fno-math-errno -fPIC -std=c11 -shared -pthread"
    tmp = tempfile.mkdtemp(prefix="wcpt_baseline_")
    atexit.register(shutil.rmtree, tmp, True)  # the loaded library stays mapped after its file is removed
    out = os.path.join(tmp, "liboracle_native.so")
    src = os.path.join(ROOT, "oracle", "pt_oracle.c")
    try:
        subprocess.run(["gcc", *flags.split(), "-o", out, src, "-lm"], check=True, capture_output=True, timeout=120)
        return out, flags
    except (OSError, subprocess.SubprocessError):
        return os.path.join(ROOT, "oracle", "liboracle.so"), "-O2 (oracle/Makefile; gcc -march=native build failed)"


def _cgroup_cpu_quota():
    """CPUs the cgroup lets this process use (cgroup v2 cpu.max "quota period"), or None when unlimited/unknown."""
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        return None


def baseline_threads(cpu_count=None, affinity=None, quota="read") -> dict:
    """The CPU baseline's thread count: one thread per CPU this process can actually use (BASELINE.md:21, SURVEY
    §8(d): the port on all host cores), i.e. min(logical CPUs the host reports, CPUs in this process's affinity mask,
    the cgroup CPU quota rounded up). A container may see many more CPUs than its quota lets it run: threads beyond
    the quota only time-slice (256 threads under a 16-CPU quota measured 1.56x below 16 threads).
    Beside it, labelled, the 16-thread per-GPU share of an 8-GPU node's host when that differs."""
    import math
    n = cpu_count if cpu_count is not None else (os.cpu_count() or 1)
    if affinity is None:
        affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    q = _cgroup_cpu_quota() if quota == "read" else quota
    usable = max(1, min(n, affinity, math.ceil(q) if q else n, 1024))
    return {"threads": usable, "share_threads": max(1, min(16, usable)), "logical_cpus": n,
            "affinity_cpus": affinity, "cgroup_cpu_quota": q}


def _cpu_rate(scene, width, height, spp, bounces, threads, budget_s, min_frames):
    """Mray/s of the oracle on `threads` threads over the same workload (full frames when min_frames of them fit in
    ~budget_s; otherwise a bounded sample of 32-row bands spread over the frame)."""
    import oracle  # test infrastructure, used here only as the reported CPU baseline
    meshes = [(m.positions, m.indices, m.nodes) for m in scene.meshes]

    def run(frame, y0, rows):
        sd = scene.scene_data(width, height, max_bounce=bounces, samples=spp, frame=frame)
        t0 = time.perf_counter()
        _, c = oracle.render(sd, scene.materials, scene.spheres, meshes, width, height, y0=y0, rows=rows,
                             threads=threads)
        return time.perf_counter() - t0, c

    band = 32
    t_warm = 0.0
    while t_warm < 1.5:                                  # warm-up: the first ~1 s of bands runs up to 6x slow
        t_warm += run(0, 0, min(band, height))[0]        # (host clock ramp, page faults); not counted
    probe = [run(0, y, band) for y in range(0, max(1, height - band + 1), max(band, (height - band) // 3))][:4]
    t_probe = sum(t for t, _ in probe)
    c_probe = {k: sum(c[k] for _, c in probe) for k in ("segments", "pixels")}
    est_frame = t_probe * height / (band * len(probe))
    if est_frame * min_frames <= budget_s:
        rates, times, segs = [], [], 0
        f = 0
        while f < min_frames or (sum(times) + est_frame <= budget_s and f < 4 * min_frames):
            t, c = run(f, 0, height)
            rates.append(c["segments"] / t / 1e6)
            times.append(t)
            segs += c["segments"]
            f += 1
        order = sorted(range(f), key=lambda i: rates[i])
        med = order[f // 2]
        return {"value": round(rates[med], 4), "frame_ms_median": round(times[med] * 1e3, 2),
                "sample": f"median of {f} full {width}x{height} frames (progressive frames 0..{f - 1}, {segs} "
                          f"segments, {sum(times):.1f} s)"}
    starts = list(range(0, max(1, height - band + 1), max(band, height // 8)))
    t_total, seg, px, bands, frame = t_probe, c_probe["segments"], c_probe["pixels"], len(probe), 0
    while t_total < budget_s:
        for y0 in starts:
            t, c = run(frame, y0, min(band, height - y0))
            t_total += t
            seg += c["segments"]
            px += c["pixels"]
            bands += 1
            if t_total >= budget_s:
                break
        frame += 1
    return {"value": round(seg / t_total / 1e6, 4),
            "sample": f"{bands} bands of <= {band} rows ({px} px, {seg} segments) of the same {width}x{height} "
                      f"workload (a full frame would take ~{est_frame:.0f} s) over {frame + 1} progressive frame(s), "
                      f"{t_total:.1f} s"}


def cpu_baseline(scene, width, height, spp, bounces, budget_s=20.0, min_frames=5):
    """The CPU oracle (a scalar C restatement of pathTracer.comp, oracle/pt_oracle.c, built -O3 -march=native on this
    host; rows claimed dynamically by its threads) on every CPU this process can use (baseline_threads, BASELINE.md:21),
    and beside it on the 16-thread per-GPU share when that differs (then ~60 % of budget_s goes to `value`, the rest to
    `per_gpu_share`)."""
    lib, flags = _native_oracle()
    os.environ["WCPT_ORACLE_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    th = baseline_threads()
    where = f"{_cpu_model()}, oracle/pt_oracle.c built {flags} (lavapipe is not available)"
    split = th["share_threads"] != th["threads"]
    allc = _cpu_rate(scene, width, height, spp, bounces, th["threads"], (0.6 if split else 1.0) * budget_s, min_frames)
    out = {"value": allc["value"], "unit": "Mray/s", "cores": th["threads"], "kind": "port",
           "sample": f"{allc['sample']} on {th['threads']} threads (the CPUs this process can use: "
                     f"{th['logical_cpus']} logical CPUs reported, {th['affinity_cpus']} in its affinity mask, cgroup "
                     f"quota {th['cgroup_cpu_quota'] or 'none'}) of {where}",
           "logical_cpus": th["logical_cpus"], "affinity_cpus": th["affinity_cpus"],
           "cgroup_cpu_quota": th["cgroup_cpu_quota"]}
    if "frame_ms_median" in allc:
        out["frame_ms_median"] = allc["frame_ms_median"]
    if split:
        sh = _cpu_rate(scene, width, height, spp, bounces, th["share_threads"], 0.4 * budget_s, min_frames)
        out["per_gpu_share"] = {"value": sh["value"], "unit": "Mray/s", "cores": th["share_threads"],
                                "label": "16 threads: one GPU's share of an 8-GPU node's host (not the baseline)",
                                "sample": sh["sample"]}
    return out



# ---- topology and frame sequence (host logic, CPU-tested: tests/test_bench_cli.py) ------------------------------------
def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default 1; under torchrun WORLD_SIZE, which --gpus must then equal)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed renders of frame 0 for this long before the warmup steps, so that the timed steps "
                         "do not run while the GPU clocks ramp up (measured: 3 warmup frames of c2 leave the timed "
                         "region ~9%% slow); frame 0 overwrites the image, so the timed frames are unchanged")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", type=int, default=-1,
                    help="0 megakernel, 2 wavefront, -1 per-config default (DEFAULT_KERNEL)")
    ap.add_argument("--wf-refill", type=int, default=0,
                    help="WCPT_OPTION_WF_REFILL: idle lanes before a trace wave refetches (0: the library default)")
    ap.add_argument("--wf-fetch", type=int, default=-1, choices=[-1, 0, 1],
                    help="WCPT_OPTION_WF_FETCH: wavefront trace fetch rounds per iteration (-1: the library's choice)")
    ap.add_argument("--wf-persist", type=int, default=-1, choices=[-1, 0, 1],
                    help="WCPT_OPTION_WF_PERSIST: the path-persistent wavefront trace (-1: the library's choice)")
    ap.add_argument("--frame-overlap", type=int, default=-1, choices=[-1, 0, 1, 2],
                    help="WCPT_OPTION_FRAME_OVERLAP: megakernel frames overlapped on two pipes (-1: the library's default)")
    ap.add_argument("--wf-pipes", type=int, default=0,
                    help="wavefront kernel: concurrent pipelines (WCPT_OPTION_WF_PIPES; 0 = the library default)")
    ap.add_argument("--camera", default="still", choices=["still", "orbit"],
                    help="still: progressive frames of a still camera (renderedFramesCount = 0, 1, ...); orbit: the "
                         "camera moves every frame as in an editor drag (strafe + yaw, renderedFramesCount = 0 each "
                         "frame, editor.jai:149-150), so the primary-ray records are rebuilt for every frame")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--pmc-json", default=None,
                    help="PMC HBM-traffic summary for roofline.traffic (default profiles/pmc_traffic_<config>.json, "
                         "written by tools/pmc_summary.py)")
    ap.add_argument("--bvh", default="midpoint", choices=["midpoint", "sah"],
                    help="BVH builder: the reference's midpoint split (default: the benchmarked workload) or the "
                         "optional binned SAH (a different tree, reported as a separate workload)")
    ap.add_argument("--gather", default="rgb", choices=sorted(GATHER_FORMATS),
                    help="N>1 wire format of the row blocks: rgb (default; alpha is always 1.0 and is restored on "
                         "the root, bit-identical frame, 12 B/px), the full rgba32f block (16 B/px), or display: "
                         "composite.comp's RGBA8 display value written by the render itself "
                         "(WCPT_PAYLOAD_DISPLAY_RGBA8, 4 B/px; what the root presents, not the accumulation)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: gather each frame in line with the renders instead of overlapping it with the next "
                         "render (WCPT_GROUP_OPTION_OVERLAP 0)")
    ap.add_argument("--group-threads", type=int, default=None, choices=[-1, 0, 1],
                    help="one-process group: issue each rank's share of a frame from a host thread of its own "
                         "(WCPT_GROUP_OPTION_THREADS; default: the library's, 0 = off; -1 = on when the ranks span "
                         "several devices)")
    ap.add_argument("--transport", default="rccl", choices=["rccl", "copy", "direct"],
                    help="one-process group: RCCL send/recv (default), hipMemcpyPeerAsync of each block, or direct: "
                         "each rank's render writes its rows of the root's frame over xGMI (no transfer step)")
    ap.add_argument("--devices", default=None,
                    help="one-process group: device of each rank, comma-separated (default 0..N-1); a device listed "
                         "more than once rehearses N ranks on fewer GPUs (needs --transport copy)")
    ap.add_argument("--watchdog-s", type=float, default=900.0,
                    help="end the process (exit 3, message on stderr) if the run has not finished after this many "
                         "seconds: a rank whose peer died, or a collective set-up that never completes, must not hang "
                         "the launcher (0 = off)")
    ap.add_argument("--events-after", action="store_true",
                    help="time the kernels in an untimed re-render after the timed region (as at N > 1) instead of "
                         "with HIP events inside it (measures what the per-render event records cost)")
    ap.add_argument("--verify", action="store_true",
                    help="the root re-renders the timed frame sequence on one device and checks the presented frame "
                         "against it bit for bit (adds 'verified' to the JSON line)")
    ap.add_argument("--rccl-rehearsal", action="store_true",
                    help="under torchrun on fewer GPUs than ranks: give each rank its own NCCL_HOSTID so that RCCL, "
                         "which refuses two ranks of one communicator on one device of one host, runs the product's "
                         "one-process-per-GPU group with its ranks on one GPU, exchanging over its network transport "
                         "(sockets on the loopback) instead of xGMI: the same wcpt_group_create_rank / ncclSend / "
                         "ncclRecv calls, another wire")
    ap.add_argument("--dist-backend", default="rccl", choices=["rccl", "gloo", "gloo-host", "torch-nccl"],
                    help="under torchrun: rccl (default) = the product's one-process-per-device group over RCCL, no "
                         "torch; gloo / gloo-host / torch-nccl = the torch.distributed gather (gloo rehearses N ranks "
                         "on one GPU, where RCCL refuses two ranks on one device)")
    ap.add_argument("--one-process", action="store_true",
                    help="N > 1 without a launcher: drive every rank from this one process and thread "
                         "(wcpt_group_create_ex; RCCL ncclCommInitAll) instead of spawning one process per GPU. With "
                         "RCCL over several GPUs this form has never run on hardware, and the line says so")
    ap.add_argument("--row-stripe", type=int, default=0,
                    help="N > 1: interleaved row stripes of this many rows (WCPT_GROUP_OPTION_ROW_STRIPE; rank r renders "
                         "stripes r, r + N, ...) instead of contiguous row blocks (0, the default)")
    ap.add_argument("--group-timeout-ms", type=int, default=None,
                    help="WCPT_GROUP_OPTION_TIMEOUT_MS: how long wcpt_group_sync waits for a frame's exchange before "
                         "it aborts the communicator and returns WCPT_ERROR_DEVICE_LOST (default: the library's; "
                         "0 = wait forever)")
    return ap.parse_args(argv)


def launch_plan(args, env) -> str:
    """How this invocation runs its ranks, decided before anything touches the GPU:
      "ranks"  -- under a launcher (WORLD_SIZE set): this process is one rank of a one-process-per-GPU group;
      "spawn"  -- plain `python bench.py --gpus N` (N > 1, RCCL): this process spawns N fresh rank processes, each
                  running the one-process-per-GPU path that torchrun runs (wcpt_group_create_rank), and waits for them;
      "group"  -- one process drives every rank (N = 1; or --one-process, --transport copy|direct, --devices)."""
    if int(env.get("WORLD_SIZE", "1")) > 1:
        return "ranks"
    n = 1 if args.gpus is None else args.gpus
    if n > 1 and not args.one_process and args.transport == "rccl" and not args.devices:
        return "spawn"
    return "group"


def _free_tcp_port(addr: str = "127.0.0.1") -> int:
    import socket
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    try:
        s.bind((addr, 0))
        return s.getsockname()[1]
    finally:
        s.close()


def spawn_env(env, n: int, rank: int, port: int, run_id: str) -> dict:
    """The environment of spawned rank `rank` of `n`: what torchrun gives its workers (RANK, LOCAL_RANK, WORLD_SIZE,
    LOCAL_WORLD_SIZE, MASTER_ADDR/PORT, a run id for the rendezvous token), plus WCPT_BENCH_LAUNCH=spawn so the line
    names the launch."""
    e = dict(env)
    e.update(WORLD_SIZE=str(n), RANK=str(rank), LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
             MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_RUN_ID=run_id, WCPT_BENCH_LAUNCH="spawn")
    return e


def spawn_ranks(argv, n: int, env=None, child_cmd=None, timeout_s: float = 0.0, poll_s: float = 0.05) -> int:
    """Run `n` rank processes of this bench (the same argv; each sees WORLD_SIZE = n) and wait for them. The parent
    never loads libwcpt or touches a GPU, and never execs: every rank is a fresh child process (subprocess), which
    inherits stdout/stderr, so rank 0's JSON line is this command's output. When a rank fails, the others are
    terminated (they would wait for its exchange); returns 0, the first failing rank's exit status (128 + signal for a
    signalled one), or 3 when the ranks outlive `timeout_s`."""
    import secrets
    import signal
    import subprocess
    env = dict(os.environ if env is None else env)
    cmd = list(child_cmd) if child_cmd else [sys.executable, os.path.abspath(__file__)]
    port = _free_tcp_port()
    run_id = f"wcpt-spawn-{os.getpid()}-{secrets.token_hex(4)}"
    procs = []

    def die_with_parent():
        # in the child before it runs the rank: a SIGKILL when this spawner dies, so no rank outlives it holding a GPU
        # (Linux prctl PR_SET_PDEATHSIG; the spawner has made no HIP call, so forking it is safe)
        try:
            import ctypes
            ctypes.CDLL(None, use_errno=True).prctl(1, signal.SIGKILL)
        except (OSError, AttributeError):
            pass

    def on_term(signum, frame):   # a launcher's SIGTERM / SIGINT: stop the ranks (the finally below), then exit
        raise SystemExit(128 + signum)

    old = {sig: signal.signal(sig, on_term) for sig in (signal.SIGTERM, signal.SIGINT)}
    try:
        for r in range(n):
            procs.append(subprocess.Popen(cmd + list(argv), env=spawn_env(env, n, r, port, run_id),
                                          preexec_fn=die_with_parent))
        deadline = time.monotonic() + timeout_s if timeout_s and timeout_s > 0 else None
        rc = 0
        while [p.poll() for p in procs].count(None):      # poll every rank (any() would stop at the first)
            bad = [p for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0].returncode
                sys.stderr.write(f"bench.py: rank {procs.index(bad[0])} exited with {rc}; stopping the other ranks\n")
                break
            if deadline is not None and time.monotonic() > deadline:
                sys.stderr.write(f"bench.py: spawned ranks still running after {timeout_s:.0f} s; stopping them\n")
                rc = 3
                break
            time.sleep(poll_s)
        else:
            rc = next((p.returncode for p in procs if p.returncode), 0)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        for sig, h in old.items():
            signal.signal(sig, h)
    return 128 - rc if rc < 0 else rc


def resolve_topology(args, env) -> dict:
    """Which ranks this process drives. Raises SystemExit on a contradiction instead of measuring something else."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world > 1:
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} under a launcher with WORLD_SIZE={world}: one rank per "
                             f"GPU, so they must agree")
        if args.devices or args.one_process:
            raise SystemExit("bench.py: --devices / --one-process are for the one-process group (no WORLD_SIZE)")
        local = int(env.get("LOCAL_RANK", env.get("RANK", "0")))
        if args.rccl_rehearsal and args.dist_backend != "rccl":
            raise SystemExit("bench.py: --rccl-rehearsal rehearses the RCCL group (--dist-backend rccl)")
        if args.row_stripe and args.dist_backend != "rccl":
            raise SystemExit("bench.py: --row-stripe is an option of the C-ABI group (--dist-backend rccl)")
        return {"mode": "ranks" if args.dist_backend == "rccl" else "torch", "nranks": world,
                "rank": int(env.get("RANK", "0")), "local_rank": local, "devices": [local]}
    if args.dist_backend != "rccl":
        raise SystemExit(f"bench.py: --dist-backend {args.dist_backend} needs a torchrun launch (WORLD_SIZE > 1)")
    if args.rccl_rehearsal:
        raise SystemExit("bench.py: --rccl-rehearsal needs several ranks (--gpus N > 1, or a launcher's WORLD_SIZE)")
    n = 1 if args.gpus is None else args.gpus
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}")
    devices = [int(x) for x in args.devices.split(",")] if args.devices else list(range(n))
    if len(devices) != n:
        raise SystemExit(f"bench.py: --devices names {len(devices)} devices for --gpus {n}")
    if len(set(devices)) < n and args.transport == "rccl":
        raise SystemExit("bench.py: a device listed twice needs --transport copy or direct (RCCL: one rank per device)")
    return {"mode": "group", "nranks": n, "rank": 0, "local_rank": 0, "devices": devices}


def orbit_camera(cam, step: int):
    """The editor's camera after `step` frames of strafing while dragging (editor.jai:88-143): D with a rightward drag
    for ORBIT_HALF_PERIOD frames, then A with a leftward drag as long, and so on, applied from `cam`."""
    c = type(cam)()
    import ctypes as C
    C.pointer(c)[0] = cam
    for i in range(step):
        sign = 1.0 if (i // ORBIT_HALF_PERIOD) % 2 == 0 else -1.0
        yaw90 = np.radians(c.yaw + 90.0)
        speed = 4.0 * ORBIT_DT
        c.position[0] += sign * float(np.cos(yaw90)) * speed
        c.position[2] += sign * float(np.sin(yaw90)) * speed
        c.yaw -= sign * ORBIT_YAW_DEG
    return c


class FrameSource:
    """SceneData of frame k of the run (settle frames use k = 0). Still camera: renderedFramesCount = k (progressive
    accumulation). Orbit: camera moved k editor steps, renderedFramesCount = 0 (editor.jai:149-150). The SceneData
    arrays are built before the timed region (host camera math is not the path)."""

    def __init__(self, scene, W, H, bounces, spp, camera: str, frames: int):
        self.still = camera == "still"
        self.sd = [scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)]
        if not self.still:
            cam = scene.camera
            self.sd = [scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0, camera=orbit_camera(cam, k))
                       for k in range(frames)]

    def __call__(self, k: int):
        if self.still:
            sd = self.sd[0]
            sd["renderedFramesCount"] = k
            return sd
        return self.sd[k]

    def copy(self, k: int):
        return np.array(self(k), copy=True)


# ---- drivers: the product's C-ABI group, or the torch.distributed rehearsal ------------------------------------------
class GroupBench:
    """wcpt_group_* (include/wcpt.h): all ranks in this process (mode "group") or this process's rank of a
    one-process-per-device group (mode "ranks", RCCL id through the rendezvous)."""

    def __init__(self, args, topo, scene, W, H, rdzv=None):
        T = wcpt._lib
        self.topo, self.W, self.H = topo, W, H
        if topo["mode"] == "group":
            transport = {"rccl": T.GROUP_TRANSPORT_RCCL, "copy": T.GROUP_TRANSPORT_COPY,
                         "direct": T.GROUP_TRANSPORT_DIRECT}[args.transport]
            self.g = wcpt.Group(topo["devices"], root=0, transport=transport)
        else:
            uid = wcpt.group_unique_id() if topo["rank"] == 0 else None
            uid = rdzv.broadcast(uid)
            # LOCAL_RANK names the device; a launcher that shows each process fewer devices (one per process) gets
            # its LOCAL_RANK folded onto what it sees
            dev = topo["local_rank"]
            seen = wcpt.device_count()
            if seen > 0 and dev >= seen:
                dev %= seen
            topo["devices"] = [dev]
            self.g = wcpt.Group.rank(dev, topo["nranks"], topo["rank"], root=0, uid=uid)
        self.ctxs = self.g.contexts
        self.ranks = self.g.ranks
        self.devs = []
        for c in self.ctxs:
            c.set_kernel(args.kernel)
            if args.wf_pipes:
                c.set_option(T.OPTION_WF_PIPES, args.wf_pipes)
            if args.wf_refill:
                c.set_option(T.OPTION_WF_REFILL, args.wf_refill)
            if args.wf_fetch >= 0:
                c.set_option(T.OPTION_WF_FETCH, args.wf_fetch)
            if args.wf_persist >= 0:
                c.set_option(T.OPTION_WF_PERSIST, args.wf_persist)
            if getattr(args, "frame_overlap", -1) >= 0:
                c.set_option(T.OPTION_FRAME_OVERLAP, args.frame_overlap)
            self.devs.append(wcpt.DeviceScene(c, scene))
        self.g.set_option(T.GROUP_OPTION_OVERLAP, 0 if args.no_overlap else 1)
        if getattr(args, "group_threads", None) is not None:
            self.g.set_option(T.GROUP_OPTION_THREADS, args.group_threads)
        if getattr(args, "group_timeout_ms", None) is not None:
            self.g.set_option(T.GROUP_OPTION_TIMEOUT_MS, args.group_timeout_ms)
        if getattr(args, "row_stripe", 0):
            self.g.set_option(T.GROUP_OPTION_ROW_STRIPE, args.row_stripe)
        self.g.create_screen(W, H)
        self.fmt, self.px = GATHER_FORMATS[args.gather]
        self.out = None
        if topo["nranks"] > 1:
            root = self.g.context(0)
            nbytes = W * H * self.px
            if root is not None:
                self.out = root.buffer_alloc(nbytes)
                self.g.set_output(self.fmt, root.buffer_address(self.out), nbytes)
            else:
                self.g.set_output(self.fmt, 0, nbytes)  # every process passes the output's size (wcpt.h)
        self.addr = [list(a) for a in zip(*[d.addresses() for d in self.devs])]
        # the per-rank address arrays, built once: a step's host work is one ctypes call (at 8 ranks a c2 block renders
        # in ~0.07 ms, so the host's per-step cost has to stay well below that)
        import ctypes as C
        n = len(self.ranks)
        self._arrs = [(C.c_uint64 * n)(*[int(v) for v in a]) for a in self.addr]
        self._render = wcpt.lib.wcpt_group_render

    def render(self, sd):
        rc = self._render(self.g.h, sd.ctypes.data, *self._arrs)
        if rc:
            wcpt._lib.check(rc)

    def sync(self):
        self.g.sync()

    def presenting(self, on: bool):
        if self.topo["nranks"] == 1:
            return
        if on:
            root = self.g.context(0)
            if root is not None:
                self.g.set_output(self.fmt, root.buffer_address(self.out), self.W * self.H * self.px)
            else:
                self.g.set_output(self.fmt, 0, self.W * self.H * self.px)
        else:
            self.g.set_output(0, 0, 0)

    def profile_begin(self, region=False):
        for c in self.ctxs:
            c.set_option(wcpt._lib.OPTION_PROFILE_REGION, 1 if region else 0)
            c.profile_begin()

    def profile_end(self):
        return [c.profile_end() for c in self.ctxs]

    def counters(self, sd):
        tot = {}
        for c, d in zip(self.ctxs, self.devs):
            for k, v in c.render_counters(sd, *d.addresses()).items():
                tot[k] = max(tot.get(k, 0), v) if k == "ref_stack_max" else tot.get(k, 0) + v
        return tot

    def frame(self):
        """The presented frame on the root's process (None elsewhere): [H, W, 4] float32 (rgb: alpha restored), or
        [H, W, 4] uint8 for the display format."""
        root = self.g.context(0)
        if root is None:
            return None
        if self.out is None:
            return root.readback(self.H)
        raw = root.buffer_download(self.out, self.W * self.H * self.px)
        if self.fmt == wcpt._lib.PAYLOAD_DISPLAY_RGBA8:
            return np.frombuffer(raw, np.uint8).reshape(self.H, self.W, 4)
        img = np.frombuffer(raw, np.float32).reshape(self.H, self.W, self.fmt)
        if self.fmt == 3:
            img = np.concatenate([img, np.ones(img.shape[:2] + (1,), np.float32)], axis=2)
        return img

    def info(self):
        return self.g.info()

    def close(self):
        for d in self.devs:
            d.free()
        if self.out is not None:
            self.g.context(0).buffer_free(self.out)
        self.g.close()


class TorchBench:
    """The rounds 1-3 multi-process path: each process renders its row block with its own context on device
    LOCAL_RANK and torch.distributed gathers the render-written payloads on a communication stream (gloo rehearses
    N ranks on one GPU; torch-nccl is RCCL through torch). torch was imported before libwcpt, so both share torch's
    bundled HIP runtime."""

    def __init__(self, args, topo, scene, W, H):
        import torch
        import torch.distributed as dist
        from wcpt.dist import row_block
        self.torch, self.dist = torch, dist
        self.W, self.H, self.world, self.rank = W, H, topo["nranks"], topo["rank"]
        device = topo["local_rank"] % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "torch-nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        self.host_staged = args.dist_backend == "gloo-host"
        # one explicit stream for the renders and the payload hand-off (torch's default stream handle 0 would be read
        # by wcpt_set_stream as "the context's own stream", leaving the gather unordered with the render)
        self.stream = torch.cuda.Stream(device=device)
        torch.cuda.set_stream(self.stream)
        self.ctx = wcpt.Context(device)
        self.ctx.set_stream(self.stream.cuda_stream)
        self.ctx.set_kernel(args.kernel)
        if args.wf_pipes:
            self.ctx.set_option(wcpt._lib.OPTION_WF_PIPES, args.wf_pipes)
        if args.wf_refill:
            self.ctx.set_option(wcpt._lib.OPTION_WF_REFILL, args.wf_refill)
        if args.wf_fetch >= 0:
            self.ctx.set_option(wcpt._lib.OPTION_WF_FETCH, args.wf_fetch)
        if args.wf_persist >= 0:
            self.ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, args.wf_persist)
        if getattr(args, "frame_overlap", -1) >= 0:
            self.ctx.set_option(wcpt._lib.OPTION_FRAME_OVERLAP, args.frame_overlap)
        self.dev = wcpt.DeviceScene(self.ctx, scene)
        self.ctx.create_screen(W, H)
        y0, rows = row_block(H, self.world, self.rank)
        self.ctx.set_row_range(y0, rows)
        max_rows = -(-H // self.world)
        self.shard = torch.zeros((max_rows, W, 4), dtype=torch.float32, device="cuda")
        self.ctx.set_external_image(self.shard.data_ptr(), self.shard.numel() * 4)
        self.channels = GATHER_FORMATS[args.gather][0]
        pdt, pch = (torch.uint8, 4) if args.gather == "display" else (torch.float32, self.channels)
        self.overlap = not args.no_overlap
        nbuf = 3 if self.overlap else 1
        self.comm = torch.cuda.Stream(device=device) if self.overlap else None
        self.payload = [torch.empty((max_rows, W, pch), dtype=pdt, device="cuda") for _ in range(nbuf)]
        self.gathered = [[torch.empty(self.payload[0].shape, dtype=pdt, device="cpu" if self.host_staged else "cuda")
                          for _ in range(self.world)] for _ in range(nbuf)] if self.rank == 0 else None
        self.ready_ev = [torch.cuda.Event() for _ in range(nbuf)]
        self.done_ev = [torch.cuda.Event() for _ in range(nbuf)]
        self.done_used = [False] * nbuf
        self.k = 0
        self.last = 0
        self.on = True
        self.ctxs = [self.ctx]
        self.ranks = [self.rank]

    def render(self, sd):
        if not self.on:
            self.ctx.render(sd, *self.dev.addresses())
            return
        nbuf = len(self.payload)
        i = self.k % nbuf
        self.k += 1
        self.last = i
        out = self.gathered[i] if self.rank == 0 else None
        if self.overlap and self.done_used[i]:
            self.done_ev[i].synchronize()
        p = self.payload[i]
        self.ctx.set_gather_output(p.data_ptr(), p.numel() * p.element_size(), self.channels)
        self.ctx.render(sd, *self.dev.addresses())
        src = p.cpu() if self.host_staged else p
        if not self.overlap:
            self.dist.gather(src, out, dst=0)
            return
        self.ready_ev[i].record(self.stream)
        with self.torch.cuda.stream(self.comm):
            self.comm.wait_event(self.ready_ev[i])
            self.dist.gather(p.cpu() if self.host_staged else p, out, dst=0)
            self.done_ev[i].record(self.comm)
        self.done_used[i] = True

    def sync(self):
        self.torch.cuda.synchronize()

    def presenting(self, on: bool):
        self.on = on
        if not on:
            self.ctx.set_gather_output(0, 0)

    def profile_begin(self, region=False):
        self.ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 1 if region else 0)
        self.ctx.profile_begin()

    def profile_end(self):
        return [self.ctx.profile_end()]

    def counters(self, sd):
        return self.ctx.render_counters(sd, *self.dev.addresses())

    def frame(self):
        if self.rank != 0:
            return None
        from wcpt.dist import assemble
        img = assemble([g.to("cpu") for g in self.gathered[self.last]], self.H, self.world).numpy()
        return img

    def info(self):
        return {"nranks": self.world, "local_ranks": 1, "first_local_rank": self.rank, "root": 0, "transport": -1,
                "overlap": int(self.overlap), "distinct_devices": 1, "broken": 0, "frames": self.k}

    def close(self):
        self.ctx.set_gather_output(0, 0)
        self.ctx.set_external_image(0, 0)
        self.dev.free()
        self.ctx.close()
        self.dist.destroy_process_group()


class _Collective:
    """Barriers and the cross-rank sums / maxima of the report, over whichever host channel the mode has."""

    def __init__(self, topo, rdzv=None, torch_dist=None):
        self.topo, self.rdzv, self.td = topo, rdzv, torch_dist

    def barrier(self):
        if self.rdzv is not None:
            self.rdzv.barrier()
        elif self.td is not None:
            self.td.barrier()

    def agree(self, flag: bool) -> bool:
        """Rank 0's flag on every rank (a loop whose length one rank decides by its clock must run as many times on
        all of them: each iteration posts a frame's exchange, and a rank that posts one more waits forever)."""
        if self.rdzv is not None:
            return bool(self.rdzv.broadcast(b"\x01" if flag else b"\x00")[0])
        if self.td is not None:
            box = [bool(flag)]
            self.td.broadcast_object_list(box, src=0)
            return bool(box[0])
        return flag

    def gather_obj(self, obj):
        """Every rank's obj on rank 0 (list in rank order), None elsewhere."""
        if self.rdzv is not None:
            return self.rdzv.gather_obj(obj)
        if self.td is not None:
            out = [None] * self.topo["nranks"] if self.topo["rank"] == 0 else None
            self.td.gather_object(obj, out, dst=0)
            return out
        return [obj]


def verify_frame(args, topo, scene, W, H, spp, bounces, frames: FrameSource, nframes, got):
    """The presented frame against one context on the root's device rendering the same frame sequence: bit-equal
    float bit patterns (rgb: alpha restored), or bytes for the display format (wcpt_composite of that render)."""
    with wcpt.Context(topo["devices"][0]) as vctx:
        vdev = wcpt.DeviceScene(vctx, scene)
        vctx.set_kernel(args.kernel)
        vctx.create_screen(W, H)
        for f in range(nframes):
            vctx.render(frames(f), *vdev.addresses())
        if got.dtype == np.uint8:
            buf = vctx.buffer_alloc(W * H * 4)
            vctx.composite(vctx.buffer_address(buf), rgba8=True)
            vctx.sync()
            ref = np.frombuffer(vctx.buffer_download(buf, W * H * 4), np.uint8).reshape(H, W, 4)
            vctx.buffer_free(buf)
        else:
            ref = vctx.readback()
        vdev.free()
    bits = np.uint8 if ref.dtype == np.uint8 else np.uint32
    same = got.view(bits) == ref.view(bits)
    ok = bool(same.all())
    if not ok:
        bad_rows = np.nonzero(~same.all(axis=(1, 2)))[0]
        print(f"verify: {bad_rows.size} of {H} rows differ (first {bad_rows[:8].tolist()}, last "
              f"{bad_rows[-4:].tolist()}); pixel fraction {1.0 - same.all(axis=2).mean():.4f}", file=sys.stderr,
              flush=True)
        if os.environ.get("WCPT_VERIFY_DUMP"):
            np.savez(os.environ["WCPT_VERIFY_DUMP"], got=got, ref=ref)
    return ok


def _gpu_identity(device: int) -> str:
    try:
        return wcpt.device_pci_bus_id(device)
    except Exception:  # an older library or a runtime without the query: the ordinal, this process's view
        return f"ordinal {device}"


def _start_watchdog(seconds, topo):
    """A daemon timer that ends this process if the run outlives `seconds` (a hung collective: a peer that died, an
    RCCL set-up that never completes). os._exit, not an exception: the main thread may be blocked inside a device
    wait. Started before anything touches the GPU; cancelled when the line has been printed."""
    if not seconds or seconds <= 0:
        return None
    import threading

    def fire():
        sys.stderr.write(f"bench.py: watchdog: rank {topo['rank']} of {topo['nranks']} still running after "
                         f"{seconds:.0f} s; exiting. Where every thread was:\n")
        sys.stderr.flush()
        import faulthandler
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(3)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def rccl_rehearsal_env(env, rank: int):
    """--rccl-rehearsal: RCCL detects two ranks on one device by (host hash, PCI bus id) and refuses them; a per-rank
    NCCL_HOSTID gives each rank a host of its own, so the communicator forms and its peers talk over the network
    transport (sockets; the loopback interface unless NCCL_SOCKET_IFNAME says otherwise, no InfiniBand). Set before
    the first RCCL call of the process (ncclGetUniqueId / ncclCommInitRank read the environment then)."""
    env["NCCL_HOSTID"] = f"wcpt-rehearsal-{rank}"
    env.setdefault("NCCL_SOCKET_IFNAME", "lo")
    env.setdefault("NCCL_IB_DISABLE", "1")


def main(argv=None):
    global wcpt
    args = parse_args(argv)
    if launch_plan(args, os.environ) == "spawn":
        # before any GPU call in this process: the ranks are fresh processes (never an exec of this one)
        wd = args.watchdog_s + 120.0 if args.watchdog_s and args.watchdog_s > 0 else 0.0
        return spawn_ranks(sys.argv[1:] if argv is None else list(argv), args.gpus, timeout_s=wd)
    topo = resolve_topology(args, os.environ)
    watchdog = _start_watchdog(args.watchdog_s, topo)
    if args.rccl_rehearsal:
        rccl_rehearsal_env(os.environ, topo["rank"])
    if topo["mode"] == "torch":
        import torch  # noqa: F401  (first: libwcpt.so then binds the HIP runtime torch loaded; one runtime per process)
        import torch.distributed as tdist
    import wcpt as _wcpt
    wcpt = _wcpt
    from wcpt import scene as wscene
    if topo["mode"] != "torch":
        assert "torch" not in sys.modules, "the C-ABI bench must not load torch's HIP runtime"

    name, W, H, spp, bounces, desc = CONFIGS[args.config]
    if args.kernel < 0:
        args.kernel = DEFAULT_KERNEL[args.config]
    args.build_id = wcpt.build_id()
    rank, nranks = topo["rank"], topo["nranks"]
    scene = wscene.generate(name, bvh=args.bvh)
    frames = FrameSource(scene, W, H, bounces, spp, args.camera, args.warmup + args.steps)
    rdzv = None
    if topo["mode"] == "ranks":
        from wcpt.rdzv import Rendezvous
        rdzv = Rendezvous.from_env()
    if topo["mode"] == "torch":
        drv = TorchBench(args, topo, scene, W, H)
        coll = _Collective(topo, torch_dist=tdist)
    else:
        drv = GroupBench(args, topo, scene, W, H, rdzv)
        coll = _Collective(topo, rdzv=rdzv)

    t_settle = time.perf_counter()
    # the settle phase's length is rank 0's clock's decision, agreed every 8 frames (each frame posts an exchange)
    while coll.agree((time.perf_counter() - t_settle) * 1e3 < args.settle_ms):
        for _ in range(8):
            drv.render(frames(0))
        drv.sync()
    for f in range(args.warmup):
        drv.render(frames(f))
    drv.sync()
    args.kernel_auto = args.kernel == wcpt.KERNEL_AUTO
    if args.kernel_auto:  # the variant the library chose for this scene: the profiles and the line name that one
        args.kernel = int(drv.ctxs[0].last_kernel())
    coll.barrier()
    drv.sync()
    # Kernel time for the roofline. With one rank: two HIP events on the render stream bracket the timed renders
    # (WCPT_OPTION_PROFILE_REGION), and the launch duration is their interval over the renders, the gaps between
    # launches included; a pair of events around every render would cost ~1.3 % of a c2 frame
    # (profiles/r05_events_ab.log). With more ranks the events are left out of the timed region (at 8 ranks a c2 block
    # renders in ~0.07 ms, and event records per render and rank are host work of that order): the same frames are
    # re-rendered afterwards, untimed, with a pair of events around every render and presenting off.
    live_events = nranks == 1 and not args.events_after
    if live_events:
        drv.profile_begin(region=True)
    t0 = time.perf_counter()
    for k in range(args.steps):
        drv.render(frames(args.warmup + k))
    drv.sync()
    elapsed = time.perf_counter() - t0
    coll.barrier()
    got = drv.frame() if args.verify else None
    if not live_events:
        drv.presenting(False)
        drv.profile_begin()
        for k in range(args.steps):
            drv.render(frames(args.warmup + k))
    prof = drv.profile_end()
    drv.sync()  # surfaces a traversal-stack overflow, if any

    # exact work of the timed frames (instrumented kernel, untimed), this process's ranks
    tot = {}
    for k in range(args.steps):
        for n, v in drv.counters(frames.copy(args.warmup + k)).items():
            tot[n] = max(tot.get(n, 0), v) if n == "ref_stack_max" else tot.get(n, 0) + v
    if spp > 1:
        # primary segments (samples = 1, no bounce): the same rays every sample of a frame traces first; the render
        # traces them once per pixel and samples 1..spp-1 reuse that record (pt_wavefront.hip wf_shade, pt_device.h)
        sd0 = frames.copy(args.warmup)
        sd0["maxBounceCount"], sd0["samples"] = 0, 1
        cp = drv.counters(sd0)
        tot["reused_primary_lines"] = (spp - 1) * (cp["interior_visits"] + cp["triangle_tests"]) * args.steps
        tot["reused_primary_segments"] = (spp - 1) * cp["segments"] * args.steps
    per_rank = [{"rank": int(r), "block_ms": round(ms / max(1, n), 4), "launches": int(n)}
                for r, (ms, n) in zip(drv.ranks, prof)]
    mine = {"elapsed": elapsed, "tot": tot, "per_rank": per_rank, "devices": [int(c.device) for c in drv.ctxs],
            "gpus": [_gpu_identity(int(c.device)) for c in drv.ctxs],
            "kernel_ms": sum(ms for ms, _ in prof), "launches": sum(n for _, n in prof)}
    allr = coll.gather_obj(json.loads(json.dumps(mine, default=int)))

    verified = None
    if args.verify and got is not None:
        verified = verify_frame(args, topo, scene, W, H, spp, bounces, frames, args.warmup + args.steps, got)

    if rank == 0:
        elapsed_max = max(a["elapsed"] for a in allr)
        T = {}
        for a in allr:
            for n, v in a["tot"].items():
                T[n] = max(T.get(n, 0), v) if n == "ref_stack_max" else T.get(n, 0) + v
        blocks = sorted((b for a in allr for b in a["per_rank"]), key=lambda b: b["rank"])
        # the roofline's kernel time: the slowest rank's average render (with one rank, the render itself)
        avg_kernel_s = max(b["block_ms"] for b in blocks) / 1e3
        ms_per_step = elapsed_max / args.steps * 1e3
        segs_all, prim_all = float(T["segments"]), float(T["pixels"] * spp)
        value = segs_all / elapsed_max / 1e6
        info = drv.info()
        # physical GPUs the ranks ran on, by PCI bus id (device ordinals differ between processes that see different
        # devices; a rehearsal repeats one GPU)
        distinct = len({gp for a in allr for gp in a["gpus"]})
        kind = {"group": "one process, one host thread, all ranks (wcpt_group_create_ex)",
                "ranks": "one process per GPU (wcpt_group_create_rank, ncclCommInitRank; host rendezvous wcpt.rdzv)",
                "torch": f"one process per GPU, torch.distributed {args.dist_backend} gather (rehearsal path)"}
        transport = {0: "rccl", 1: "copy", 2: "direct"}.get(info["transport"], args.dist_backend)
        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": distinct,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (procedural scene generated in-process, no dataset)" if name not in
                    wscene.REFERENCE_SCENES else "the reference's own Init scene (mushroom.obj fixture + 4 spheres)",
            "config": {"workload": desc, "config": args.config, "scene": name, "width": W, "height": H,
                       "spp": spp, "max_bounce": bounces,
                       "frames": ("progressive, renderedFramesCount=warmup.." if args.camera == "still" else
                                  "moving camera (editor strafe + yaw every frame), renderedFramesCount=0"),
                       "camera": args.camera,
                       "kernel": {0: "megakernel", 2: "wavefront"}[args.kernel] +
                                 (" (WCPT_KERNEL_AUTO's choice)" if args.kernel_auto else ""), "bvh": args.bvh,
                       "frame_overlap": {-1: "library default (auto)", 0: "off", 1: "auto", 2: "on"}[args.frame_overlap],
                       "parallelism": ((f"row-stripes of {args.row_stripe} rows x{nranks}" if args.row_stripe else
                                        f"row-block x{nranks}") + f" + {transport} gather of {args.gather} blocks"
                                       + ("" if args.no_overlap else " overlapped with the next frame")
                                       if nranks > 1 else "one device")},
            "ranks": nranks,
            "launch": launch_label(topo["mode"], os.environ),
            "group": {"kind": kind[topo["mode"]], "transport": transport, "rccl_ranks": info["nranks"]
                      if transport == "rccl" else None, "overlap": not args.no_overlap, "devices": topo["devices"]
                      if topo["mode"] == "group" else None},
            "hip_runtime": hip_runtime_label(topo["mode"]),
            "build_id": args.build_id,
            "primary_mrays_per_s": round(prim_all / elapsed_max / 1e6, 3),
            "segments_per_frame": int(segs_all / args.steps),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 4),
            "kernel_launches_per_frame": round(sum(a["launches"] for a in allr) / max(1, len(blocks)) / args.steps, 2),
            "kernel_timing": ("two HIP events on the render stream bracketing the timed renders: launch duration = "
                              "their interval / renders (inter-launch gaps included)" if live_events
                              else "HIP events around each render on each rank's render stream, in an untimed "
                                   "re-render of the timed frames (N > 1: kept out of the timed steps); the slowest "
                                   "rank's average"),
            "ref_stack": {"overflow_segments": T["ref_stack_overflow_segments"], "max": T["ref_stack_max"],
                          "note": "segments of the timed frames that would write past the reference's uint "
                                  "nodeStack[32] (pathTracer.comp:151), and the deepest stack they reach"},
            "roofline": roofline(args, T, avg_kernel_s, ms_per_step / 1e3, devices=distinct, ranks=nranks),
        }
        if nranks > 1:
            out["per_rank_block_ms"] = [b["block_ms"] for b in blocks]
            if topo["mode"] == "group" and transport == "rccl" and distinct > 1:
                out["unrehearsed"] = ("the one-process RCCL group (ncclCommInitAll, every rank issued from one thread) "
                                      "over several GPUs has never run on hardware before this line; the default "
                                      "N-GPU command spawns one process per GPU instead")
            if distinct < nranks:
                out["rehearsal"] = f"{nranks} ranks on {distinct} device(s): not a scaling measurement"
                if args.rccl_rehearsal:
                    out["rehearsal"] += (" (RCCL with a NCCL_HOSTID per rank: ncclCommInitRank, ncclSend / ncclRecv "
                                         "over RCCL's socket transport instead of xGMI)")
        if spp > 1:
            # samples 1..spp-1 shade their primary segment from sample 0's Intersect record (same ray): the reference
            # executes those segments, this implementation does not (pathTracer.comp:309-310)
            executed = segs_all - float(T["reused_primary_segments"])
            out["executed_segments_per_frame"] = int(executed / args.steps)
            out["executed_mrays_per_s"] = round(executed / elapsed_max / 1e6, 3)
            out["value_note"] = ("value counts the reference's segments (Intersect calls of pathTracer.comp); "
                                 "executed_* leaves out the primary segments of samples after the first, which reuse "
                                 "sample 0's record")
        if verified is not None:
            out["verified"] = verified
        if nranks == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, W, H, spp, bounces, budget_s=args.cpu_seconds)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
            if "per_gpu_share" in out["cpu_baseline"]:
                out["speedup_vs_cpu_share"] = round(value / out["cpu_baseline"]["per_gpu_share"]["value"], 1)
        print(json.dumps(out), flush=True)

    drv.close()
    if rdzv is not None:
        rdzv.close()
    if watchdog is not None:
        watchdog.cancel()


def launch_label(mode: str, env) -> str:
    """Which launch produced this line: bench.py's own rank spawner, an external launcher (torchrun), or one process."""
    if mode == "group":
        return "one process (no launcher)"
    if env.get("WCPT_BENCH_LAUNCH") == "spawn":
        return "spawned by bench.py: one fresh process per rank (plain --gpus N, no launcher)"
    return "external launcher (torchrun or equivalent: WORLD_SIZE / RANK / LOCAL_RANK in the environment)"


def hip_runtime_label(mode: str) -> str:
    v = wcpt.runtime_version()
    where = ("the system /opt/rocm runtime (torch not imported)" if mode != "torch" else
             "the HIP runtime torch bundles (torch.distributed is imported first)")
    return f"HIP {v // 10000000}.{(v // 100000) % 100} ({v}), {where}"


if __name__ == "__main__":
    sys.exit(main() or 0)
