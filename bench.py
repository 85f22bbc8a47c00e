"""bench.py — Mray/s + ms/frame of the MI355X path-tracing compute path (BASELINE.json metric).

Default workload (N=1): BASELINE.json configs[1] = Cornell box (34 triangles + 4 spheres), 1920x1080, 1 spp,
maxBounceCount 4, progressive frames (renderedFramesCount = 0, 1, 2, ...). A "step" is one frame: one
wcpt_render over the whole frame (with N ranks: each rank renders its row block, SURVEY.md §8(e), and the
blocks are gathered to rank 0 over RCCL). Rays = ray segments = Intersect() calls, counted exactly by the
instrumented kernel for the very frames that were timed (untimed re-run).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c1|c3|c4|ref] [--no-cpu-baseline]

Prints one JSON line on rank 0.

N = 1 runs on the product's own runtime: torch is NOT imported, libwcpt.so binds the system HIP runtime (/opt/rocm)
exactly as the Jai host would, renders on the context's own stream and is timed with host clocks around
wcpt_sync (the JSON line's "hip_runtime" names the runtime). N > 1 imports torch for torch.distributed (RCCL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

WORLD = int(os.environ.get("WORLD_SIZE", "1"))
if WORLD > 1:
    # torch first: libwcpt.so then binds to the HIP runtime torch already loaded (one runtime per process).
    import torch  # noqa: E402
    import torch.distributed as dist  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd")]

import numpy as np  # noqa: E402
import wcpt  # noqa: E402
from wcpt import scene as wscene  # noqa: E402
from wcpt.dist import assemble, row_block  # noqa: E402

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
BASELINE_METRIC = "Mray/s + ms/frame at 1920\u00d71080 1spp; achieved HBM GB/s vs peak"  # BASELINE.json "metric"
# rays = ray segments (Intersect() calls), counted exactly by the instrumented kernel
# Measured best kernel per workload: the megakernel wins on the coherent, L1-resident
# Cornell box; the wavefront variant wins on the 262k-triangle atrium (incoherent, MALL-resident).
DEFAULT_KERNEL = {"c1": wcpt.KERNEL_MEGAKERNEL, "c2": wcpt.KERNEL_MEGAKERNEL, "c3": wcpt.KERNEL_WAVEFRONT,
                  "c4": wcpt.KERNEL_WAVEFRONT, "ref": wcpt.KERNEL_MEGAKERNEL}
# VALU issue ceiling (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD per 4 cycles at the
# 2.4 GHz peak engine clock (tools/valu_peak.hip measures it: profiles/r03_valu_peak.log)
SIMDS = 1024
CLOCK_GHZ = 2.4
CYCLES_PER_VALU = 2  # a wave64 VALU instruction issues over 2 cycles on the 32-lane SIMD (MI355X_MICROARCH.md)
VALU_PEAK_GINSTR = SIMDS * CLOCK_GHZ / CYCLES_PER_VALU  # spec: 1,228.8 G wave64 VALU instructions/s


def algorithmic_bytes(c: dict) -> int:
    """B_seg = 20*S + sum_draw[32*N_pop + 64*N_interior + 48*N_tri] + 60*[hit] + 28*N_draw,
    plus 164 (SceneData) + 32 (image read-modify-write) per pixel."""
    return (20 * c["sphere_tests"] + 32 * c["node_pops"] + 64 * c["interior_visits"] + 48 * c["triangle_tests"]
            + 60 * c["hits"] + 28 * c["draw_fetches"] + (164 + 32) * c["pixels"])


def _profile_json(path, args):
    """A committed profile summary (profiles/*.json) when it was measured on this config, kernel and tree."""
    if not os.path.exists(path):
        return None
    try:
        pm = json.load(open(path))
    except (OSError, ValueError):
        return None
    if pm.get("config") == args.config and pm.get("kernel") == args.kernel and args.bvh == "midpoint":
        return pm
    return None


def roofline(args, tot, render_s, frame_s) -> dict:
    """The dominant kernel against the ceiling of the resource that binds it, measured per render.

    valu_issue (megakernel; c2): SQ_INSTS_VALU wave-instructions per render from the committed SQ counter pass
      (profiles/sq_<config>.json) over the live render time, against the spec issue rate (1024 SIMDs x 2.4 GHz, one
      wave64 instruction per 2 cycles); measured_ceiling = the rate the kernel's VALU instruction mix could reach
      (profiles/valu_mix_<config>.json x profiles/valu_ceiling.json).
    memory_latency (wavefront trace; c3): dependent scene-line visits (one 64-B child pair per interior visit, one
      triangle record per test) per second of the frame, against the best rate of dependent random line visits the
      cache hierarchy sustains at 8 waves/SIMD (L2-resident chain, tools/gather_bench.hip, profiles/gather_ceiling.json).
    Beside it: the SURVEY 8(d) algorithmic bytes, which price every scene fetch at HBM cost although these scenes are
      served from L1/L2/MALL (so they exceed the HBM peak: "cache-served"), and the HBM bytes the PMC counters measured
      (FETCH_SIZE x 2 + WRITE_SIZE, the gfx950 correction), the only true HBM load."""
    steps = max(1, args.steps)
    alg_bytes = algorithmic_bytes(tot) / steps
    r = {"algorithmic_bytes_per_render": int(alg_bytes),
         "algorithmic_gbs": round(alg_bytes / render_s / 1e9, 1),
         "algorithmic_frac": round(alg_bytes / render_s / 1e9 / HBM_PEAK_GBS, 3),
         "algorithmic_note": "cache-served: SURVEY 8(d) bytes priced at HBM cost; the scene stays in L1/L2/MALL"}
    pm = _profile_json(args.pmc_json or os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json"), args)
    traffic = None if pm is None else pm.get("hbm_bytes_per_launch", pm.get("hbm_bytes_per_frame"))
    r["traffic"] = traffic
    if traffic is not None:
        r["hbm_measured_gbs"] = round(traffic / render_s / 1e9, 2)
        r["hbm_measured_frac"] = round(traffic / render_s / 1e9 / HBM_PEAK_GBS, 4)
    sq = _profile_json(os.path.join(ROOT, "profiles", f"sq_{args.config}.json"), args)
    bound = None if sq is None else sq.get("bound")
    if bound == "valu_issue":
        valu = sq["counters_per_launch"]["SQ_INSTS_VALU"] * sq.get("launches_per_frame", 1.0)
        achieved = valu / render_s / 1e9
        head = {"bound": "valu_issue", "achieved": round(achieved, 1), "peak": VALU_PEAK_GINSTR,
                "unit": "G wave64 VALU instructions/s", "frac": round(achieved / VALU_PEAK_GINSTR, 3),
                "source": f"SQ_INSTS_VALU {valu:.4g}/render ({sq.get('source', 'profiles')}) over the live render "
                          f"time; peak {SIMDS} SIMDs x {CLOCK_GHZ} GHz / {CYCLES_PER_VALU} cycles"}
        ceil = _valu_mix_ceiling(args.config)
        if ceil:
            # what this kernel's VALU mix can reach: each instruction class at the fastest rate measured for an
            # instruction of that class (tools/valu_peak.hip; v_add/v_mul/v_mov issue about twice as fast as v_fma)
            head["measured_ceiling"] = ceil
            head["measured_frac"] = round(achieved / ceil, 3)
    elif bound == "memory_latency":
        ceil = _gather_ceiling()
        # the line visits the kernels execute: with samples > 1 every sample after the first shades its primary
        # segment from sample 0's Intersect record (the same ray), so those traversals are counted by the reference's
        # work (COUNT build) but never run, and are taken out here
        reused = tot.get("reused_primary_lines", 0)
        lines = (tot["interior_visits"] + tot["triangle_tests"] - reused) / steps
        achieved = lines / frame_s / 1e9
        head = {"bound": "memory_latency", "achieved": round(achieved, 2), "peak": ceil,
                "unit": "G dependent line-visits/s", "frac": round(achieved / ceil, 3),
                "source": "interior visits + triangle tests executed per frame over the frame time (the reference's "
                          "counts less the primary traversals of samples after the first, which reuse sample 0's "
                          "record); peak: dependent random 64-B line visits at 8 waves/SIMD from an L2-resident "
                          "table (profiles/gather_ceiling.json)"}
        if reused:
            head["reused_primary_lines_per_frame"] = int(reused / steps)
    else:
        head = {"bound": "unprofiled", "achieved": None, "peak": None, "unit": None, "frac": None,
                "source": f"no SQ counter pass committed for {args.config} (profiles/sq_{args.config}.json)"}
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


def _valu_mix_ceiling(config: str):
    """Mix-weighted VALU ceiling (G wave64 instructions/s) of the config's dominant kernel: 1 / sum(f_c / R_c) over the
    instruction classes c of profiles/valu_mix_<config>.json (fractions f_c of SQ_INSTS_VALU) with the class rates R_c
    of profiles/valu_ceiling.json."""
    try:
        rates = json.load(open(os.path.join(ROOT, "profiles", "valu_ceiling.json")))["class_gwave_instr_per_s"]
        mix = json.load(open(os.path.join(ROOT, "profiles", f"valu_mix_{config}.json")))["class_fraction"]
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


def cpu_baseline(scene, width, height, spp, bounces, budget_s=20.0, min_frames=5):
    """The CPU oracle (a scalar C restatement of pathTracer.comp, oracle/pt_oracle.c, built -O3 -march=native on this
    host) on 16 host cores (the GPU box's share per GPU). Full frames of the same workload (progressive frame numbers
    0, 1, ...), median of >= min_frames (BASELINE.md:21), when min_frames frames fit in ~budget_s; otherwise (c4:
    ~minutes per 4K 16-spp frame) a bounded sample of 32-row bands spread over the frame, until ~budget_s."""
    lib, flags = _native_oracle()
    os.environ["WCPT_ORACLE_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure, used here only as the reported CPU baseline
    threads = max(1, min(16, os.cpu_count() or 1))
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
    where = f"{_cpu_model()}, {threads} threads, oracle/pt_oracle.c built {flags} (lavapipe is not available)"
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
        return {"value": round(rates[med], 4), "unit": "Mray/s", "cores": threads, "kind": "port",
                "frame_ms_median": round(times[med] * 1e3, 2),
                "sample": f"median of {f} full {width}x{height} frames (progressive frames 0..{f - 1}, {segs} "
                          f"segments, {sum(times):.1f} s) on {where}"}
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
    return {"value": round(seg / t_total / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "sample": f"{bands} bands of <= {band} rows ({px} px, {seg} segments) of the same {width}x{height} "
                      f"workload (a full frame would take ~{est_frame:.0f} s) over {frame + 1} progressive frame(s), "
                      f"{t_total:.1f} s on {where}"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--settle-ms", type=float, default=200.0,
                    help="untimed renders of frame 0 for this long before the warmup steps, so that the timed steps "
                         "do not run while the GPU clocks ramp up (measured: 3 warmup frames of c2 leave the timed "
                         "region ~9%% slow); frame 0 overwrites the image, so the timed frames are unchanged")
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--kernel", type=int, default=-1,
                    help="0 megakernel, 2 wavefront, -1 per-config default (DEFAULT_KERNEL)")
    ap.add_argument("--wf-pipes", type=int, default=0,
                    help="wavefront kernel: concurrent pipelines (WCPT_OPTION_WF_PIPES; 0 = the library default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--pmc-json", default=None,
                    help="PMC HBM-traffic summary for roofline.traffic (default profiles/pmc_traffic_<config>.json, "
                         "written by tools/pmc_summary.py)")
    ap.add_argument("--bvh", default="midpoint", choices=["midpoint", "sah"],
                    help="BVH builder: the reference's midpoint split (default: the benchmarked workload) or the "
                         "optional binned SAH (a different tree, reported as a separate workload)")
    ap.add_argument("--gather", default="rgb", choices=["rgb", "rgba", "display"],
                    help="N>1 wire format of the row blocks: rgb (default; alpha is always 1.0 and is restored on "
                         "rank 0, bit-identical frame, 12 B/px), the full rgba32f block (16 B/px), or display: "
                         "composite.comp's RGBA8 display value written by the render itself "
                         "(WCPT_PAYLOAD_DISPLAY_RGBA8, 4 B/px; what rank 0 presents, not the accumulation)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="N>1: gather each frame on the render stream instead of overlapping it with the next render")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 re-renders the timed frame sequence on the full frame and checks the gathered "
                         "row blocks against it bit-for-bit (adds 'verified' to the JSON line)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo", "gloo-host"],
                    help="nccl (= RCCL over xGMI, the product path); gloo (device tensors) or gloo-host (host-staged) "
                         "rehearse N>1 ranks on one GPU, where RCCL refuses duplicate devices")
    args = ap.parse_args()


    world = WORLD
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    name, W, H, spp, bounces, desc = CONFIGS[args.config]
    if args.kernel < 0:
        args.kernel = DEFAULT_KERNEL[args.config]
    scene = wscene.generate(name, bvh=args.bvh)
    y0, rows = row_block(H, world, rank)
    overlap = world > 1 and not args.no_overlap
    host_staged = world > 1 and args.dist_backend == "gloo-host"
    # Per-step host work is kept small (at 8 ranks a c2 row block renders in ~0.1 ms): the camera is static, so
    # SceneData is built once and only renderedFramesCount changes per frame (PathTracingRenderer.jai:423).
    sd = scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=0)

    if world == 1:
        # The product's runtime: no torch in the process, so libwcpt.so binds /opt/rocm's HIP runtime as a Jai host
        # would; the context renders on its own stream into its own image (wcpt_create_screen), timed by host clocks
        # around wcpt_sync (which waits for that stream).
        device = local % max(1, wcpt.device_count())
        ctx = wcpt.Context(device)
        ctx.set_kernel(args.kernel)
        if args.wf_pipes:
            ctx.set_option(wcpt._lib.OPTION_WF_PIPES, args.wf_pipes)
        dev = wcpt.DeviceScene(ctx, scene)
        ctx.create_screen(W, H)
        addrs = dev.addresses()

        def step(frame):
            sd["renderedFramesCount"] = frame
            ctx.render(sd, *addrs)

        def sync():
            ctx.sync()

        def barrier():
            pass
    else:
        device = local % max(1, torch.cuda.device_count())  # == local on a node with >= N GPUs
        torch.cuda.set_device(device)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group("gloo")
        # One explicit stream for everything: the renders (wcpt), the payload hand-off and the collective. Torch's
        # default current stream is the legacy null stream (handle 0), which wcpt_set_stream takes as "use the
        # context's own stream" -- that would leave the gather unordered with the render.
        stream = torch.cuda.Stream(device=device)
        torch.cuda.set_stream(stream)
        ctx = wcpt.Context(device)
        ctx.set_stream(stream.cuda_stream)
        ctx.set_kernel(args.kernel)
        if args.wf_pipes:
            ctx.set_option(wcpt._lib.OPTION_WF_PIPES, args.wf_pipes)
        dev = wcpt.DeviceScene(ctx, scene)
        ctx.create_screen(W, H)
        ctx.set_row_range(y0, rows)
        addrs = dev.addresses()
        max_rows = -(-H // world)
        shard = torch.zeros((max_rows, W, 4), dtype=torch.float32, device="cuda")
        ctx.set_external_image(shard.data_ptr(), shard.numel() * 4)
        # payload format code of wcpt_set_gather_output: 3 / 4 float channels, or 8 = WCPT_PAYLOAD_DISPLAY_RGBA8
        channels = {"rgb": 3, "rgba": 4, "display": 8}[args.gather]
        pdt, pch = (torch.uint8, 4) if args.gather == "display" else (torch.float32, channels)
        # The gather payload is written by the render itself (wcpt_set_gather_output): each frame's kernel stores the
        # rank's row block as RGB (alpha is always 1.0 and is restored on rank 0) or RGBA into one of the payload
        # buffers, so no copy kernel runs between the render and the collective. Overlap: frame k's payload is
        # gathered on a separate communication stream while frame k+1 renders into another buffer. Every frame is
        # still rendered and gathered; the timed region ends with a device-wide synchronize that includes the last
        # gather. Three payload buffers, and the host (which runs frames ahead of the GPU) waits for a buffer's
        # previous gather before the render that rewrites it: measured ~6 us/frame cheaper at 8 ranks than a
        # render-stream wait on that event.
        nbuf = 3 if overlap else 1
        comm = torch.cuda.Stream(device=device) if overlap else None
        payload = [torch.empty((max_rows, W, pch), dtype=pdt, device="cuda") for _ in range(nbuf)]
        gathered = [[torch.empty(payload[0].shape, dtype=pdt, device="cpu" if host_staged else "cuda")
                     for _ in range(world)] for _ in range(nbuf)] if rank == 0 else None
        last = {"buf": 0}
        ready_ev = [torch.cuda.Event() for _ in range(nbuf)]   # payload[i] holds frame k's block
        done_ev = [torch.cuda.Event() for _ in range(nbuf)]    # the gather that last read payload[i] has finished
        done_used = [False] * nbuf

        def step(frame):
            sd["renderedFramesCount"] = frame
            i = frame % nbuf
            last["buf"] = i
            out = gathered[i] if rank == 0 else None
            if overlap and done_used[i]:
                done_ev[i].synchronize()                    # payload[i]'s gather (frame k-3) has finished
            ctx.set_gather_output(payload[i].data_ptr(), payload[i].numel() * payload[i].element_size(), channels)
            ctx.render(sd, *addrs)
            if not overlap:
                dist.gather(payload[i].cpu() if host_staged else payload[i], out, dst=0)
                return
            ready_ev[i].record(stream)
            with torch.cuda.stream(comm):
                comm.wait_event(ready_ev[i])
                dist.gather(payload[i].cpu() if host_staged else payload[i], out, dst=0)
                done_ev[i].record(comm)
            done_used[i] = True

        def sync():
            torch.cuda.synchronize()

        def barrier():
            dist.barrier()

    t_settle = time.perf_counter()
    while (time.perf_counter() - t_settle) * 1e3 < args.settle_ms:
        sd["renderedFramesCount"] = 0
        for _ in range(8):
            ctx.render(sd, *addrs)
        sync()
    for f in range(args.warmup):
        step(f)
    sync()
    barrier()
    sync()
    # Kernel time for the roofline: HIP events around every launch on the render stream. At N = 1 they run inside
    # the timed region (~1 % of a c2 frame). At N > 1 they are left out of it -- with the gather hand-off they cost
    # ~16 us of a ~84 us 135-row step (tools/host_step_probe.py --profile) -- and the same frames are re-rendered
    # afterwards, untimed, with the events on.
    live_events = world == 1
    if live_events:
        ctx.profile_begin()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if not live_events:
        ctx.set_gather_output(0, 0)
        ctx.profile_begin()
        for k in range(args.steps):
            sd["renderedFramesCount"] = args.warmup + k
            ctx.render(sd, *addrs)
    kernel_ms, launches = ctx.profile_end()
    ctx.sync()  # surfaces a traversal-stack overflow, if any

    # exact work of the timed frames (instrumented kernel, untimed)
    tot = {k: 0 for k in wcpt.COUNTER_FIELDS}
    for k in range(args.steps):
        sdk = scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=args.warmup + k)
        c = ctx.render_counters(sdk, *addrs)
        for n in tot:
            tot[n] = max(tot[n], c[n]) if n == "ref_stack_max" else tot[n] + c[n]
    if spp > 1:
        # primary segments (samples = 1, no bounce): the same rays every sample of a frame traces first; the render
        # traces them once per pixel and samples 1..spp-1 reuse that record (pt_wavefront.hip wf_shade, pt_device.h)
        cp = ctx.render_counters(scene.scene_data(W, H, max_bounce=0, samples=1, frame=args.warmup), *addrs)
        tot["reused_primary_lines"] = (spp - 1) * (cp["interior_visits"] + cp["triangle_tests"]) * args.steps
    if world > 1:
        t = torch.tensor([elapsed, float(tot["segments"]), float(tot["pixels"] * spp)], dtype=torch.float64,
                         device="cpu" if host_staged else "cuda")
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed_max, segs_all, prim_all = float(tmax[0]), float(tsum[0]), float(tsum[1])
    else:
        elapsed_max, segs_all, prim_all = elapsed, float(tot["segments"]), float(tot["pixels"] * spp)

    verified = None
    if args.verify and rank == 0:
        if world > 1:
            frame_img = assemble([g.to("cpu") for g in gathered[last["buf"]]], H, world).numpy()
        else:
            frame_img = ctx.readback(H)
        with wcpt.Context(device) as vctx:
            vdev = wcpt.DeviceScene(vctx, scene)
            vctx.set_kernel(args.kernel)
            vctx.create_screen(W, H)
            for f in range(args.warmup + args.steps):
                vctx.render(scene.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f), *vdev.addresses())
            if world > 1 and args.gather == "display":
                disp = torch.empty((H, W, 4), dtype=torch.uint8, device="cuda")
                vctx.composite(disp.data_ptr(), rgba8=True)
                vctx.sync()
                ref = disp.cpu().numpy()
            else:
                ref = vctx.readback()
            vdev.free()
        bits = np.uint8 if ref.dtype == np.uint8 else np.uint32  # display bytes, or the float image's bit patterns
        same = frame_img.view(bits) == ref.view(bits)
        verified = bool(same.all())
        if not verified:
            bad_rows = np.nonzero(~same.all(axis=(1, 2)))[0]
            print(f"verify: {bad_rows.size} of {H} rows differ (first {bad_rows[:8].tolist()}, "
                  f"last {bad_rows[-4:].tolist()}); pixel fraction {1.0 - same.all(axis=2).mean():.4f}",
                  file=sys.stderr, flush=True)
            if os.environ.get("WCPT_VERIFY_DUMP"):
                np.savez(os.environ["WCPT_VERIFY_DUMP"], got=frame_img, ref=ref)

    if rank == 0:
        ms_per_step = elapsed_max / args.steps * 1e3
        value = segs_all / elapsed_max / 1e6
        avg_kernel_s = kernel_ms / max(1, launches) / 1e3
        out = {
            "metric": BASELINE_METRIC,
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
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
                       "spp": spp, "max_bounce": bounces, "frames": "progressive, renderedFramesCount=warmup..",
                       "kernel": {0: "megakernel", 2: "wavefront"}[args.kernel], "bvh": args.bvh,
                       "parallelism": f"row-block x{world}" + ((" + RCCL gather" if args.dist_backend == "nccl"
                                                               else f" + {args.dist_backend} gather (rehearsal)")
                                                              + f" of {args.gather} blocks"
                                                              + (" overlapped with the next frame" if overlap else "")
                                                              if world > 1 else "")},
            "hip_runtime": hip_runtime_label(world),
            "primary_mrays_per_s": round(prim_all / elapsed_max / 1e6, 3),
            "segments_per_frame": int(segs_all / args.steps),
            "kernel_ms_avg": round(avg_kernel_s * 1e3, 4),
            "kernel_launches_per_frame": round(launches / args.steps, 2),
            "kernel_timing": ("HIP events around each launch on the render stream, in the timed region" if live_events
                              else "HIP events around each launch on the render stream, in an untimed re-render of "
                                   "the timed frames (N > 1: kept out of the timed steps)"),
            "ref_stack": {"overflow_segments": tot["ref_stack_overflow_segments"], "max": tot["ref_stack_max"],
                          "note": "segments of the timed frames (this rank) that would write past the reference's "
                                  "uint nodeStack[32] (pathTracer.comp:151), and the deepest stack they reach"},
            "roofline": roofline(args, tot, avg_kernel_s, ms_per_step / 1e3),
        }
        if verified is not None:
            out["verified"] = verified
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(scene, W, H, spp, bounces, budget_s=args.cpu_seconds)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 1)
        print(json.dumps(out), flush=True)

    if world > 1:
        ctx.set_gather_output(0, 0)
        ctx.set_external_image(0, 0)
    dev.free()
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def hip_runtime_label(world: int) -> str:
    v = wcpt.runtime_version()
    where = ("system /opt/rocm runtime (torch not imported)" if world == 1 else
             "the HIP runtime torch bundles (torch.distributed is imported first)")
    return f"HIP {v // 10000000}.{(v // 100000) % 100} ({v}), {where}"


if __name__ == "__main__":
    main()
