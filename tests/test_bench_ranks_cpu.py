"""bench.py's one-process-per-GPU mode (what the driver's torchrun scaling run executes) end to end on CPU: two
processes with torchrun's environment run bench.main() against a stand-in for the wcpt device API, so the host plumbing
-- rendezvous, the RCCL id handed from rank 0 to every rank, barriers, per-rank work and block times gathered to rank 0,
the max-over-ranks time and the one JSON line -- is exercised without a GPU. The device side of the same calls is
covered by tests/test_gpu_multi.py (the group itself) and can only run with RCCL on a multi-GPU node."""
import json
import multiprocessing as mproc
import os
import socket
import time
import sys
import types

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UID = bytes((7 * i) % 256 for i in range(128))


def _fake_wcpt(rank, nranks, log, one_visible=False, slow_ranks=False):
    """The slice of the wcpt package bench.py uses in its group modes, recording what it was asked to do.
    one_visible: the launcher shows each process only its own GPU (device 0 everywhere, distinct PCI ids)."""
    import wcpt._lib as L
    from wcpt import scene as real_scene

    class Ctx:
        def __init__(self, rows):
            self.rows, self.prof, self.device = rows, [], 0 if one_visible else rank

        def set_kernel(self, k):
            log.append(("kernel", k))

        def set_option(self, o, v):
            pass

        def profile_begin(self):
            self.prof = []

        def profile_end(self):
            return 0.1 * len(self.prof) * (1 + rank), len(self.prof)

        def render_counters(self, sd, *a):
            c = {k: 0 for k in L.COUNTER_FIELDS}
            c.update(pixels=self.rows * 8, segments=self.rows * 8 * 3, interior_visits=5, triangle_tests=7)
            return c

        def readback(self, rows=None):
            return np.zeros((rows or self.rows, 8, 4), np.float32)

        def buffer_alloc(self, n):
            log.append(("output", n))
            return 1

        def buffer_address(self, b):
            return 4096

        def buffer_free(self, b):
            pass

    class Group:
        def __init__(self, ctx, r):
            self.ctx, self.ranks, self.contexts, self.frames = ctx, [r], [ctx], 0
            self.h = self

        @classmethod
        def rank(cls, device, n, r, root=0, uid=None):
            assert (device, n, r, root) == (0 if one_visible else rank, nranks, rank, 0)
            assert uid == UID, "the RCCL id must reach every rank unchanged"
            log.append(("group", device, n, r))
            return cls(Ctx(5 if r == 0 else 4), r)

        def context(self, r):
            return self.ctx if r in self.ranks else None

        def set_option(self, o, v):
            log.append(("overlap", v))

        def create_screen(self, W, H):
            log.append(("screen", W, H))

        def set_output(self, fmt, dst, n):
            assert fmt == 0 or n > 0, "every process passes the output's byte count (wcpt.h wcpt_group_set_output)"
            log.append(("set_output", fmt, dst != 0))

        def render(self, sd, m, s, d):
            assert len(m) == len(s) == len(d) == 1
            self.ctx.prof.append(1)
            self.frames += 1
            if slow_ranks:
                time.sleep(0.0005 * rank)   # the ranks' clocks see different frame times
            return 0

        def sync(self):
            pass

        def info(self):
            return {"nranks": nranks, "local_ranks": 1, "first_local_rank": rank, "root": 0, "transport": 0,
                    "overlap": 1, "distinct_devices": 1, "broken": 0, "frames": self.frames}

        def close(self):
            log.append(("closed",))
            log.append(("frames", self.frames))

    class DeviceScene:
        def __init__(self, ctx, scene):
            pass

        def addresses(self):
            return 1, 2, 3

        def free(self):
            pass

    m = types.ModuleType("wcpt")
    m.__path__ = []
    m._lib, m.scene, m.Group, m.DeviceScene = L, real_scene, Group, DeviceScene
    m.group_unique_id = lambda: UID
    m.runtime_version = lambda: 70226015
    m.build_id = lambda: "stand-in"
    m.KERNEL_AUTO = L.KERNEL_AUTO
    # torchrun: every process sees every GPU, so LOCAL_RANK is the device; one_visible: each sees one, its own
    m.device_count = lambda: 1 if one_visible else nranks
    m.device_pci_bus_id = lambda d: f"0000:{0x11 + 0x20 * (rank if one_visible else d):02x}:00.0"
    # bench.py calls wcpt_group_render through the library with prebuilt arrays: route it to the stand-in group
    m.lib = types.SimpleNamespace(wcpt_group_render=lambda h, sd, mm, ss, dd: h.render(sd, list(mm), list(ss), list(dd)))
    m.SCENE_DATA_DTYPE = L.SCENE_DATA_DTYPE
    return m


def _rank_main(rank, world, port, out_dir, one_visible=False, settle_ms=0):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "wc-path-tracer_amd")]
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port - 1))
    import wcpt  # noqa: F401  (the real package: its scene module builds the Cornell box on the host)
    import wcpt.rdzv  # noqa: F401  (the real rendezvous, which stays registered under its name)
    log = []
    sys.modules["wcpt"] = _fake_wcpt(rank, world, log, one_visible, slow_ranks=settle_ms > 0)
    import bench
    out = open(os.path.join(out_dir, f"rank{rank}.out"), "w")
    sys.stdout = out
    bench.main(["--gpus", str(world), "--config", "c1", "--steps", "3", "--warmup", "2", "--settle-ms", str(settle_ms),
                "--no-cpu-baseline"])
    out.close()
    json.dump([list(x) for x in log], open(os.path.join(out_dir, f"rank{rank}.log"), "w"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,one_visible", [(2, False), (3, False), (3, True)])
def test_bench_one_process_per_gpu_plumbing(tmp_path, world, one_visible):
    """one_visible: a launcher that shows each process only its GPU -- LOCAL_RANK folds onto device 0, and n_gpus still
    counts the distinct GPUs (by PCI bus id), not the ordinals the processes see."""
    ctx = mproc.get_context("spawn")
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, str(tmp_path), one_visible)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    lines = [ln for ln in open(tmp_path / "rank0.out").read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    for r in range(1, world):
        assert not open(tmp_path / f"rank{r}.out").read().strip()      # one JSON line, from rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["ranks"] == world and d["steps"] == 3
    assert d["group"]["transport"] == "rccl" and d["group"]["rccl_ranks"] == world
    assert d["group"]["kind"].startswith("one process per GPU")
    assert d["launch"].startswith("external launcher")          # torchrun's environment, not bench.py's spawner
    assert "torch not imported" in d["hip_runtime"]
    # per-rank render times gathered in rank order (the stand-in's rank r takes 0.1 * (1 + r) ms per render); the
    # roofline's kernel time is the slowest rank's
    assert d["per_rank_block_ms"] == [pytest.approx(0.1 * (1 + r)) for r in range(world)]
    assert d["kernel_ms_avg"] == pytest.approx(0.1 * world)
    # the work of all ranks: rank 0 holds 5 rows, the others 4 (stand-in), 24 segments per row, 3 timed frames
    assert d["segments_per_frame"] == 24 * (5 + 4 * (world - 1))
    assert d["value"] > 0 and d["ms_per_step"] > 0
    logs = [json.load(open(tmp_path / f"rank{r}.log")) for r in range(world)]
    for r, log in enumerate(logs):
        assert ["group", 0 if one_visible else r, world, r] in log and ["closed"] in log
        assert ["set_output", 3, r == 0] in log                      # rgb payloads; only the root names a frame
        assert (["output", 256 * 256 * 12] in log) == (r == 0)         # c1: 256x256, rgb 12 B/px, on the root
        assert ["set_output", 0, False] in log                         # presenting off for the untimed re-render


def test_settle_phase_runs_the_same_frames_on_every_rank(tmp_path):
    """The untimed settle phase lasts --settle-ms by a clock; each of its frames posts an exchange, so a rank that
    rendered one batch more than the root would wait for a receive that never comes (a 4-rank RCCL rehearsal hung this
    way). Rank 0's clock decides for all: with ranks whose frames take different times, every rank renders the same
    number of frames."""
    ctx = mproc.get_context("spawn")
    port = _free_port()
    world = 3
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, str(tmp_path), False, 40)) for r in range(world)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
        assert p.exitcode == 0
    counts = [[x[1] for x in json.load(open(tmp_path / f"rank{r}.log")) if x[0] == "frames"][0] for r in range(world)]
    assert len(set(counts)) == 1 and counts[0] > 2 + 3, counts


# ---- plain `python bench.py --gpus N` (no launcher): bench.py spawns the rank processes itself ----
def test_launch_plan_picks_the_spawner_for_plain_multi_gpu_runs():
    import bench
    p = lambda argv, env=None: bench.launch_plan(bench.parse_args(argv), env or {})  # noqa: E731
    assert p([]) == "group" and p(["--gpus", "1"]) == "group"
    assert p(["--gpus", "8"]) == "spawn" and p(["--gpus", "2", "--rccl-rehearsal"]) == "spawn"
    assert p(["--gpus", "8", "--one-process"]) == "group"                      # explicit, labelled "unrehearsed"
    assert p(["--gpus", "3", "--transport", "copy", "--devices", "0,0,0"]) == "group"
    assert p(["--gpus", "4", "--transport", "direct"]) == "group"
    assert p(["--gpus", "4"], {"WORLD_SIZE": "4"}) == "ranks"                   # under torchrun: this is one rank


def test_main_spawns_before_touching_the_gpu(monkeypatch):
    """main() hands a plain N-GPU run to spawn_ranks before importing wcpt (no HIP call, no device query in the
    parent), with the argv unchanged, and returns the ranks' status."""
    import bench
    seen = {}

    def fake_spawn(argv, n, **kw):
        seen.update(argv=list(argv), n=n, wcpt_loaded=bench.wcpt is not None)
        return 5

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "wcpt", None)
    monkeypatch.setattr(bench, "spawn_ranks", fake_spawn)
    argv = ["--gpus", "4", "--config", "c1", "--steps", "3"]
    assert bench.main(argv) == 5
    assert seen == {"argv": argv, "n": 4, "wcpt_loaded": False}


def _spawn(tmp_path, world, extra_env=None, argv=None):
    import bench
    env = dict(os.environ, WCPT_TEST_OUT=str(tmp_path), **(extra_env or {}))
    env.pop("WORLD_SIZE", None)
    argv = argv or ["--gpus", str(world), "--config", "c1", "--steps", "3", "--warmup", "2", "--settle-ms", "0",
                    "--no-cpu-baseline"]
    child = [sys.executable, os.path.join(ROOT, "tests", "bench_spawn_child.py")]
    t0 = time.monotonic()
    rc = bench.spawn_ranks(argv, world, env=env, child_cmd=child, timeout_s=240)
    return rc, time.monotonic() - t0


@pytest.mark.parametrize("world", [2, 4])
def test_spawned_ranks_run_the_one_process_per_gpu_path(tmp_path, capfd, world):
    rc, _ = _spawn(tmp_path, world)
    out = capfd.readouterr().out
    assert rc == 0
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1                                   # one JSON line, rank 0's, on the spawner's stdout
    d = json.loads(lines[0])
    assert d["ranks"] == world and d["n_gpus"] == world
    assert d["launch"].startswith("spawned by bench.py")
    assert d["group"]["kind"].startswith("one process per GPU") and d["group"]["transport"] == "rccl"
    runs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]
    ids = {r["env"]["TORCHELASTIC_RUN_ID"] for r in runs}
    ports = {r["env"]["MASTER_PORT"] for r in runs}
    assert len(ids) == 1 and len(ports) == 1                 # one job: one rendezvous token and port for all ranks
    for r, run in enumerate(runs):
        e = run["env"]
        assert (e["RANK"], e["LOCAL_RANK"], e["WORLD_SIZE"], e["LOCAL_WORLD_SIZE"]) == (str(r), str(r), str(world),
                                                                                        str(world))
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["WCPT_BENCH_LAUNCH"] == "spawn"
        assert ["group", r, world, r] in run["log"] and ["closed"] in run["log"]
        assert not run["torch"]


def test_a_failing_rank_stops_the_others(tmp_path, capfd):
    """Rank 1 exits 7 before the rendezvous; the others would wait for it (up to the rendezvous timeout). The spawner
    stops them at once and returns rank 1's status."""
    rc, dt = _spawn(tmp_path, 3, extra_env={"WCPT_TEST_FAIL_RANK": "1"})
    err = capfd.readouterr().err
    assert rc == 7 and dt < 60
    assert "rank 1 exited with 7" in err


@pytest.mark.parametrize("how", ["sigterm", "sigkill"])
def test_spawner_sigterm_stops_the_ranks(tmp_path, how):
    """A launcher's SIGTERM to the spawner (or its death) must not leave rank processes holding GPUs: the spawner stops
    its ranks on SIGTERM and exits 128 + 15; each rank also has PR_SET_PDEATHSIG, so it dies with the spawner."""
    import signal
    import subprocess
    pid_dir = tmp_path / "pids"
    pid_dir.mkdir()
    rank = tmp_path / "rank.py"
    rank.write_text("import os, sys, time\nopen(os.path.join(sys.argv[1], str(os.getpid())), 'w').close()\n"
                    "time.sleep(300)\n")
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks([%r], 2, child_cmd=[sys.executable, %r]))") % (ROOT, str(pid_dir), str(rank))
    p = subprocess.Popen([sys.executable, "-c", code])
    t0 = time.monotonic()
    while len(os.listdir(pid_dir)) < 2 and time.monotonic() - t0 < 30:
        time.sleep(0.05)
    pids = [int(x) for x in os.listdir(pid_dir)]
    assert len(pids) == 2
    if how == "sigterm":
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=30) == 128 + signal.SIGTERM
    else:                      # the spawner dies without a word: PR_SET_PDEATHSIG takes its ranks with it
        p.kill()
        p.wait(timeout=30)
    for pid in pids:
        for _ in range(200):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                break
            time.sleep(0.05)
        else:
            raise AssertionError(f"rank {pid} still running")
