"""bench.py's host logic on CPU: which ranks a launch drives (--gpus against WORLD_SIZE, --devices, transports), the
moving-camera frame sequence, and the torch-free rendezvous the one-process-per-GPU mode uses.
The GPU side of the same paths is tests/test_gpu_multi.py."""
import argparse
import multiprocessing as mproc
import os
import socket
import time
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from wcpt.rdzv import Rendezvous  # noqa: E402


def _topo(argv, env=None):
    return bench.resolve_topology(bench.parse_args(argv), env or {})


def test_gpus_flag_drives_a_one_process_group():
    t = _topo([])
    assert t == {"mode": "group", "nranks": 1, "rank": 0, "local_rank": 0, "devices": [0]}
    t = _topo(["--gpus", "8"])
    assert t["mode"] == "group" and t["nranks"] == 8 and t["devices"] == list(range(8))
    t = _topo(["--gpus", "4", "--devices", "0,0,0,0", "--transport", "copy"])
    assert t["devices"] == [0, 0, 0, 0]
    with pytest.raises(SystemExit):
        _topo(["--gpus", "4", "--devices", "0,0,0,0"])            # RCCL: one rank per device
    with pytest.raises(SystemExit):
        _topo(["--gpus", "3", "--devices", "0,1"])                # a device per rank
    with pytest.raises(SystemExit):
        _topo(["--gpus", "0"])
    with pytest.raises(SystemExit):
        _topo(["--dist-backend", "gloo"])                          # torch.distributed needs a launcher


def test_under_torchrun_gpus_must_equal_world_size():
    env = {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "29500"}
    t = _topo(["--gpus", "4"], env)
    assert t == {"mode": "ranks", "nranks": 4, "rank": 2, "local_rank": 2, "devices": [2]}
    assert _topo([], env)["mode"] == "ranks"                       # --gpus omitted: WORLD_SIZE decides
    assert _topo(["--dist-backend", "gloo"], env)["mode"] == "torch"
    with pytest.raises(SystemExit):
        _topo(["--gpus", "8"], env)                                # the driver's N and the launcher's must agree
    with pytest.raises(SystemExit):
        _topo(["--gpus", "4", "--devices", "0,1,2,3"], env)


def test_main_refuses_a_mismatched_launch_before_touching_a_device(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    with pytest.raises(SystemExit):
        bench.main(["--gpus", "1"])


def test_orbit_frames_move_the_camera_and_restart_accumulation():
    import wcpt
    from wcpt import scene as wscene
    s = wscene.generate("cornell")
    fs = bench.FrameSource(s, 64, 36, 4, 1, "orbit", 5)
    sds = [fs.copy(k) for k in range(5)]
    assert all(int(sd["renderedFramesCount"]) == 0 for sd in sds)   # editor.jai:149-150 while moving
    pos = np.array([sd["position"] for sd in sds])
    step = np.linalg.norm(np.diff(pos, axis=0), axis=1)
    assert np.allclose(step, 4.0 * bench.ORBIT_DT, rtol=1e-4)       # MovementSpeed = 4 * deltaTime (editor.jai:91)
    assert not np.array_equal(sds[0]["inverseView"], sds[1]["inverseView"])
    cam = bench.orbit_camera(s.camera, 3)
    assert cam.yaw == pytest.approx(s.camera.yaw - 3 * bench.ORBIT_YAW_DEG)
    # back and forth: the camera stays within one half period's travel of where it started
    far = max(np.linalg.norm(np.array(bench.orbit_camera(s.camera, k).position) - np.array(s.camera.position))
              for k in range(0, 200, 5))
    assert far <= bench.ORBIT_HALF_PERIOD * 4.0 * bench.ORBIT_DT * 1.01   # (float32 positions drift slightly)
    still = bench.FrameSource(s, 64, 36, 4, 1, "still", 5)
    assert [int(still.copy(k)["renderedFramesCount"]) for k in range(4)] == [0, 1, 2, 3]
    assert np.array_equal(still.copy(3)["position"], sds[0]["position"])
    assert wcpt.SCENE_DATA_DTYPE == sds[0].dtype


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rdzv_worker(rank, world, port, q):
    with Rendezvous(rank, world, "127.0.0.1", port, timeout=60) as rz:
        uid = rz.broadcast(bytes(range(128)) if rank == 0 else None)
        rz.barrier()
        got = rz.gather_obj({"rank": rank, "elapsed": 0.5 + rank})
        every = rz.allgather_obj(rank * rank)
        q.put((rank, uid, got, every))


@pytest.mark.parametrize("world", [2, 3])
def test_rendezvous_broadcast_gather_barrier(world):
    """The host exchanges of the one-process-per-GPU bench: the root's 128-byte RCCL id reaches every rank, per-rank
    objects gather to rank 0 in rank order (the max-over-ranks time is taken from them), barriers return."""
    ctx = mproc.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rdzv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, uid, got, every = q.get(timeout=60)
        res[r] = (uid, got, every)
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):
        uid, got, every = res[r]
        assert uid == bytes(range(128))
        assert every == [k * k for k in range(world)]
        assert (got is None) == (r != 0)
    assert [g["rank"] for g in res[0][1]] == list(range(world))
    assert max(g["elapsed"] for g in res[0][1]) == 0.5 + world - 1


def test_rendezvous_from_env_uses_master_port_plus_one(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("MASTER_PORT", "29500")
    rz = Rendezvous.from_env()
    assert rz.world == 1 and rz.broadcast(b"x") == b"x" and rz.gather(b"y") == [b"y"]
    rz.barrier()
    with pytest.raises(ValueError):
        Rendezvous(2, 2)
    assert isinstance(bench.parse_args([]), argparse.Namespace)


def test_rendezvous_skips_a_busy_port_and_a_foreign_listener():
    """The hub's first port is taken by an unrelated listener (which accepts and never answers): the hub binds the next
    free port, clients skip the silent one after their handshake times out, and the exchange works."""
    port = _free_port()
    squat = socket.socket()
    squat.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    squat.bind(("127.0.0.1", port))
    squat.listen(8)
    try:
        ctx = mproc.get_context("spawn")
        q = ctx.Queue()
        ps = [ctx.Process(target=_rdzv_worker, args=(r, 2, port, q)) for r in range(2)]
        for p in ps:
            p.start()
        got = dict(q.get(timeout=60)[:2] for _ in range(2))
        for p in ps:
            p.join(timeout=30)
            assert p.exitcode == 0
        assert got[0] == got[1] == bytes(range(128))
    finally:
        squat.close()


def _abandoning_client(port):
    """A client of rank 1 that sends its hello and closes before the hub answers (it gave up waiting)."""
    import hashlib
    import struct
    from wcpt import rdzv
    tok = hashlib.sha256(b"").digest()[:16]
    deadline = time.monotonic() + 30
    while time.monotonic() < deadline:
        try:
            c = socket.create_connection(("127.0.0.1", port), timeout=1.0)
        except OSError:
            time.sleep(0.02)
            continue
        c.sendall(rdzv.MAGIC_CLIENT + tok + struct.pack("<I", 1))
        c.close()
        return
    raise AssertionError("no hub")


def test_rendezvous_ignores_a_client_that_gave_up():
    """a client that sent its hello and closed before the hub answered must not be registered in place of
    its own retry (the hub registers a client only after the client acknowledges the hub's answer)."""
    port = _free_port()
    ctx = mproc.get_context("spawn")
    q = ctx.Queue()
    hub = ctx.Process(target=_rdzv_worker, args=(0, 2, port, q))
    hub.start()
    _abandoning_client(port)                  # first in the hub's queue, gone before the answer
    time.sleep(0.5)
    peer = ctx.Process(target=_rdzv_worker, args=(1, 2, port, q))
    peer.start()
    got = dict(q.get(timeout=60)[:2] for _ in range(2))
    for p in (hub, peer):
        p.join(timeout=30)
        assert p.exitcode == 0
    assert got[0] == got[1] == bytes(range(128))


def test_watchdog_ends_a_hung_run():
    """--watchdog-s: a rank stuck past the limit (a peer died in a collective) exits with code 3 and says so, instead of
    hanging the launcher; a run that finishes in time cancels it."""
    import subprocess
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "bench._start_watchdog(0.5, {'rank': 1, 'nranks': 2}); time.sleep(30)") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=25)
    assert p.returncode == 3 and "watchdog: rank 1 of 2" in p.stderr
    code = ("import sys, time; sys.path.insert(0, %r); import bench; "
            "t = bench._start_watchdog(0.5, {'rank': 0, 'nranks': 1}); t.cancel(); time.sleep(1.0)") % ROOT
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=25)
    assert p.returncode == 0
    assert bench._start_watchdog(0, {"rank": 0, "nranks": 1}) is None


def test_cpu_baseline_threads_follow_the_plan():
    """the CPU baseline runs the port on one thread per CPU the process can actually use --
    min(logical CPUs reported, affinity mask, cgroup quota rounded up) -- not on every logical CPU a container sees (256
    threads under a 16-CPU quota only time-slice). The 16-thread per-GPU share is reported beside it when it differs."""
    t = bench.baseline_threads(cpu_count=256, affinity=256, quota=16.0)      # the GPU box: 256 logical, quota 16
    assert t["threads"] == 16 and t["share_threads"] == 16 and t["logical_cpus"] == 256
    assert bench.baseline_threads(cpu_count=256, affinity=24, quota=None)["threads"] == 24
    assert bench.baseline_threads(cpu_count=64, affinity=64, quota=12.5)["threads"] == 13
    t = bench.baseline_threads(cpu_count=64, affinity=64, quota=None)
    assert t["threads"] == 64 and t["share_threads"] == 16
    assert bench.baseline_threads(cpu_count=4, affinity=4, quota=None)["share_threads"] == 4
    assert bench.baseline_threads(cpu_count=4096, affinity=4096, quota=None)["threads"] == 1024  # the oracle's cap
    here = bench.baseline_threads()
    q = bench._cgroup_cpu_quota()
    assert here["threads"] == max(1, min(os.cpu_count(), len(os.sched_getaffinity(0)), 1024,
                                         -(-int(q * 100) // 100) if q else 1024))


def test_cpu_baseline_runs_on_the_usable_cores():
    """The baseline leg itself on a small workload: cores = the CPUs this process can use, a positive rate, and the
    share figure labelled beside it only when that differs from 16."""
    sys.path.insert(0, os.path.join(ROOT, "wc-path-tracer_amd"))
    from wcpt import scene as wscene
    s = wscene.generate("cornell")
    th = bench.baseline_threads()
    cb = bench.cpu_baseline(s, 64, 64, 1, 1, budget_s=1.0, min_frames=2)
    assert cb["cores"] == th["threads"] and cb["kind"] == "port" and cb["value"] > 0
    assert ("per_gpu_share" in cb) == (th["threads"] > 16)


def test_rccl_rehearsal_flag_and_environment():
    """--rccl-rehearsal is a torchrun-only mode of the RCCL group: it gives each rank its own NCCL_HOSTID (RCCL then
    lets two ranks share one device and exchanges over sockets), on the loopback unless the host chose an interface."""
    with pytest.raises(SystemExit):
        _topo(["--rccl-rehearsal"])                                   # no launcher
    with pytest.raises(SystemExit):
        _topo(["--rccl-rehearsal", "--dist-backend", "gloo"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    t = _topo(["--rccl-rehearsal"], {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"})
    assert t["mode"] == "ranks" and t["rank"] == 1
    env = {"NCCL_SOCKET_IFNAME": "eth7"}
    bench.rccl_rehearsal_env(env, 1)
    assert env == {"NCCL_HOSTID": "wcpt-rehearsal-1", "NCCL_SOCKET_IFNAME": "eth7", "NCCL_IB_DISABLE": "1"}
    env = {}
    bench.rccl_rehearsal_env(env, 0)
    assert env["NCCL_SOCKET_IFNAME"] == "lo" and env["NCCL_HOSTID"] == "wcpt-rehearsal-0"


def test_frame_overlap_flag():
    """--frame-overlap sets WCPT_OPTION_FRAME_OVERLAP on every context (-1, the default, leaves the library's auto);
    the option id matches the header's."""
    assert bench.parse_args([]).frame_overlap == -1
    assert bench.parse_args(["--frame-overlap", "0"]).frame_overlap == 0
    with pytest.raises(SystemExit):
        bench.parse_args(["--frame-overlap", "3"])
    import wcpt
    hdr = open(os.path.join(ROOT, "include", "wcpt.h")).read()
    assert "#define WCPT_OPTION_FRAME_OVERLAP 15" in hdr and wcpt._lib.OPTION_FRAME_OVERLAP == 15
