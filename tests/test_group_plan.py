"""The group's frame plan on a simulated device (CPU): the order in which wcpt_group_render issues its device
operations (wc-path-tracer_amd/csrc/group_plan.h, compiled here with g++ from the product header) is run through a
model of HIP streams and events with random durations, and the ordering rules of the overlapped gather are checked
("the overlap is verified by event ordering in a CPU-runnable bookkeeping test"):

- a sender's render never rewrites a payload buffer before the transfer that read it has finished;
- a transfer starts only after the render that wrote its payload has finished;
- every send has exactly one matching receive on the root (RCCL), for the same frame and buffer;
- with overlap on, frame k + 1's renders (the root's included) run while frame k's transfers are in flight; with it
  off, a rank's next render starts only after its transfer;
- the plan never deadlocks, and one process per rank issues the same operations as one process for all ranks.

The model: each (rank, stream) executes its operations in issue order; an event wait completes at the time of the
latest record of that event issued before it (HIP semantics; no record = no wait); a send and its receive start
together when both streams reach them (a rendezvous) and end together.
"""
import ctypes
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "wc-path-tracer_amd", "csrc", "group_plan.h")

WAIT_SENT, SET_OUTPUT, RENDER, RECORD_READY, COMM_WAIT_READY, SEND, RECV, RECORD_SENT, SCATTER = range(9)
RENDER_STREAM, COMM_STREAM = 0, 1


def _parse_header_ops():
    """The op numbers as the header defines them (the test fails if they drift from the constants above)."""
    ops = {}
    for line in open(HEADER):
        line = line.strip()
        for name in ("kWaitSent", "kSetOutput", "kRender", "kRecordReady", "kCommWaitReady", "kSend", "kRecv",
                     "kRecordSent", "kScatter"):
            if line.startswith(name + " ="):
                ops[name] = int(line.split("=")[1].split(",")[0])
    return ops


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = tmp_path_factory.mktemp("plan") / "libgroup_plan_shim.so"
    src = os.path.join(ROOT, "tests", "group_plan_shim.cpp")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", src, "-o", str(out)], check=True)
    lib = ctypes.CDLL(str(out))
    I32P = ctypes.POINTER(ctypes.c_int32)
    lib.plan_frames.argtypes = [ctypes.c_int] * 5 + [I32P, I32P, ctypes.c_int, I32P, ctypes.c_int, ctypes.c_int]
    lib.plan_frames.restype = ctypes.c_int
    return lib


def plan(shim, nranks, root, overlap, copy, local, presenting, stripes=False):
    cap = 100000
    out = (ctypes.c_int32 * (6 * cap))()
    loc = (ctypes.c_int32 * len(local))(*local)
    pres = (ctypes.c_int32 * len(presenting))(*[1 if p else 0 for p in presenting])
    n = shim.plan_frames(nranks, root, int(overlap), int(copy), len(local), loc, pres, len(presenting), out, cap,
                         int(stripes))
    assert n >= 0
    return [dict(frame=out[6 * i], op=out[6 * i + 1], rank=out[6 * i + 2], buffer=out[6 * i + 3],
                 peer=out[6 * i + 4], stream=out[6 * i + 5]) for i in range(n)]


def simulate(steps_per_process, durations):
    """Times of every operation. steps_per_process: one issue-ordered step list per process."""
    ops = []
    for steps in steps_per_process:
        last_record = {}  # (rank, event kind, buffer) -> index of the latest record issued so far in this process
        for s in steps:
            o = dict(s)
            o["stream_key"] = (s["rank"], s["stream"])
            o["dep"] = None
            if s["op"] == WAIT_SENT:
                o["dep"] = last_record.get((s["rank"], "sent", s["buffer"]))
            elif s["op"] == COMM_WAIT_READY:
                o["dep"] = last_record.get((s["rank"], "ready", s["buffer"]))
            o["dur"] = durations(o)
            ops.append(o)
            if s["op"] == RECORD_READY:
                last_record[(s["rank"], "ready", s["buffer"])] = len(ops) - 1
            elif s["op"] == RECORD_SENT:
                last_record[(s["rank"], "sent", s["buffer"])] = len(ops) - 1
    # stream order and transfer partners
    prev = {}
    for i, o in enumerate(ops):
        o["prev"] = prev.get(o["stream_key"])
        prev[o["stream_key"]] = i
    sends = {(o["frame"], o["rank"]): i for i, o in enumerate(ops) if o["op"] == SEND}
    recvs = {(o["frame"], o["peer"]): i for i, o in enumerate(ops) if o["op"] == RECV}
    for key, i in recvs.items():
        assert key in sends, f"receive without a send: frame {key[0]} from rank {key[1]}"
        ops[i]["partner"] = sends[key]
        ops[sends[key]]["partner"] = i
    for o in ops:
        o.setdefault("partner", None)
        o["start"] = o["end"] = 0.0
    for _ in range(10 * len(ops) + 10):
        changed = False
        for o in ops:
            ready = ops[o["prev"]]["end"] if o["prev"] is not None else 0.0
            if o["dep"] is not None:
                ready = max(ready, ops[o["dep"]]["end"])
            o["ready"] = ready
        for o in ops:
            start = o["ready"]
            if o["partner"] is not None:
                start = max(start, ops[o["partner"]]["ready"])
            end = start + o["dur"]
            if start != o["start"] or end != o["end"]:
                o["start"], o["end"], changed = start, end, True
        if not changed:
            return ops
    raise AssertionError("the plan deadlocks (times never settle)")


def check_rules(ops, nranks, root, overlap, copy, presenting):
    renders = {(o["frame"], o["rank"]): o for o in ops if o["op"] == RENDER}
    sends = {(o["frame"], o["rank"]): o for o in ops if o["op"] == SEND}
    outputs = {(o["frame"], o["rank"]): o for o in ops if o["op"] == SET_OUTPUT}
    recvs = [o for o in ops if o["op"] == RECV]
    frames = len(presenting)
    exch = [p and nranks > 1 for p in presenting]
    for k in range(frames):
        for r in range(nranks):
            assert (k, r) in renders
            if not exch[k] or r == root:
                assert (k, r) not in sends
                continue
            rend, send, so = renders[(k, r)], sends[(k, r)], outputs[(k, r)]
            b = send["buffer"]
            assert so["buffer"] == b == rend["buffer"]
            assert b == (k % 2 if overlap else 0)
            # the transfer reads what this frame's render wrote
            assert send["start"] >= rend["end"] - 1e-9, (k, r)
            # the render rewrote payload b only after the previous transfer that read b had finished
            earlier = [sends[(j, r)] for j in range(k) if (j, r) in sends and sends[(j, r)]["buffer"] == b]
            if earlier:
                assert rend["start"] >= earlier[-1]["end"] - 1e-9, (k, r)
            assert send["peer"] == root
    if copy:
        assert not recvs
    else:
        assert len(recvs) == len(sends)
        for o in recvs:
            s = sends[(o["frame"], o["peer"])]
            assert o["rank"] == root and o["buffer"] == s["buffer"] and o["start"] == s["start"]


@pytest.mark.parametrize("nranks,root", [(2, 0), (3, 0), (4, 2), (8, 0)])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("copy", [False, True])
def test_plan_orders_every_frame(shim, nranks, root, overlap, copy):
    assert _parse_header_ops() == dict(kWaitSent=WAIT_SENT, kSetOutput=SET_OUTPUT, kRender=RENDER,
                                       kRecordReady=RECORD_READY, kCommWaitReady=COMM_WAIT_READY, kSend=SEND,
                                       kRecv=RECV, kRecordSent=RECORD_SENT, kScatter=SCATTER)
    presenting = [True, True, True, False, True, True, True, True, False, False, True, True]
    steps = plan(shim, nranks, root, overlap, copy, list(range(nranks)), presenting)
    for seed in range(6):
        rng = random.Random(seed * 101 + nranks)

        def dur(o):
            if o["op"] == RENDER:
                return rng.uniform(1.0, 3.0)
            if o["op"] in (SEND, RECV):
                return rng.uniform(0.2, 6.0)
            return 0.0

        ops = simulate([steps], dur)
        check_rules(ops, nranks, root, overlap, copy, presenting)


@pytest.mark.parametrize("copy", [False, True])
def test_overlap_lets_the_next_render_run_during_the_transfer(shim, copy):
    """Slow transfers (10x a render): with overlap, frame k + 1 renders while frame k's blocks are still moving -- on
    the senders and on the root; in line (overlap off), a sender's next render waits for its transfer."""
    n, root, frames = 4, 0, 6
    slow = lambda o: 1.0 if o["op"] == RENDER else (10.0 if o["op"] in (SEND, RECV) else 0.0)  # noqa: E731
    for overlap in (True, False):
        ops = simulate([plan(shim, n, root, overlap, copy, list(range(n)), [True] * frames)], slow)
        check_rules(ops, n, root, overlap, copy, [True] * frames)
        renders = {(o["frame"], o["rank"]): o for o in ops if o["op"] == RENDER}
        sends = {(o["frame"], o["rank"]): o for o in ops if o["op"] == SEND}
        for r in range(1, n):
            overlapped = renders[(1, r)]["start"] < sends[(0, r)]["end"]
            assert overlapped == overlap, (overlap, r)
        xfer_end = max(o["end"] for o in ops if o["op"] in (SEND, RECV) and o["frame"] == 0)
        # the root's next render never waits for the gather, with or without overlap of the senders
        assert renders[(1, root)]["start"] < xfer_end or not overlap


def test_one_process_per_rank_issues_the_same_operations(shim):
    """wcpt_group_create_rank: each process plans only its own rank; the union of the processes' plans is the
    single-process plan, and simulating the processes side by side keeps every rule."""
    n, root = 4, 1
    presenting = [True, True, False, True, True]
    whole = plan(shim, n, root, True, False, list(range(n)), presenting)
    per = [plan(shim, n, root, True, False, [r], presenting) for r in range(n)]
    key = lambda s: (s["frame"], s["op"], s["rank"], s["buffer"], s["peer"], s["stream"])  # noqa: E731
    assert sorted(map(key, whole)) == sorted(key(s) for p in per for s in p)
    rng = random.Random(7)
    ops = simulate(per, lambda o: rng.uniform(1, 3) if o["op"] == RENDER else
                   (rng.uniform(0.5, 5) if o["op"] in (SEND, RECV) else 0.0))
    check_rules(ops, n, root, True, False, presenting)


def test_group_of_one_plans_only_renders(shim):
    steps = plan(shim, 1, 0, True, False, [0], [True] * 4)
    assert [s["op"] for s in steps] == [RENDER] * 4


@pytest.mark.parametrize("overlap", [True, False])
def test_direct_transport_plans_only_renders(shim, overlap):
    """WCPT_GROUP_TRANSPORT_DIRECT: each sender's render writes its rows of the root's frame itself, so a frame is the
    renders alone -- one launch per rank, nothing for the host to order between devices."""
    n = 8
    steps = plan(shim, n, 0, overlap, 2, list(range(n)), [True, False, True])
    assert [(s["frame"], s["op"], s["rank"]) for s in steps] == [(f, RENDER, r) for f in range(3) for r in range(n)]



@pytest.mark.parametrize("nranks,root", [(2, 0), (4, 2), (8, 0)])
@pytest.mark.parametrize("overlap", [True, False])
def test_row_stripes_scatter_each_received_block_after_its_transfer(shim, nranks, root, overlap):
    """Interleaved row stripes over RCCL (WCPT_GROUP_OPTION_ROW_STRIPE): the root receives every block into its staging
    buffer and then copies it to its frame rows (kScatter) on the same stream -- after the receive of that frame, before
    the next frame's receive into the same staging area, and outside the ncclGroupStart/End (every send and receive of
    the frame stay contiguous in the plan, so one host thread can post them in one group). COPY needs no scatter."""
    presenting = [True, True, False, True, True, True]
    steps = plan(shim, nranks, root, overlap, False, list(range(nranks)), presenting, stripes=True)
    assert not [s for s in plan(shim, nranks, root, overlap, True, list(range(nranks)), presenting, stripes=True)
                if s["op"] == SCATTER]
    for f in range(len(presenting)):
        fs = [s for s in steps if s["frame"] == f]
        xfer = [i for i, s in enumerate(fs) if s["op"] in (SEND, RECV)]
        assert xfer == list(range(xfer[0], xfer[-1] + 1)) if xfer else True      # one contiguous group
        sc = [s for s in fs if s["op"] == SCATTER]
        assert sorted(s["peer"] for s in sc) == ([r for r in range(nranks) if r != root] if presenting[f] else [])
        for s in sc:
            assert s["rank"] == root and fs.index(s) > xfer[-1]
            assert s["stream"] == [r for r in fs if r["op"] == RECV and r["peer"] == s["peer"]][0]["stream"]
    for seed in range(4):
        rng = random.Random(seed)
        ops = simulate([steps], lambda o: rng.uniform(1, 3) if o["op"] == RENDER else
                       (rng.uniform(0.5, 5) if o["op"] in (SEND, RECV, SCATTER) else 0.0))
        check_rules(ops, nranks, root, overlap, False, presenting)
        recv_end = {(o["frame"], o["peer"]): o["end"] for o in ops if o["op"] == RECV}
        recv_start = {(o["frame"], o["peer"]): o["start"] for o in ops if o["op"] == RECV}
        for o in ops:
            if o["op"] != SCATTER:
                continue
            assert o["start"] >= recv_end[(o["frame"], o["peer"])] - 1e-9
            later = [t for (f, p), t in recv_start.items() if p == o["peer"] and f > o["frame"]]
            if later:                                     # the next receive into this staging area waits for it
                assert min(later) >= o["end"] - 1e-9

# ---- the bounded wait of wcpt_group_sync (csrc/group_wait.h) ------------------------------------------------------------
DONE, FAILED, TRANSPORT_ERROR, TIMED_OUT = range(4)


def wait(shim, ready_after=-1, error_after=-1, fail_at=-1, timeout_ms=1000.0, ms_per_poll=0.001):
    f = shim.wait_sim
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_double,
                  ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    f.restype = ctypes.c_int
    el, polls, naps = ctypes.c_double(), ctypes.c_int(), ctypes.c_int()
    r = f(ready_after, error_after, fail_at, timeout_ms, ms_per_poll, ctypes.byref(el), ctypes.byref(polls),
          ctypes.byref(naps))
    return r, el.value, polls.value, naps.value


def test_bounded_wait_returns_when_the_streams_drain(shim):
    r, el, polls, naps = wait(shim, ready_after=3)
    assert (r, polls, naps) == (DONE, 4, 0)            # a stream that drains at once: spins, never sleeps
    r, el, polls, naps = wait(shim, ready_after=5000, timeout_ms=60000.0)  # a long frame: naps of up to 1 ms
    assert r == DONE and polls == 5001 and 0 < naps < polls and el <= 5001 * 1.001


def test_bounded_wait_is_late_by_a_small_fraction(shim):
    """A wait returns within 0.5 % (or 10 us) of the stream's drain: the naps grow with the time waited, not by doubling
    (round 6 first doubled them up to 1 ms, and a 7-ms wait for a 20-frame bench window overslept by up to 1 ms)."""
    f = shim.wait_sim_time
    f.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                  ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    f.restype = ctypes.c_int
    for ms_per_poll in (0.001, 0.003):
        for drain in (0.02, 0.5, 7.0, 70.0, 700.0, 7000.0):
            el, polls, naps = ctypes.c_double(), ctypes.c_int(), ctypes.c_int()
            r = f(drain, 60000.0, ms_per_poll, ctypes.byref(el), ctypes.byref(polls), ctypes.byref(naps))
            assert r == DONE
            late = el.value - drain
            assert 0.0 <= late <= max(0.005 * drain * 1.01, 0.010) + 2 * ms_per_poll
            if drain >= 7.0:                           # and it slept: far fewer polls than a spin of the whole wait
                assert polls.value < drain / ms_per_poll / 5


def test_peer_that_never_posts_ends_in_a_timeout(shim):
    """a rank whose peer died (or skipped its part of a frame) has a transfer that never completes.
    The sync's wait ends at the group's timeout (the caller then aborts the communicators and returns
    WCPT_ERROR_DEVICE_LOST) instead of blocking for ever; the naps are bounded, so it ends within a nap of it."""
    for timeout in (50.0, 3000.0):
        r, el, polls, naps = wait(shim, ready_after=-1, timeout_ms=timeout)
        assert r == TIMED_OUT
        assert timeout <= el <= timeout + 1.0 + 0.002
        assert polls < timeout * 40                    # it sleeps between polls: no busy spin (50,000 polls per 50 ms)


def test_transport_error_ends_the_wait_before_the_timeout(shim):
    r, el, polls, naps = wait(shim, ready_after=-1, error_after=40, timeout_ms=60000.0)
    assert r == TRANSPORT_ERROR and polls == 41 and el < 60000.0


def test_failed_poll_and_no_deadline(shim):
    assert wait(shim, ready_after=-1, fail_at=7)[0] == FAILED
    # timeout 0 (WCPT_GROUP_OPTION_TIMEOUT_MS = 0): no deadline; only a drain, an error or a failed poll ends it
    r, el, polls, naps = wait(shim, ready_after=20000, timeout_ms=0.0)
    assert r == DONE and el > 1000.0


def test_a_skipped_frame_leaves_the_root_one_receive_without_a_send(shim):
    """RCCL pairs a rank's sends with the root's receives in posting order. A rank that skips one frame's
    wcpt_group_render posts one send fewer than the root posts receives, so the root's last receive -- and everything
    queued behind it on its communication stream -- never completes: exactly the wait the bound above ends."""
    n, root, frames, skip = 2, 0, 5, 3
    per = [plan(shim, n, root, True, False, [r], [True] * (frames if r == root else frames - 1)) for r in range(n)]
    recvs = [s for s in per[root] if s["op"] == RECV and s["peer"] == 1]
    sends = [s for s in per[1] if s["op"] == SEND]
    assert len(recvs) == frames and len(sends) == frames - 1
    assert skip < frames and recvs[-1]["stream"] == COMM_STREAM
    assert wait(shim, ready_after=-1, timeout_ms=100.0)[0] == TIMED_OUT
