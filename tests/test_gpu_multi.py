"""Multi-device paths on the GPU box, through the product library:

- the C-ABI group (wcpt_group_*: one context per device from one host thread, row blocks, RCCL gather of each presented
  frame to the root) at n = 1, bit-identical to a plain context, in every payload format; its error paths;
- two ranks with libwcpt.so each rendering their row block of the frame on the one GPU, gathered over gloo (RCCL refuses
  two ranks on one device), against a one-context render.

The N = 8 RCCL run itself is the driver's scaling bench (bench.py over torch.distributed); the group's N > 1 send/recv
path needs distinct devices and is not reachable on a one-GPU box.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import wcpt
import oracle

from test_gpu_parity import assert_close, get_scene

pytestmark = pytest.mark.gpu

PB = wcpt._lib.PAYLOAD_PIXEL_BYTES


def _context_frames(s, W, H, frames, bounces=4, kernel=wcpt.KERNEL_MEGAKERNEL):
    with wcpt.Context(0) as ctx:
        dev = wcpt.DeviceScene(ctx, s)
        ctx.set_kernel(kernel)
        ctx.create_screen(W, H)
        for f in frames:
            ctx.render(s.scene_data(W, H, max_bounce=bounces, frame=f), *dev.addresses())
        ctx.sync()
        img = ctx.readback()
        dev.free()
    return img


@pytest.mark.parametrize("fmt", [wcpt._lib.PAYLOAD_RGBA32F, wcpt._lib.PAYLOAD_RGB32F,
                                 wcpt._lib.PAYLOAD_DISPLAY_RGBA8])
@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
def test_group_of_one_equals_context(gpu_ctx, fmt, kernel):
    """wcpt_group_* at n = 1 on device 0: progressive frames presented into a root-context buffer equal a plain
    context's accumulation image bit for bit (RGBA / RGB floats), or its composite.comp display value (RGBA8)."""
    s = get_scene("cornell")
    W, H, frames = 72, 40, (0, 1, 2)
    ref = _context_frames(s, W, H, frames, kernel=kernel)
    with wcpt.Group([0], root=0) as g:
        ctx = g.context(0)
        dev = wcpt.DeviceScene(ctx, s)
        ctx.set_kernel(kernel)
        g.create_screen(W, H)
        nbytes = W * H * PB[fmt]
        out = ctx.buffer_from(np.full(nbytes // 4, -3.0, np.float32))
        g.set_output(fmt, ctx.buffer_address(out), nbytes)
        for f in frames:
            g.render(s.scene_data(W, H, max_bounce=4, frame=f), [dev.materials], [dev.spheres], [dev.draws])
        g.sync()
        raw = ctx.buffer_download(out, nbytes)
        img = ctx.readback()
        ctx.buffer_free(out)
        dev.free()
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    if fmt == wcpt._lib.PAYLOAD_DISPLAY_RGBA8:
        assert np.array_equal(np.frombuffer(raw, np.uint8).reshape(H, W, 4), oracle.composite(ref)[1])
    else:
        ch = 4 if fmt == wcpt._lib.PAYLOAD_RGBA32F else 3
        got = np.frombuffer(raw, np.float32).reshape(H, W, ch)
        assert np.array_equal(got.view(np.uint32), ref[..., :ch].view(np.uint32))


def test_group_matches_oracle_and_resizes(gpu_ctx):
    """The group's frame equals the oracle's; after a resize (CreateScreen of the group) the next frame 0 is again the
    oracle's, and an output too small for the new frame is refused."""
    s = get_scene("default_dielectric")
    with wcpt.Group([0]) as g:
        ctx = g.context(0)
        dev = wcpt.DeviceScene(ctx, s)
        for (W, H) in ((48, 40), (64, 24)):
            g.create_screen(W, H)
            nbytes = W * H * 16
            out = ctx.buffer_alloc(nbytes)
            g.set_output(wcpt._lib.PAYLOAD_RGBA32F, ctx.buffer_address(out), nbytes)
            sd = s.scene_data(W, H, max_bounce=3, frame=0)
            g.render(sd, [dev.materials], [dev.spheres], [dev.draws])
            g.sync()
            got = np.frombuffer(ctx.buffer_download(out, nbytes), np.float32).reshape(H, W, 4)
            ref, _ = oracle.render_scene(s, W, H, sd=sd, threads=8)
            assert_close(got.copy(), ref)
            with pytest.raises(wcpt.WcptError):
                g.set_output(wcpt._lib.PAYLOAD_RGBA32F, ctx.buffer_address(out), nbytes - 16)
            g.set_output(wcpt._lib.PAYLOAD_RGBA32F, 0, 0)
            ctx.buffer_free(out)
        dev.free()


def test_group_errors(gpu_ctx):
    with pytest.raises(wcpt.WcptError):
        wcpt.Group([0, 0])                      # one rank per device (RCCL refuses duplicates)
    with pytest.raises(wcpt.WcptError):
        wcpt.Group([0], root=1)
    with pytest.raises(wcpt.WcptError):
        wcpt.Group([wcpt.device_count()])       # no such device
    with wcpt.Group([0]) as g:
        s = get_scene("cornell")
        dev = wcpt.DeviceScene(g.context(0), s)
        with pytest.raises(wcpt.WcptError) as e:
            g.render(s.scene_data(8, 8), [dev.materials], [dev.spheres], [dev.draws])
        assert e.value.code == -1003            # no screen yet
        with pytest.raises(wcpt.WcptError):
            g.set_output(5, 4096, 4096)         # unknown format
        dev.free()


# ---- two ranks with libwcpt.so, gathered over gloo --------------------------------------------------------------
def _free_port():
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    p = sk.getsockname()[1]
    sk.close()
    return p


def _rank(rank, world, port, W, H, frames, kernel, out_path):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "wc-path-tracer_amd")]
    import wcpt as w
    from wcpt import scene as wscene
    from wcpt.dist import gather_frame, row_block
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = wscene.generate("cornell")
    y0, rows = row_block(H, world, rank)
    with w.Context(0) as ctx:
        dev = w.DeviceScene(ctx, s)
        ctx.set_kernel(kernel)
        ctx.create_screen(W, H)
        ctx.set_row_range(y0, rows)
        for f in frames:
            ctx.render(s.scene_data(W, H, max_bounce=4, frame=f), *dev.addresses())
        ctx.sync()
        block = ctx.readback(rows)
        dev.free()
    shard = torch.zeros((-(-H // world), W, 4), dtype=torch.float32)
    shard[:rows] = torch.from_numpy(block)
    frame = gather_frame(shard, H, world, rank, rgb_only=True)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
def test_two_ranks_libwcpt_gather_equals_one_device(gpu_ctx, tmp_path, kernel):
    """Two processes, each with its own libwcpt context on the GPU, render rows [0, H/2) and [H/2, H) of the same
    progressive frames; the blocks gathered on rank 0 (RGB wire format, alpha restored) equal one context's frame
    bit for bit, and that frame equals the oracle's."""
    W, H, frames = 64, 45, (0, 1)
    out = str(tmp_path / "frame.npy")
    mp.spawn(_rank, args=(2, _free_port(), W, H, frames, kernel, out), nprocs=2, join=True)
    got = np.load(out)
    s = get_scene("cornell")
    ref = _context_frames(s, W, H, frames, kernel=kernel)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    acc = None
    for f in frames:
        acc, _ = oracle.render_scene(s, W, H, max_bounce=4, frame=f, image=acc, threads=8)
    assert_close(got, acc)


def _rank_display(rank, world, port, W, H, frames, kernel, out_path):
    """One rank of the display-payload gather (bench.py --gather display): the render itself writes composite.comp's
    RGBA8 display value of the rank's row block into a device payload (WCPT_PAYLOAD_DISPLAY_RGBA8), which travels
    at 4 B/px."""
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "wc-path-tracer_amd")]
    import wcpt as w
    from wcpt import scene as wscene
    from wcpt.dist import assemble, row_block
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = wscene.generate("cornell")
    y0, rows = row_block(H, world, rank)
    payload = torch.zeros((-(-H // world), W, 4), dtype=torch.uint8, device="cuda")
    with w.Context(0) as ctx:
        dev = w.DeviceScene(ctx, s)
        ctx.set_kernel(kernel)
        ctx.create_screen(W, H)
        ctx.set_row_range(y0, rows)
        ctx.set_gather_output(payload.data_ptr(), payload.numel(), w._lib.PAYLOAD_DISPLAY_RGBA8)
        for f in frames:
            ctx.render(s.scene_data(W, H, max_bounce=4, frame=f), *dev.addresses())
        ctx.sync()
        dev.free()
    block = payload.cpu()
    parts = [torch.empty_like(block) for _ in range(world)] if rank == 0 else None
    dist.gather(block, parts, dst=0)
    if rank == 0:
        np.save(out_path, assemble(parts, H, world).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
def test_two_ranks_display_payload_gather_equals_oracle_composite(gpu_ctx, tmp_path, kernel):
    """Two ranks render their row blocks with the RGBA8 display payload written by the render, gather the 4-B/px
    blocks over gloo, and rank 0's frame equals composite.comp (oracle.composite) of the oracle's accumulated frame
    byte for byte (composite.comp:36-53)."""
    W, H, frames = 64, 45, (0, 1, 2)
    out = str(tmp_path / "display.npy")
    mp.spawn(_rank_display, args=(2, _free_port(), W, H, frames, kernel, out), nprocs=2, join=True)
    got = np.load(out)
    s = get_scene("cornell")
    acc = None
    for f in frames:
        acc, _ = oracle.render_scene(s, W, H, max_bounce=4, frame=f, image=acc, threads=8)
    _, want = oracle.composite(acc)
    assert got.dtype == np.uint8 and got.shape == (H, W, 4)
    assert np.array_equal(got, want)
