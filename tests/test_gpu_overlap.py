"""Frame overlap (WCPT_OPTION_FRAME_OVERLAP) on the GPU: consecutive megakernel renders split the cost-ordered tiles
between two pipes (pt_kernels.hip launch_megakernel) and the wavefront kernel's pipelines skip their per-frame join
(pt_wavefront.hip launch_wavefront), so each pipe runs on into its next frame. Each pixel stays with one pipe, and
every other entry point joins the pipes into the context's stream first, so the results must be the plain stream's bit
for bit:

- progressive frames across the re-sorts (renders 1, 4, 16) against the oracle's accumulation and a context with the
  overlap off;
- the same sequence interleaved with every kind of call that has to join (readback, sync, counting renders, profiled
  regions, per-render timing, a tile-order change, a kernel switch, a resize, a row range);
- a one-process COPY group whose contexts overlap, against the same group without;
- the 1920x1080 Cornell frame, where the default (auto) turns the overlap on.
"""
import numpy as np
import pytest

import wcpt
import oracle

from test_gpu_parity import assert_close, get_scene

pytestmark = pytest.mark.gpu

T = wcpt._lib


def _frames(ctx, dev, s, W, H, frames, bounces, spp=1):
    for f in frames:
        ctx.render(s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f), *dev.addresses())


def _bits(img):
    return np.ascontiguousarray(img).view(np.uint32)


def _kernel_setup(ctx, kernel):
    """The megakernel (its cost order and pipes), or the wavefront kernel with three per-bounce pipelines (the
    path-persistent trace, one pipeline, off)."""
    ctx.set_kernel(kernel)
    if kernel == wcpt.KERNEL_WAVEFRONT:
        ctx.set_option(T.OPTION_WF_PERSIST, 0)
        ctx.set_option(T.OPTION_WF_PIPES, 3)


KERNELS = [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name,W,H,bounces,spp", [("cornell", 67, 45, 4, 1), ("reference_init", 96, 64, 3, 1),
                                                   ("default_dielectric", 40, 27, 3, 2)])
def test_overlap_frames_match_oracle(name, W, H, bounces, spp, kernel):
    """20 progressive frames with the overlap forced on (megakernel: every render after the first sort runs as two
    pipes, the re-sorts after renders 4 and 16 join and fork again; wavefront: each pipeline runs on into its next
    frame): bit-exact against the oracle's accumulation and against the same frames with the overlap off."""
    s = get_scene(name)
    frames = range(20)
    imgs = {}
    for ov in (2, 0):
        with wcpt.Context(0) as ctx:
            _kernel_setup(ctx, kernel)
            ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
            dev = wcpt.DeviceScene(ctx, s)
            try:
                ctx.create_screen(W, H)
                _frames(ctx, dev, s, W, H, frames, bounces, spp)
                ctx.sync()
                imgs[ov] = ctx.readback(H)
            finally:
                dev.free()
    assert np.array_equal(_bits(imgs[2]), _bits(imgs[0]))
    acc = None
    for f in frames:
        sd = s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f)
        acc, _ = oracle.render_scene(s, W, H, sd=sd, image=acc, threads=8)
    assert_close(imgs[2], acc)


def _interleaved(ov, kernel):
    """One sequence of renders and joining calls; returns every image it read."""
    s = get_scene("cornell")
    W, H, b = 72, 48, 4
    other = wcpt.KERNEL_WAVEFRONT if kernel == wcpt.KERNEL_MEGAKERNEL else wcpt.KERNEL_MEGAKERNEL
    out = []
    with wcpt.Context(0) as ctx:
        _kernel_setup(ctx, kernel)
        ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
        dev = wcpt.DeviceScene(ctx, s)
        try:
            ctx.create_screen(W, H)
            _frames(ctx, dev, s, W, H, range(0, 6), b)
            out.append(ctx.readback(H))                       # readback joins (no sync before it)
            _frames(ctx, dev, s, W, H, range(6, 9), b)
            cnt = ctx.render_counters(s.scene_data(W, H, max_bounce=b, frame=9), *dev.addresses())
            out.append(np.array([cnt["segments"], cnt["triangle_tests"]], np.float32))
            _frames(ctx, dev, s, W, H, range(9, 12), b)
            ctx.set_option(T.OPTION_PROFILE_REGION, 1)       # one timed region over overlapped renders
            ctx.profile_begin()
            _frames(ctx, dev, s, W, H, range(12, 18), b)
            ms, n = ctx.profile_end()
            assert n == 6 and ms > 0
            ctx.set_option(T.OPTION_PROFILE_REGION, 0)       # per-render events: no overlap under them
            ctx.profile_begin()
            _frames(ctx, dev, s, W, H, range(18, 21), b)
            ms, n = ctx.profile_end()
            assert n == 3 and ms > 0
            ctx.set_option(T.OPTION_MK_TILE_ORDER, 1)        # scattered order: the pipes stop ...
            _frames(ctx, dev, s, W, H, range(21, 23), b)
            ctx.set_option(T.OPTION_MK_TILE_ORDER, 2)        # ... and start again after the next sort
            _frames(ctx, dev, s, W, H, range(23, 27), b)
            ctx.set_kernel(other)                             # another kernel on the same image
            _frames(ctx, dev, s, W, H, range(27, 29), b)
            ctx.set_kernel(kernel)
            _frames(ctx, dev, s, W, H, range(29, 36), b)
            ctx.sync()
            out.append(ctx.readback(H))
            ctx.set_row_range(8, 24)                          # a new geometry: costs, order and pipes start over
            _frames(ctx, dev, s, W, H, range(0, 7), b)
            ctx.sync()
            out.append(ctx.readback(24))
            ctx.set_row_range(0, 0)
            ctx.resize(W + 16, H - 9)
            _frames(ctx, dev, s, W + 16, H - 9, range(0, 7), b)
            out.append(ctx.readback(H - 9))
        finally:
            dev.free()
    return out


@pytest.mark.parametrize("kernel", KERNELS)
def test_overlap_interleaved_calls_equal_plain_stream(kernel):
    """Every kind of call between overlapped renders (readback, counting render, timed regions, per-render events, a
    tile-order change, a kernel switch, a row range, a resize) sees and leaves the same bytes as on the plain stream."""
    a = _interleaved(2, kernel)
    b = _interleaved(0, kernel)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x.shape == y.shape and np.array_equal(_bits(x), _bits(y))
    # the first image also against the oracle (frames 0-5)
    s = get_scene("cornell")
    acc = None
    for f in range(6):
        acc, _ = oracle.render_scene(s, 72, 48, max_bounce=4, frame=f, image=acc, threads=8)
    assert_close(a[0], acc)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("n,transport,gov,stripe", [(1, "copy", 1, 0), (2, "copy", 1, 0), (3, "copy", 1, 0),
                                                    (3, "copy", 0, 0), (2, "direct", 1, 0), (3, "copy", 1, 8)])
def test_overlap_in_a_group_equals_plain(n, transport, gov, stripe, kernel):
    """A one-process group on the one GPU whose contexts overlap their renders: the root's presented frames and every
    rank's block equal the group without overlap. With communication streams (GROUP_OPTION_OVERLAP 1) a sender's pipes
    run on: each frame is fenced by an event on every stream holding part of it, and the next frame's streams wait for
    the payload's previous transfer; with transfers in line (0) the group keeps the overlap off; DIRECT renders write
    the root's frame themselves; stripes interleave the ranks' rows."""
    s = get_scene("cornell")
    W, H, frames = 72, 45, range(10)
    fmt = T.PAYLOAD_RGBA32F
    tr = {"copy": T.GROUP_TRANSPORT_COPY, "direct": T.GROUP_TRANSPORT_DIRECT}[transport]
    res = {}
    for ov in (2, 0):
        with wcpt.Group([0] * n, root=0, transport=tr) as g:
            g.set_option(T.GROUP_OPTION_OVERLAP, gov)
            if stripe:
                g.set_option(T.GROUP_OPTION_ROW_STRIPE, stripe)
            devs = []
            for r in range(n):
                c = g.context(r)
                _kernel_setup(c, kernel)
                c.set_option(T.OPTION_FRAME_OVERLAP, ov)
                devs.append(wcpt.DeviceScene(c, s))
            g.create_screen(W, H)
            rc = g.context(0)
            nbytes = W * H * T.PAYLOAD_PIXEL_BYTES[fmt]
            out = rc.buffer_from(np.full(nbytes // 4, -5.0, np.float32)) if n > 1 else None
            if out is not None:
                g.set_output(fmt, rc.buffer_address(out), nbytes)
            addr = [list(a) for a in zip(*[d.addresses() for d in devs])]
            for f in frames:
                g.render(s.scene_data(W, H, max_bounce=4, frame=f), *addr)
            g.sync()
            raw = rc.buffer_download(out, nbytes) if out is not None else b""
            blocks = [g.context(r).readback() for r in range(n)]
            if out is not None:
                rc.buffer_free(out)
            for d in devs:
                d.free()
        res[ov] = (raw, blocks)
    assert res[2][0] == res[0][0]
    for x, y in zip(res[2][1], res[0][1]):
        assert np.array_equal(_bits(x), _bits(y))


def _moving_camera_frames(ov, s, W, H, n_frames, upload_at=None):
    """Progressive frames while the camera moves every frame, then stays, then moves again (the editor's drag); the
    megakernel with pair records, so every frame's first segments use the primary-ray records of its position."""
    import ctypes
    cams = []
    for f in range(n_frames):
        cam = wcpt.Camera()
        ctypes.pointer(cam)[0] = s.camera
        k = f if f < 8 else (8 if f < 14 else f - 6)      # moving, still for 6 frames, moving again
        cam.position[0] += 0.03 * k
        cam.position[1] += 0.015 * k
        cams.append(cam)
    sds = [s.scene_data(W, H, max_bounce=3, samples=2, frame=f, camera=c) for f, c in enumerate(cams)]
    with wcpt.Context(0) as ctx:
        ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        ctx.set_option(T.OPTION_PAIR_RECORDS, 1)
        ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
        dev = wcpt.DeviceScene(ctx, s)
        try:
            ctx.create_screen(W, H)
            for f, sd in enumerate(sds):
                if f == upload_at:   # the mesh re-uploaded: records rebuilt, both copies of the primary records follow
                    m = s.meshes[0]
                    ctx.buffer_upload(dev.buffers[2], np.ascontiguousarray(m.positions, dtype=np.float32))
                ctx.render(sd, *dev.addresses())
            ctx.sync()
            img = ctx.readback(H)
        finally:
            dev.free()
    return img, sds


@pytest.mark.parametrize("name,W,H", [("cornell", 67, 45), ("reference_init", 96, 64)])
def test_overlap_moving_camera(name, W, H):
    """A camera that moves between frames: only the primary-ray records are derived again, pipe 0's copy on the
    context's stream and pipe 1's on its own, so the overlap goes on without a join. Bit-exact against the same frames
    without the overlap and against the oracle's accumulation; again with a mesh re-upload in the middle."""
    import copy
    s = get_scene(name)
    a, sds = _moving_camera_frames(2, s, W, H, 22)
    b, _ = _moving_camera_frames(0, s, W, H, 22)
    assert np.array_equal(_bits(a), _bits(b))
    acc = None
    for sd in sds:
        acc, _ = oracle.render_scene(copy.copy(s), W, H, sd=sd, image=acc, threads=8)
    assert_close(a, acc)
    c, _ = _moving_camera_frames(2, s, W, H, 22, upload_at=11)
    assert np.array_equal(_bits(c), _bits(a))


@pytest.mark.parametrize("kernel", KERNELS)
def test_overlap_auto_on_full_frame(kernel):
    """The bench's frame (Cornell, 1920x1080, 4 bounces) with the default option, where the auto rule overlaps, equals
    the frames with the overlap off, bit for bit, across the first re-sorts."""
    s = get_scene("cornell")
    W, H = 1920, 1080
    imgs = {}
    for ov in (1, 0):
        with wcpt.Context(0) as ctx:
            ctx.set_kernel(kernel)
            ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
            dev = wcpt.DeviceScene(ctx, s)
            try:
                ctx.create_screen(W, H)
                _frames(ctx, dev, s, W, H, range(18), 4)
                ctx.sync()
                imgs[ov] = ctx.readback(H)
            finally:
                dev.free()
    assert np.array_equal(_bits(imgs[1]), _bits(imgs[0]))


def test_overlap_option_range():
    with wcpt.Context(0) as ctx:
        for v in (0, 1, 2):
            ctx.set_option(T.OPTION_FRAME_OVERLAP, v)
        for v in (-1, 3):
            with pytest.raises(T.WcptError):
                ctx.set_option(T.OPTION_FRAME_OVERLAP, v)


def _checkpoints(ov, name, kernel, frames, every):
    s = get_scene(name)
    W, H = 1920, 1080
    out = []
    with wcpt.Context(0) as ctx:
        ctx.set_kernel(kernel)
        ctx.set_option(T.OPTION_FRAME_OVERLAP, ov)
        dev = wcpt.DeviceScene(ctx, s)
        try:
            ctx.create_screen(W, H)
            for f in range(frames):
                ctx.render(s.scene_data(W, H, max_bounce=4, frame=f), *dev.addresses())
                if (f + 1) % every == 0:
                    out.append(ctx.readback(H))        # joins the pipes mid-run; the next render forks again
        finally:
            dev.free()
    return out


@pytest.mark.parametrize("name,kernel,frames,every", [("cornell", wcpt.KERNEL_MEGAKERNEL, 200, 50),
                                                      ("reference_init", wcpt.KERNEL_MEGAKERNEL, 140, 35),
                                                      ("atrium", wcpt.KERNEL_WAVEFRONT, 48, 16)])
def test_overlap_long_run_checkpoints(name, kernel, frames, every):
    """Full 1080p frames over a long progressive run -- the re-sorts at renders 64 and 128 included -- with the image
    read back at checkpoints (each one joins the pipes): bit-identical to the same run with the overlap off."""
    a = _checkpoints(1, name, kernel, frames, every)
    b = _checkpoints(0, name, kernel, frames, every)
    assert len(a) == len(b) == frames // every
    for x, y in zip(a, b):
        assert np.array_equal(_bits(x), _bits(y))

