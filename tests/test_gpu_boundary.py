"""GPU tests of the C-ABI boundary's robustness (include/wcpt.h): draw commands written without
wcpt_buffer_upload, draw commands whose indexCount exceeds the index buffer, vertex indices past the vertex
buffer, and the range checks of buffer uploads / downloads.

The reference (PathTracingRenderer.jai:251-256, BufferManager.jai:52-64) only ever fills its draw-command buffer
through DBufferManager.Update; a host that writes device memory by other means must still get the frame its
draw commands describe.
"""
import ctypes as C

import numpy as np
import pytest

import wcpt
from wcpt import scene as wscene
import oracle

from test_gpu_parity import assert_close, get_scene, _with_mesh

pytestmark = pytest.mark.gpu

_H2D = 1  # hipMemcpyHostToDevice


def _hip():
    """The HIP runtime instance libwcpt.so is bound to (the already-mapped library, not a second copy)."""
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64.so" in ln})
    if not paths:
        pytest.fail("HIP runtime library not mapped")
    h = C.CDLL(paths[0])
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipMemcpy.restype = C.c_int
    return h


def _device_write(addr: int, arr: np.ndarray):
    """hipMemcpy host -> device address, bypassing wcpt_buffer_upload (as an application kernel would)."""
    arr = np.ascontiguousarray(arr)
    assert _hip().hipMemcpy(C.c_void_p(addr), arr.ctypes.data, arr.nbytes, _H2D) == 0


def _moved_positions(s, dx):
    m = s.meshes[0]
    return np.ascontiguousarray(m.positions + np.float32(dx), dtype=np.float32)


@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
def test_draw_commands_written_on_device_cache_off(gpu_ctx, kernel):
    """Draw commands first uploaded for geometry A, then overwritten on the device (hipMemcpy) to point at a second
    vertex buffer B. With WCPT_OPTION_TRIANGLE_CACHE = 0 the render reads the draw commands from the device and
    derives the records from B: the frame equals the oracle's frame of B."""
    s = get_scene("cornell")
    W, H = 64, 48
    dev = wcpt.DeviceScene(gpu_ctx, s)
    posB = _moved_positions(s, 0.07)
    bufB = gpu_ctx.buffer_from(posB)
    gpu_ctx.set_kernel(kernel)
    try:
        gpu_ctx.create_screen(W, H)
        sd = s.scene_data(W, H, max_bounce=3)
        gpu_ctx.render(sd, *dev.addresses())          # geometry A: records derived and cached
        gpu_ctx.sync()
        draws = np.zeros(1, dtype=wcpt._lib.DRAW_COMMAND_DTYPE)
        draws[0] = (gpu_ctx.buffer_address(bufB), gpu_ctx.buffer_address(dev.buffers[3]),
                    gpu_ctx.buffer_address(dev.buffers[4]), s.meshes[0].indices.size, 0)
        _device_write(dev.draws, draws)
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 0)
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        img = gpu_ctx.readback(H)
        m = s.meshes[0]
        ref, _ = oracle.render_scene(_with_mesh(s, wscene.HostBVH(posB, m.indices, m.nodes)), W, H, max_bounce=3,
                                     threads=8)
        assert_close(img, ref)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 1)
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        gpu_ctx.buffer_free(bufB)
        dev.free()


def test_draw_commands_never_uploaded_are_read_from_device(gpu_ctx):
    """A draw-command buffer that was allocated but never written through wcpt_buffer_upload (its host copy holds
    nothing) is read from the device even with the triangle cache on."""
    s = get_scene("cornell")
    W, H = 64, 48
    dev = wcpt.DeviceScene(gpu_ctx, s)
    dbuf = gpu_ctx.buffer_alloc(32)
    try:
        draws = np.zeros(1, dtype=wcpt._lib.DRAW_COMMAND_DTYPE)
        draws[0] = (gpu_ctx.buffer_address(dev.buffers[2]), gpu_ctx.buffer_address(dev.buffers[3]),
                    gpu_ctx.buffer_address(dev.buffers[4]), s.meshes[0].indices.size, 0)
        _device_write(gpu_ctx.buffer_address(dbuf), draws)
        gpu_ctx.create_screen(W, H)
        sd = s.scene_data(W, H, max_bounce=3)
        gpu_ctx.render(sd, dev.materials, dev.spheres, gpu_ctx.buffer_address(dbuf))
        gpu_ctx.sync()
        img = gpu_ctx.readback(H)
        ref, _ = oracle.render_scene(s, W, H, max_bounce=3, threads=8)
        assert_close(img, ref)
    finally:
        gpu_ctx.buffer_free(dbuf)
        dev.free()


def test_index_count_past_index_buffer_is_rejected(gpu_ctx):
    s = get_scene("cornell")
    dev = wcpt.DeviceScene(gpu_ctx, s)
    try:
        n = s.meshes[0].indices.size
        draws = np.zeros(1, dtype=wcpt._lib.DRAW_COMMAND_DTYPE)
        draws[0] = (gpu_ctx.buffer_address(dev.buffers[2]), gpu_ctx.buffer_address(dev.buffers[3]),
                    gpu_ctx.buffer_address(dev.buffers[4]), n + 3, 0)
        gpu_ctx.buffer_upload(dev.buffers[5], draws)
        gpu_ctx.create_screen(32, 32)
        with pytest.raises(wcpt.WcptError) as e:
            gpu_ctx.render(s.scene_data(32, 32, max_bounce=1), *dev.addresses())
        assert e.value.code == -1000 and "indexCount" in str(e.value)
        # a valid indexCount renders again on the same context
        draws[0]["indexCount"] = n
        gpu_ctx.buffer_upload(dev.buffers[5], draws)
        gpu_ctx.render(s.scene_data(32, 32, max_bounce=1), *dev.addresses())
        gpu_ctx.sync()
    finally:
        dev.free()


@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
@pytest.mark.parametrize("path", ["singles", "pairs", "index"])
def test_vertex_index_past_vertex_buffer_never_hits(gpu_ctx, kernel, path):
    """An index past the vertex buffer (undefined in the reference) gives a triangle no ray accepts: the frame equals
    the oracle's frame in which that triangle's vertex is NaN. Through the derived records (single and pair records;
    the one leaf ends at the draw's last triangle) and through the index path (the draw's indexCount covers only the
    first triangle, so the leaf is not record-backed and its triangles are gathered from the index and vertex
    buffers, pt_device.h tri_from_indices), in both kernels."""
    pairs = {"singles": 0, "pairs": 1, "index": -1}[path]
    rng = np.random.default_rng(11)
    ntri = 24
    pos = (rng.random((ntri * 3, 3), dtype=np.float32) * 2.0 - 1.0).astype(np.float32)
    pos[:, 0] = pos[:, 0] * 0.25 + 1.5                 # in front of the default camera (looking along +x)
    idx = np.arange(ntri * 3, dtype=np.uint32)
    bad = 10                                           # triangle 10's second vertex index is out of range
    idx_dev = idx.copy()
    idx_dev[3 * bad + 1] = pos.shape[0] + 100000
    lo, hi = pos.min(axis=0), pos.max(axis=0)
    nodes = np.zeros(1, dtype=wcpt._lib.NODE_DTYPE)
    nodes[0] = (lo, hi, 0, 3 * ntri)                   # one leaf
    s = _with_mesh(get_scene("default"), wscene.HostBVH(pos, idx_dev, nodes))
    dev = wcpt.DeviceScene(gpu_ctx, s)
    gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, pairs)
    gpu_ctx.set_kernel(kernel)
    try:
        if path == "index":
            draws = np.zeros(1, dtype=wcpt._lib.DRAW_COMMAND_DTYPE)
            draws[0] = (gpu_ctx.buffer_address(dev.buffers[2]), gpu_ctx.buffer_address(dev.buffers[3]),
                        gpu_ctx.buffer_address(dev.buffers[4]), 3, 0)
            gpu_ctx.buffer_upload(dev.buffers[5], draws)
        W, H = 48, 40
        gpu_ctx.create_screen(W, H)
        sd = s.scene_data(W, H, max_bounce=2)
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        img = gpu_ctx.readback(H)
        pos_ref = np.concatenate([pos, np.full((1, 3), np.nan, np.float32)])
        idx_ref = idx.copy()
        idx_ref[3 * bad + 1] = pos.shape[0]
        ref, _ = oracle.render_scene(_with_mesh(s, wscene.HostBVH(pos_ref, idx_ref, nodes)), W, H, max_bounce=2,
                                     threads=8)
        assert_close(img, ref)
        full, _ = oracle.render_scene(_with_mesh(s, wscene.HostBVH(pos, idx, nodes)), W, H, max_bounce=2, threads=8)
        assert (full != ref).any(), "the test triangle must be visible"
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, -1)
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()


def test_buffer_range_checks_do_not_wrap(gpu_ctx):
    b = gpu_ctx.buffer_alloc(64)
    try:
        huge = (1 << 64) - 16
        with pytest.raises(wcpt.WcptError):
            gpu_ctx.buffer_download(b, 32, offset=huge)
        with pytest.raises(wcpt.WcptError):
            gpu_ctx.buffer_upload(b, np.zeros(32, np.uint8), offset=huge)
        assert gpu_ctx.buffer_size(b) == 64             # no grow to a wrapped size
    finally:
        gpu_ctx.buffer_free(b)


def _fat_leaf_bvh(nodes, min_tris=90, max_tris=600):
    """The same BVH with one interior node turned into a leaf over its whole (contiguous) subtree: a valid tree for
    the same triangles whose new leaf holds >= 255 index positions, outside what the wavefront's fast leaf layout was
    scanned for."""
    def span(i):
        n = nodes[i]
        if n["triangleCount"]:
            return int(n["leftNodeOrTriangleIndex"]), int(n["leftNodeOrTriangleIndex"] + n["triangleCount"])
        a0, a1 = span(int(n["leftNodeOrTriangleIndex"]))
        b0, b1 = span(int(n["leftNodeOrTriangleIndex"]) + 1)
        assert a1 == b0 or b1 == a0
        return min(a0, b0), max(a1, b1)
    for i in range(1, len(nodes)):
        n = nodes[i]
        if n["triangleCount"]:
            continue
        lo, hi = span(i)
        if min_tris * 3 <= hi - lo <= max_tris * 3:
            out = nodes.copy()
            out[i]["leftNodeOrTriangleIndex"] = lo
            out[i]["triangleCount"] = hi - lo
            return out, i
    raise AssertionError("no subtree of the wanted size")


def test_bvh_rewritten_behind_the_triangle_cache_stays_in_bounds(gpu_ctx):
    """the wavefront's fast leaf layout is chosen from a scan of the draw's BVH that the triangle cache
    keeps per buffer generation. A BVH rewritten by hipMemcpy (not wcpt_buffer_upload) with the cache on keeps the
    stale layout: the frame may be wrong (a leaf of >= 255 index positions no longer fits a stack entry), but every
    record load is bounded by the draw's records, so the render completes and reports no error. With the cache off,
    or after the same bytes go through wcpt_buffer_upload, the frame is the oracle's for the rewritten tree."""
    s = get_scene("atrium")
    W, H = 48, 27
    fat, node = _fat_leaf_bvh(s.meshes[0].nodes)
    assert fat[node]["triangleCount"] >= 255
    rewritten = _with_mesh(s, wscene.HostBVH(s.meshes[0].positions, s.meshes[0].indices, fat))
    ref, _ = oracle.render_scene(rewritten, W, H, max_bounce=4, threads=8)
    gpu_ctx.set_kernel(wcpt.KERNEL_WAVEFRONT)
    dev = wcpt.DeviceScene(gpu_ctx, s)
    try:
        gpu_ctx.create_screen(W, H)
        sd = s.scene_data(W, H, max_bounce=4)
        gpu_ctx.render(sd, *dev.addresses())            # the scan learns the original tree: fast layout
        gpu_ctx.sync()
        bvh_addr = gpu_ctx.buffer_address(dev.buffers[4])  # materials, spheres, vertices, indices, BVH, draws
        _device_write(bvh_addr, fat)                     # behind the cache
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()                                   # completes; no stack or memory fault
        stale = gpu_ctx.readback(H)
        assert np.isfinite(stale).all()
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 0)
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        assert_close(gpu_ctx.readback(H), ref)
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 1)
        gpu_ctx.buffer_upload(dev.buffers[4], fat)      # through the runtime: re-scanned, the general layout
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        assert_close(gpu_ctx.readback(H), ref)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 1)
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()


@pytest.mark.parametrize("name,expect", [("cornell", wcpt.KERNEL_MEGAKERNEL), ("reference_init", wcpt.KERNEL_MEGAKERNEL),
                                         ("atrium", wcpt.KERNEL_WAVEFRONT)])
def test_kernel_auto_picks_per_scene_and_renders_the_same_frames(gpu_ctx, name, expect):
    """WCPT_KERNEL_AUTO resolves per render from the draws' leaf layout: the megakernel where leaves hold several
    triangles (Cornell, the reference's mushroom), the wavefront kernel on the atrium's thin leaves -- the faster kernel
    on each bench scene -- and the frames equal the explicitly chosen kernel's bit for bit."""
    s = get_scene(name)
    W, H = 96, 64
    imgs = {}
    for k in (wcpt.KERNEL_AUTO, expect):
        with wcpt.Context(0) as ctx:
            dev = wcpt.DeviceScene(ctx, s)
            ctx.set_kernel(k)
            ctx.create_screen(W, H)
            for f in (0, 1):
                ctx.render(s.scene_data(W, H, max_bounce=3, frame=f), *dev.addresses())
            ctx.sync()
            imgs[k] = (ctx.readback(), ctx.last_kernel())
            dev.free()
    assert imgs[wcpt.KERNEL_AUTO][1] == expect and imgs[expect][1] == expect
    assert np.array_equal(imgs[wcpt.KERNEL_AUTO][0].view(np.uint32), imgs[expect][0].view(np.uint32))
    with wcpt.Context(0) as ctx:
        with pytest.raises(wcpt.WcptError):
            ctx.set_kernel(3)


def test_kernel_choice_without_draws_is_the_megakernel(gpu_ctx):
    """a render with no draw commands runs (and reports) the megakernel under WCPT_KERNEL_AUTO, and the
    explicitly chosen variant otherwise -- not the variant an earlier AUTO render resolved to."""
    import copy
    s = get_scene("atrium")
    spheres_only = copy.copy(get_scene("cornell"))
    spheres_only.meshes = []
    W, H = 32, 16
    with wcpt.Context(0) as ctx:
        dev = wcpt.DeviceScene(ctx, s)
        dev2 = wcpt.DeviceScene(ctx, spheres_only)
        ctx.create_screen(W, H)
        ctx.set_kernel(wcpt.KERNEL_AUTO)
        ctx.render(s.scene_data(W, H, max_bounce=2, frame=0), *dev.addresses())
        assert ctx.last_kernel() == wcpt.KERNEL_WAVEFRONT
        ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        ctx.render(spheres_only.scene_data(W, H, max_bounce=2, frame=0), *dev2.addresses())
        assert ctx.last_kernel() == wcpt.KERNEL_MEGAKERNEL
        ctx.set_kernel(wcpt.KERNEL_AUTO)
        ctx.render(s.scene_data(W, H, max_bounce=2, frame=0), *dev.addresses())
        assert ctx.last_kernel() == wcpt.KERNEL_WAVEFRONT
        ctx.render(spheres_only.scene_data(W, H, max_bounce=2, frame=0), *dev2.addresses())
        assert ctx.last_kernel() == wcpt.KERNEL_MEGAKERNEL
        ctx.set_kernel(wcpt.KERNEL_WAVEFRONT)
        ctx.render(spheres_only.scene_data(W, H, max_bounce=2, frame=0), *dev2.addresses())
        assert ctx.last_kernel() == wcpt.KERNEL_WAVEFRONT
        ctx.sync()
        dev.free()
        dev2.free()


@pytest.mark.parametrize("kernel", [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT])
def test_checkpoint_and_resume_progressive_accumulation(gpu_ctx, kernel):
    """Checkpoint / resume: the accumulation state is the float4 image plus renderedFramesCount. Read it
    back after frame 2, destroy the context, seed a new one with wcpt_image_upload and continue with frames 3 and 4:
    the image equals an uninterrupted sequence's, bit for bit."""
    s = get_scene("cornell")
    W, H = 80, 48
    sds = [s.scene_data(W, H, max_bounce=4, frame=f) for f in range(5)]
    with wcpt.Context(0) as a:
        dev = wcpt.DeviceScene(a, s)
        a.set_kernel(kernel)
        a.create_screen(W, H)
        for f in range(5):
            a.render(sds[f], *dev.addresses())
            if f == 2:
                a.sync()
                checkpoint = a.readback().copy()
        a.sync()
        whole = a.readback()
        dev.free()
    with wcpt.Context(0) as b:
        dev = wcpt.DeviceScene(b, s)
        b.set_kernel(kernel)
        b.create_screen(W, H)
        b.image_upload(checkpoint)
        for f in (3, 4):
            b.render(sds[f], *dev.addresses())
        b.sync()
        resumed = b.readback()
        dev.free()
    assert np.array_equal(resumed.view(np.uint32), whole.view(np.uint32))


def test_profile_region_times_the_renders_between_two_events(gpu_ctx):
    """WCPT_OPTION_PROFILE_REGION: one event pair brackets every render between wcpt_profile_begin and
    wcpt_profile_end (bench.py's N = 1 timing), launches counts the renders, and the interval covers at least the
    per-render pairs' sum; the option is refused inside a profiled region, and 0 restores a pair per render."""
    s = get_scene("cornell")
    W, H = 256, 128
    with wcpt.Context(0) as ctx:
        dev = wcpt.DeviceScene(ctx, s)
        ctx.create_screen(W, H)
        sds = [s.scene_data(W, H, max_bounce=4, frame=f) for f in range(6)]
        ctx.render(sds[0], *dev.addresses())
        ctx.sync()
        ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 0)
        ctx.profile_begin()
        for sd in sds:
            ctx.render(sd, *dev.addresses())
        per_ms, per_n = ctx.profile_end()
        ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 1)
        ctx.profile_begin()
        with pytest.raises(wcpt.WcptError):
            ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 0)
        for sd in sds:
            ctx.render(sd, *dev.addresses())
        reg_ms, reg_n = ctx.profile_end()
        assert per_n == reg_n == len(sds)
        assert per_ms > 0 and reg_ms > 0
        assert reg_ms >= 0.5 * per_ms  # same renders; the region adds the gaps and drops the per-render records
        ctx.profile_begin()  # a region with no render reports nothing
        assert ctx.profile_end() == (0.0, 0)
        ctx.set_option(wcpt._lib.OPTION_PROFILE_REGION, 0)
        dev.free()
