"""GPU parity: the HIP path (through the C-ABI of libwcpt.so) against the CPU oracle on identical inputs.

Tolerance (north_star "stated per-pixel float tolerance"): per channel |gpu - oracle| <= 1e-5
for at least 99.9 % of pixels and mean |gpu - oracle| <= 1e-4. The kernel is built to be bit-exact (same
IEEE binary32 operation order, no contraction, shared deterministic log/cos/exp), and the bit-exact pixel
fraction is asserted separately where noted. Work counters are integers and must match exactly.
"""
import numpy as np
import pytest

import wcpt
from wcpt import scene as wscene
from wcpt.dist import row_block
import oracle

pytestmark = pytest.mark.gpu

TOL_ABS = 1e-5
TOL_FRAC = 0.999
TOL_MEAN = 1e-4

_scenes = {}


def get_scene(name):
    if name not in _scenes:
        _scenes[name] = wscene.generate(name)
    return _scenes[name]


def assert_close(img, ref, exact=True):
    assert img.shape == ref.shape
    assert np.isfinite(ref).all() == np.isfinite(img).all()
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    diff = np.nan_to_num(diff, nan=np.inf)
    ok = (diff <= TOL_ABS).all(axis=2)
    frac = ok.mean()
    assert frac >= TOL_FRAC, f"only {frac:.5f} of pixels within {TOL_ABS}"
    finite = np.isfinite(diff)
    assert diff[finite].mean() <= TOL_MEAN
    if exact:
        same = (img.view(np.uint32) == ref.view(np.uint32)).all(axis=2).mean()
        assert same == 1.0, f"bit-exact fraction {same:.6f}"


def gpu_render(ctx, s, W, H, bounces=3, spp=1, frame=0, y0=0, rows=None, init=None, sd=None, kernel=None):
    dev = wcpt.DeviceScene(ctx, s)
    ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL if kernel is None else kernel)
    try:
        ctx.create_screen(W, H)
        ctx.set_row_range(y0, rows or 0)
        if sd is None:
            sd = s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=frame)
        if init is not None:
            ctx.image_upload(init)
        ctx.render(sd, *dev.addresses())
        ctx.sync()
        img = ctx.readback(rows or H)
        cnt = ctx.render_counters(sd, *dev.addresses())
    finally:
        ctx.set_row_range(0, 0)
        ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()
    return img, cnt


KERNELS = [wcpt.KERNEL_MEGAKERNEL, wcpt.KERNEL_WAVEFRONT]


# ---- device functions -----------------------------------------------------------------------------------
def test_device_pcg_and_rand(gpu_ctx):
    rng = np.random.default_rng(1)
    x = rng.integers(0, 2**32, 4096, dtype=np.uint64).astype(np.uint32)
    x[:5] = [0, 1, 2, 719393, 2073599]
    h = gpu_ctx.selftest(0, x)
    assert [int(v) for v in h[:5]] == [129708002, 2831084092, 2055130248, 1815429807, 2921424543]
    assert all(int(h[i]) == oracle.pcg_hash(int(x[i])) for i in range(0, 4096, 7))
    r = gpu_ctx.selftest(1, x[:512]).view(np.float32).reshape(-1, 4)
    for i in range(0, 512, 5):
        vals, _ = oracle.rand_stream(int(x[i]), 4)
        assert np.array_equal(r[i].view(np.uint32), vals.view(np.uint32))


@pytest.mark.parametrize("fn,lo,hi", [(2, 0.0, 1.0), (3, 0.0, 6.2831855), (4, -60.0, 0.0)])
def test_device_libm_bit_exact(gpu_ctx, fn, lo, hi):
    rng = np.random.default_rng(fn)
    x = rng.uniform(lo, hi, 20000).astype(np.float32)
    x[:4] = [lo, hi, np.float32(1.0), np.float32(0.5)]
    out = gpu_ctx.selftest(fn, x.view(np.uint32)).view(np.float32)
    f = {2: oracle.logf, 3: oracle.cosf, 4: oracle.expf}[fn]
    ref = np.array([f(float(v)) for v in x], np.float32)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_device_sqrt_div_ieee(gpu_ctx):
    rng = np.random.default_rng(7)
    a = (rng.standard_normal(50000) * 10.0 ** rng.uniform(-30, 30, 50000)).astype(np.float32)
    b = (rng.standard_normal(50000) * 10.0 ** rng.uniform(-30, 30, 50000)).astype(np.float32)
    s = gpu_ctx.selftest(5, np.abs(a).view(np.uint32)).view(np.float32)
    assert np.array_equal(s, np.sqrt(np.abs(a)))
    d = gpu_ctx.selftest(6, a.view(np.uint32), b.view(np.uint32)).view(np.float32)
    with np.errstate(all="ignore"):
        assert np.array_equal(d.view(np.uint32), (a / b).view(np.uint32))


def test_device_fast_reciprocal_exhaustive(gpu_ctx):
    """The kernels' reciprocal (v_rcp_f32 + one FMA Newton step on |x| in [2^-126, 2^126), IEEE division
    elsewhere) equals IEEE 1/x for ALL 2^32 binary32 inputs: the fast path is checked exhaustively on the
    device, the whole function on the boundary and special values against numpy."""
    hi = np.arange(65536, dtype=np.uint32)
    bad = gpu_ctx.selftest(8, hi)
    assert int(bad.sum()) == 0, f"fast reciprocal differs from IEEE on {int(bad.sum())} inputs"
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.1754942e-38, 1.17549435e-38,
                        2.0 ** -126, 2.0 ** 126, 8.5070587e37, 3.4028235e38, -3.4028235e38, 1.0, -1.0, 3.0, 0.1,
                        2.0 ** 125, 2.0 ** -125, 5.877472e-39, 9.860761e-32], np.float32)
    rng = np.random.default_rng(4)
    rand = rng.integers(0, 2**32, 20000, dtype=np.uint64).astype(np.uint32).view(np.float32)
    x = np.concatenate([special, rand])
    got = gpu_ctx.selftest(9, x.view(np.uint32)).view(np.float32)
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        ref = (np.float32(1.0) / x).astype(np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    assert np.array_equal(got[~nan].view(np.uint32), ref[~nan].view(np.uint32))


def test_device_reciprocal_result_check_exhaustive(gpu_ctx):
    """The kernels validate the fast reciprocal on its result class (pt_device.h rcp_exact / rcp2_exact): over
    ALL 2^32 inputs, in the scalar form and in both halves of the packed pair form, the result is IEEE 1/x
    (fn 12), and the general division runs exactly for the inputs outside [2^-126, 2^126] (fn 13): zeros and
    denormals (exponent field 0), |x| in (2^126, 2^128), infinities and NaNs (exponent fields 253..255 minus the
    two patterns +-2^126, whose quotient +-2^-126 is normal): 2 * 4 * 2^23 - 2 = 2^26 - 2 bit patterns."""
    hi = np.arange(65536, dtype=np.uint32)
    bad = gpu_ctx.selftest(12, hi)
    assert int(bad.sum()) == 0, f"reciprocal differs from IEEE on {int(bad.sum())} inputs"
    slow = int(gpu_ctx.selftest(13, hi).astype(np.uint64).sum())
    assert slow == 2 ** 26 - 2


def test_device_sqrt_exhaustive(gpu_ctx):
    """The kernels' square root (pt_device.h sqrt_exact: the 9-VALU correction core for x >= 2^-96, hipcc's full
    sequence elsewhere) equals hipcc's correctly rounded sqrtf on ALL 2^32 inputs (fn 15); test_device_sqrt_div_ieee
    checks it against numpy on random magnitudes."""
    bad = gpu_ctx.selftest(15, np.arange(65536, dtype=np.uint32))
    assert int(bad.sum()) == 0, f"sqrt differs on {int(bad.sum())} inputs, first high halves {np.nonzero(bad)[0][:8]}"


def test_device_acceptance_forms_agree(gpu_ctx):
    """accept_tri (four compares, the reference's :132 minus the implied u <= 1) and accept_tri_w (minimum3 form
    used by the pair test) decide identically on special and random (u, v)."""
    special = np.array([0.0, -0.0, 1.0, -1.0, 0.5, 1e-45, -1e-45, 1.0000001, 0.99999994, 0.49999997, 0.50000006,
                        np.inf, -np.inf, np.nan, -np.nan, 3.4028235e38, -3.4028235e38, 2.0, 1e-30, -1e-30],
                       np.float32)
    uu, vv = np.meshgrid(special, special)
    rng = np.random.default_rng(14)
    ru = rng.uniform(-0.2, 1.2, 200000).astype(np.float32)
    rv = rng.uniform(-0.2, 1.2, 200000).astype(np.float32)
    # near the u + v = 1 edge: v = 1 - u and its neighbours
    eu = rng.uniform(0.0, 1.0, 100000).astype(np.float32)
    ev = (np.float32(1.0) - eu).view(np.uint32) + rng.integers(-2, 3, 100000).astype(np.int64).astype(np.uint32)
    u = np.concatenate([uu.ravel(), ru, eu])
    v = np.concatenate([vv.ravel(), rv, ev.view(np.float32)])
    out = gpu_ctx.selftest(14, u.view(np.uint32), v.view(np.uint32))
    assert np.array_equal(out & 1, out >> 1), f"{int(((out & 1) != (out >> 1)).sum())} disagreements"
    assert int((out & 1).sum()) > 1000  # both accepting and rejecting cases are exercised
    assert int((out & 1).sum()) < u.size


def test_device_integer_take_exhaustive(gpu_ctx):
    """The integer form of the triangle take (pt_device.h take_bits, WCPT_PAIR_ITAKE): for rec.t any positive float the
    kernel can hold (kInfinity, the largest floats, ordinary distances, the smallest normal and denormal values, +inf),
    `t > 0 && t < rec.t` equals `bits(t) - 1 < bits(rec.t) - 1` on ALL 2^32 t (zeros, denormals, negatives, NaNs)."""
    rts = np.array([3.402823466e38, 3.4028233e38, np.inf, 1.0, 0.5, 2.0, 1e-3, 7.25, 123456.0, 1.1754944e-38,
                    1.4e-45, 2.8e-45, 1e-40], np.float32)
    hi = np.arange(65536, dtype=np.uint32)
    for rt in rts:
        bad = gpu_ctx.selftest(17, hi, np.full(hi.size, rt, np.float32).view(np.uint32))
        assert int(bad.sum()) == 0, f"rec.t {rt}: the forms differ on {int(bad.sum())} t"


def test_device_random_direction(gpu_ctx):
    x = np.arange(1000, dtype=np.uint32) * 2654435761
    out = gpu_ctx.selftest(7, x).view(np.float32).reshape(-1, 3)
    for i in range(0, 1000, 9):
        d, _ = oracle.random_direction(int(x[i]))
        assert np.array_equal(out[i].view(np.uint32), d.view(np.uint32))


# ---- whole frames ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name,W,H,bounces,spp", [
    ("default", 64, 64, 3, 1),
    ("default_dielectric", 64, 64, 3, 1),
    ("default_emissive", 64, 48, 3, 2),
    ("cornell", 256, 256, 1, 1),        # BASELINE config 1
    ("cornell", 128, 96, 4, 1),
    ("cornell", 67, 45, 4, 3),          # ragged: not a multiple of the 8x8 tile
    ("atrium", 96, 54, 4, 1),
    ("reference_init", 96, 54, 3, 1),        # the reference's own Init scene (mushroom.obj), start camera
    ("reference_init_glass", 96, 54, 3, 2),  # ... with material 0 made DIELECTRIC (Appendix A item 2)
])
@pytest.mark.parametrize("kernel", KERNELS)
def test_frame_parity(gpu_ctx, name, W, H, bounces, spp, kernel):
    s = get_scene(name)
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("stack", [0, 1])
def test_stack_kinds_match_oracle(gpu_ctx, stack, kernel):
    """Every traversal-stack implementation (scratch, LDS + spill) gives the oracle's image and counters."""
    s = get_scene("atrium")
    gpu_ctx.set_option(wcpt._lib.OPTION_STACK, stack)
    init = np.full((64, 120, 4), 0.5, np.float32)
    try:
        img, cnt = gpu_render(gpu_ctx, s, 120, 64, bounces=4, frame=1, init=init, kernel=kernel)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_STACK, 1)
    ref, rcnt = oracle.render_scene(s, 120, 64, max_bounce=4, frame=1, image=init, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
def test_progressive_accumulation(gpu_ctx, kernel):
    """renderedFramesCount > 0 mixes into the existing image (pathTracer.comp:314-318)."""
    s = get_scene("default_dielectric")
    W, H = 48, 40
    rng = np.random.default_rng(3)
    init = rng.uniform(0, 1, (H, W, 4)).astype(np.float32)
    for frame in (1, 7, 1000):
        img, _ = gpu_render(gpu_ctx, s, W, H, bounces=3, frame=frame, init=init, kernel=kernel)
        ref, _ = oracle.render_scene(s, W, H, max_bounce=3, frame=frame, image=init)
        assert_close(img, ref)


@pytest.mark.parametrize("kernel", KERNELS)
def test_row_block_shards_equal_full_frame(gpu_ctx, kernel):
    """the union of row blocks is bit-identical to the full-frame render."""
    s = get_scene("cornell")
    W, H = 80, 72
    full, _ = gpu_render(gpu_ctx, s, W, H, bounces=4, kernel=kernel)
    parts = []
    for r in range(3):
        y0, rows = row_block(H, 3, r)
        img, _ = gpu_render(gpu_ctx, s, W, H, bounces=4, y0=y0, rows=rows, kernel=kernel)
        parts.append(img)
    assert np.array_equal(np.concatenate(parts), full)


@pytest.mark.parametrize("kernel", KERNELS)
def test_full_size_rows_vs_oracle(gpu_ctx, kernel):
    """BASELINE config 2 at full size (1920x1080, 4 bounces): oracle on sampled row bands of the same frame."""
    s = get_scene("cornell")
    W, H = 1920, 1080
    init = np.zeros((H, W, 4), np.float32)
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=4, frame=5, init=init, kernel=kernel)
    assert cnt["pixels"] == W * H
    assert cnt["segments"] <= W * H * 5
    for y0 in (0, 333, 540, 1072):
        ref, _ = oracle.render_scene(s, W, H, max_bounce=4, frame=5, y0=y0, rows=8, threads=8)
        assert_close(img[y0:y0 + 8], ref)


def test_deterministic_repeat(gpu_ctx):
    s = get_scene("atrium")
    init = np.full((90, 160, 4), 0.25, np.float32)
    a, ca = gpu_render(gpu_ctx, s, 160, 90, bounces=4, frame=2, init=init)
    b, cb = gpu_render(gpu_ctx, s, 160, 90, bounces=4, frame=2, init=init)
    assert np.array_equal(a, b) and ca == cb


def test_renderer_mirror_frame_sequence(gpu_ctx):
    """Drive the PathTracingRenderer mirror like the editor (Init, CreateScreen, Render x3, Resize, Render)."""
    r = wcpt.PathTracingRenderer(0)
    try:
        s = get_scene("default")
        r.Init(scene=s)
        r.CreateScreen((40, 32))
        cam = wscene.update_camera(s.camera, 40 / 32)
        images = []
        for _ in range(3):
            r.Render(cam)
            images.append(r.Readback())
        assert r.renderedFramesCount == 3
        img0 = None
        acc = None
        for f in range(3):
            sd = s.scene_data(40, 32, max_bounce=3, frame=f)
            acc, _ = oracle.render_scene(s, 40, 32, sd=sd, image=acc)
            if img0 is None:
                img0 = acc
            assert_close(images[f], acc)
        r.Resize((24, 16))
        assert r.renderedFramesCount == 0
        r.Render(wscene.update_camera(s.camera, 24 / 16))
        ref, _ = oracle.render_scene(s, 24, 16, max_bounce=3, frame=0)
        assert_close(r.Readback(), ref)
    finally:
        r.Deinit()


def test_errors(gpu_ctx):
    ctx = wcpt.Context(0)
    try:
        s = get_scene("default")
        sd = s.scene_data(8, 8)
        with pytest.raises(wcpt.WcptError) as e:
            ctx.render(sd, 0, 0, 0)
        assert e.value.code == -1003           # WCPT_ERROR_NO_SCREEN
        with pytest.raises(wcpt.WcptError) as e:
            ctx.buffer_upload(12345, np.zeros(4, np.float32))
        assert e.value.code == -1001           # WCPT_ERROR_INVALID_HANDLE
        ctx.create_screen(8, 8)
        with pytest.raises(wcpt.WcptError):
            ctx.render(sd, 0, 0, 0)            # sphereCount > 0 with null buffers
        b = ctx.buffer_alloc(16)
        ctx.buffer_upload(b, np.arange(8, dtype=np.float32))   # grows 16 -> 32 bytes
        assert ctx.buffer_size(b) == 32
        assert np.frombuffer(ctx.buffer_download(b, 32), np.float32).tolist() == list(range(8))
        ctx.buffer_free(b)
    finally:
        ctx.close()


def test_golden_fixtures(gpu_ctx):
    """GPU against the committed oracle goldens (tests/golden/, made by tests/golden/make_golden.py)."""
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "images.npz")
    gold = np.load(path)
    from golden_cases import CASES
    for key, (name, W, H, bounces, spp, frames) in CASES.items():
        s = get_scene(name)
        acc = None
        for f in frames:
            img, _ = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=f, init=acc)
            acc = img
        ref = gold[key]
        assert_close(acc[..., :3].copy(), ref)


# ---- derived triangle records (wcpt.h WCPT_OPTION_TRIANGLE_CACHE) -------------------------------------------
def _with_mesh(s, mesh):
    import copy
    d = copy.copy(s)
    d.meshes = [mesh]
    return d


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("cache", [1, 0])
def test_triangle_records_follow_reuploads(gpu_ctx, kernel, cache):
    """Re-uploading the vertex buffer must re-derive the records: the second frame renders the moved geometry
    (the BVH is left as it was, which the oracle traverses identically)."""
    s = get_scene("cornell")
    W, H = 64, 48
    dev = wcpt.DeviceScene(gpu_ctx, s)
    gpu_ctx.set_kernel(kernel)
    gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, cache)
    try:
        gpu_ctx.create_screen(W, H)
        sd = s.scene_data(W, H, max_bounce=3)
        for step in range(3):
            m = s.meshes[0]
            pos = m.positions + np.float32(0.05 * step)
            gpu_ctx.buffer_upload(dev.buffers[2], np.ascontiguousarray(pos, dtype=np.float32))
            gpu_ctx.render(sd, *dev.addresses())
            gpu_ctx.sync()
            img = gpu_ctx.readback(H)
            moved = _with_mesh(s, wscene.HostBVH(np.ascontiguousarray(pos, dtype=np.float32), m.indices, m.nodes))
            ref, _ = oracle.render_scene(moved, W, H, max_bounce=3, threads=8)
            assert_close(img, ref)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_TRIANGLE_CACHE, 1)
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()


@pytest.mark.parametrize("kernel", KERNELS)
def test_leaf_not_on_triangle_boundary(gpu_ctx, kernel):
    """A hand-made BVH whose leaves start at index positions that are not multiples of 3, and a draw whose
    indexCount covers fewer triangles than the leaves reference: both take the index path and must still
    equal the oracle (the reference kernel reads indices[first + i .. + 2] whatever `first` is)."""
    rng = np.random.default_rng(7)
    ntri = 40
    pos = (rng.random((ntri * 3, 3), dtype=np.float32) * 2.0 - 1.0).astype(np.float32)
    pos[:, 2] -= 3.0
    idx = np.arange(ntri * 3 + 2, dtype=np.uint32) % (ntri * 3)
    lo, hi = pos.min(axis=0), pos.max(axis=0)
    nodes = np.zeros(3, dtype=wcpt._lib.NODE_DTYPE)
    nodes[0] = (lo, hi, 1, 0)                         # interior: children 1, 2
    nodes[1] = (lo, hi, 1, 60)                        # leaf starting at index position 1 (not a multiple of 3)
    nodes[2] = (lo, hi, 63, 3 * ntri - 63)            # leaf starting at 63 (aligned), beyond indexCount below
    s = get_scene("default")
    mesh = wscene.HostBVH(pos, idx, nodes)
    scene = _with_mesh(s, mesh)
    W, H = 48, 40
    dev = wcpt.DeviceScene(gpu_ctx, scene)
    try:
        draws = np.zeros(1, dtype=wcpt._lib.DRAW_COMMAND_DTYPE)
        draws[0] = (gpu_ctx.buffer_address(dev.buffers[2]), gpu_ctx.buffer_address(dev.buffers[3]),
                    gpu_ctx.buffer_address(dev.buffers[4]), 30, 0)   # indexCount: only 10 triangles
        gpu_ctx.buffer_upload(dev.buffers[5], draws)
        gpu_ctx.set_kernel(kernel)
        gpu_ctx.create_screen(W, H)
        sd = scene.scene_data(W, H, max_bounce=2)
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        img = gpu_ctx.readback(H)
        cnt = gpu_ctx.render_counters(sd, *dev.addresses())
        ref, rcnt = oracle.render_scene(scene, W, H, max_bounce=2, threads=8)
        assert_close(img, ref)
        assert cnt == rcnt
        assert rcnt["triangle_tests"] > 0 and rcnt["hits"] > 0
    finally:
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()


@pytest.mark.parametrize("pairs", [0, 1])
@pytest.mark.parametrize("name,W,H", [("cornell", 80, 64), ("atrium", 64, 40), ("default", 48, 40)])
def test_record_formats_match_oracle(gpu_ctx, pairs, name, W, H):
    """Megakernel leaf tests on single records and on packed pair records: both equal the oracle."""
    s = get_scene(name)
    gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, pairs)
    try:
        img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=3)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, -1)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=3, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("pairs", [0, 1])
@pytest.mark.parametrize("combo", ["atrium_twice", "cornell_then_atrium"])
def test_multi_draw_deep_trees_match_oracle(gpu_ctx, kernel, pairs, combo):
    """Several draw commands over deep BVHs (:151-201: the next draw's traversal starts with the stack of the previous
    one exhausted, closest hit over all of them, ties to the earlier draw). The megakernel walks multiple draws in
    one flat traversal loop; the atrium's 27-level midpoint tree drives its stacks into the scratch spill."""
    import copy
    s = copy.copy(get_scene("atrium"))
    atrium = s.meshes[0]
    s.meshes = [atrium, atrium] if combo == "atrium_twice" else [get_scene("cornell").meshes[0], atrium]
    W, H = 48, 32
    gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, pairs)
    try:
        img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=3, kernel=kernel)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, -1)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=3, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


def test_primary_records_follow_the_camera(gpu_ctx):
    """The megakernel tests a sample's first segment against primary-ray pair records derived for the camera
    position (pt_device.h TriPairP). They are cached per position: moving the camera between frames of one context,
    moving it back, and re-uploading the mesh at a fixed camera must each give the oracle's frame (2 spp: every
    sample's first segment starts at the camera)."""
    import copy
    import ctypes
    s = get_scene("cornell")
    W, H = 48, 40
    cams = []
    for dx in (0.0, 0.35, 0.0):
        cam = wcpt.Camera()
        ctypes.pointer(cam)[0] = s.camera
        cam.position[0] += dx
        cam.position[1] += dx * 0.5
        cams.append(cam)
    dev = wcpt.DeviceScene(gpu_ctx, s)
    gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
    gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, 1)
    try:
        gpu_ctx.create_screen(W, H)
        for f, cam in enumerate(cams + [cams[-1]]):
            if f == 3:  # same camera, mesh re-uploaded: the pair records are rebuilt, the primary records follow
                m = s.meshes[0]
                gpu_ctx.buffer_upload(dev.buffers[2], np.ascontiguousarray(m.positions, dtype=np.float32))
            sd = s.scene_data(W, H, max_bounce=3, samples=2, frame=0, camera=cam)
            gpu_ctx.render(sd, *dev.addresses())
            gpu_ctx.sync()
            img = gpu_ctx.readback()
            ref, _ = oracle.render_scene(copy.copy(s), W, H, sd=sd, threads=8)
            assert_close(img, ref)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, -1)
        dev.free()


@pytest.mark.parametrize("pairs", [0, 1])
@pytest.mark.parametrize("stack", [0, 1])
def test_megakernel_atrium_rows_all_modes(gpu_ctx, pairs, stack):
    """A 1920-wide atrium band through the render, counting and diagnostic megakernel builds (the diagnostic build
    adds wave-level ballots inside the traversal): none may report a stack overflow, the render must equal the
    oracle and the counters of both counting builds must agree. Regression test for the toolchain mis-compile of
    the nested draw loop."""
    s = get_scene("atrium")
    W, H, y0, rows = 1920, 1080, 520, 8
    gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, pairs)
    gpu_ctx.set_option(wcpt._lib.OPTION_STACK, stack)
    dev = wcpt.DeviceScene(gpu_ctx, s)
    try:
        gpu_ctx.create_screen(W, H)
        gpu_ctx.set_row_range(y0, rows)
        sd = s.scene_data(W, H, max_bounce=4, samples=1, frame=0)
        gpu_ctx.render(sd, *dev.addresses())
        gpu_ctx.sync()
        img = gpu_ctx.readback(rows)
        cnt = gpu_ctx.render_counters(sd, *dev.addresses())
        dcnt = gpu_ctx.render_counters(sd, *dev.addresses(), diagnostics=True)
    finally:
        gpu_ctx.set_row_range(0, 0)
        gpu_ctx.set_option(wcpt._lib.OPTION_PAIR_RECORDS, -1)
        gpu_ctx.set_option(wcpt._lib.OPTION_STACK, 1)
        dev.free()
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=4, y0=y0, rows=rows, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt
    assert {k: dcnt[k] for k in cnt} == cnt


# ---- composite.comp (display step) ---------------------------------------------------
@pytest.mark.parametrize("rgba8", [False, True])
def test_composite_matches_oracle(gpu_ctx, rgba8):
    """Device gamma + PBR Neutral tonemap equals the oracle bit-for-bit, on a rendered frame and on synthetic HDR
    values covering the tonemap's branches (x < 0.08, peak < 0.76, compression, > 1, 0, NaN, inf, negative)."""
    rng = np.random.default_rng(11)
    W, H = 72, 40
    s = get_scene("cornell")
    img, _ = gpu_render(gpu_ctx, s, W, H, bounces=3)
    hdr = np.ones((H, W, 4), np.float32)
    hdr[..., :3] = (rng.random((H, W, 3)) ** 4 * 16.0).astype(np.float32)
    hdr[0, :6, :3] = [[0, 0, 0], [1, 1, 1], [np.nan, 0.5, 0.5], [np.inf, 0, 0], [-1, 0.2, 0.2], [0.05, 0.07, 0.9]]
    nbytes = W * H * (4 if rgba8 else 16)
    buf = gpu_ctx.buffer_alloc(nbytes)
    try:
        gpu_ctx.create_screen(W, H)
        for src in (img, hdr):
            gpu_ctx.image_upload(src)
            gpu_ctx.composite(gpu_ctx.buffer_address(buf), rgba8=rgba8)
            gpu_ctx.sync()
            raw = gpu_ctx.buffer_download(buf, nbytes)
            ref32, ref8 = oracle.composite(src)
            if rgba8:
                assert np.array_equal(np.frombuffer(raw, np.uint8).reshape(H, W, 4), ref8)
            else:
                got = np.frombuffer(raw, np.float32).reshape(H, W, 4)
                nan = np.isnan(ref32)
                assert np.array_equal(np.isnan(got), nan)   # NaN payloads are not compared (x86 vs AMD)
                assert np.array_equal(got.view(np.uint32)[~nan], ref32.view(np.uint32)[~nan])
    finally:
        gpu_ctx.buffer_free(buf)


def test_editor_frame_sequence(gpu_ctx):
    """The editor's frame protocol (editor.jai:149-158 + PathTracingRenderer.jai:423): still camera -> the shader
    sees 1, 3, 5; after a move 0, 2, 4. Each accumulated frame equals the oracle fed the same counts."""
    s = get_scene("default")
    W, H = 32, 24
    r = wcpt.PathTracingRenderer(0)
    try:
        r.Init(scene=s)
        r.CreateScreen((W, H))
        ed = wcpt.Editor(r, s.camera)
        moves = [False, False, False, True, False, False]
        used = []
        acc = None
        for mv in moves:
            used.append(ed.frame(moved=mv))
            got = r.Readback()
            sd = s.scene_data(W, H, max_bounce=r.maxBounceCount, frame=used[-1])
            acc, _ = oracle.render_scene(s, W, H, sd=sd, image=acc)
            assert_close(got, acc)
        assert used == [1, 3, 5, 0, 2, 4]
    finally:
        r.Deinit()


def test_c_host_editor_loop(gpu_ctx, tmp_path):
    """examples/editor_loop (plain C over include/wcpt.h) runs the editor protocol with a camera move at frame 2
    and writes the composited RGBA8 frame; its frame counts and pixels equal the oracle's for the same sequence."""
    import ctypes as C
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "editor_loop")
    if not os.path.exists(exe):
        subprocess.run(["make"], cwd=os.path.join(root, "examples"), check=True)
    W, H, frames, move_at = 48, 32, 5, 2
    out = tmp_path / "f.ppm"
    p = subprocess.run([exe, "cornell", str(W), str(H), str(frames), str(out), "--move-at", str(move_at)],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    used = [int(line.split()[3]) for line in p.stdout.splitlines() if line.startswith("frame ")]
    assert used == [1, 3, 0, 2, 4]
    data = out.read_bytes()
    header = f"P6\n{W} {H}\n255\n".encode()
    assert data.startswith(header)
    rgb = np.frombuffer(data[len(header):], np.uint8).reshape(H, W, 3)
    # the same sequence on the oracle (scene without the OBJ round trip, as the C host builds it)
    s = wscene.generate("cornell", via_obj=False)
    cam = wcpt.Camera()
    C.pointer(cam)[0] = s.camera
    acc = None
    for f, n in enumerate(used):
        if f == move_at:
            cam.yaw += 1.0
        sd = s.scene_data(W, H, max_bounce=3, samples=1, frame=n, camera=cam)
        acc, _ = oracle.render_scene(s, W, H, sd=sd, image=acc)
    _, ref8 = oracle.composite(acc)
    assert np.array_equal(rgb, ref8[..., :3])


# ---- edge cases of the inputs -------------------------------------------------------------------------------
def _variant(name, kind):
    import copy
    s = copy.copy(get_scene(name))
    if kind == "no_spheres":
        s.spheres = s.spheres[:0]
    elif kind == "no_meshes":
        s.meshes = []
    elif kind == "empty":
        s.spheres = s.spheres[:0]
        s.meshes = []
    elif kind == "two_draws":          # the same mesh drawn twice: exercises the per-draw loop (:152-201)
        s.meshes = [s.meshes[0], s.meshes[0]]
    elif kind == "all_dielectric":     # type 1 everywhere, with absorption (:263-280)
        m = s.materials.copy()
        m["type"] = 1
        m["ior"] = 1.5
        m["absorptionStrength"] = 0.7
        m["absorption"] = [0.2, 0.5, 0.9]
        s.materials = m
    return s


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("kind,bounces,spp", [
    ("no_spheres", 3, 1), ("no_meshes", 3, 1), ("empty", 3, 1), ("two_draws", 3, 1),
    ("all_dielectric", 6, 2), ("base", 0, 1), ("base", 12, 1), ("base", 3, 0),
])
def test_edge_inputs_match_oracle(gpu_ctx, kernel, kind, bounces, spp):
    """Empty sphere / draw lists, an empty scene (sky only), two draw commands, dielectric everywhere,
    maxBounceCount 0 and 12, and samples = 0 (the reference divides by zero: NaN pixels, :312)."""
    s = get_scene("cornell") if kind == "base" else _variant("cornell", kind)
    W, H = 40, 24
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, threads=8)
    if spp == 0:
        assert np.isnan(ref[..., :3]).all() and np.isnan(img[..., :3]).all()
        assert np.array_equal(img[..., 3], ref[..., 3])
    else:
        assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("bounces,spp", [(0, 1), (2, 2), (4, 1), (3, 3)])
def test_last_segment_shortcuts_match_oracle(gpu_ctx, kernel, bounces, spp):
    """The last segment of a pixel's last sample ends after its emission term (WCPT_LAST_SEGMENT_SHORTCUT) and the
    wavefront traces it as any-hit (WCPT_WF_ANYHIT_LAST): exact only because every triangle carries material 0
    (:175). Material 0 is made emissive here, so the triangle answer of that segment reaches the image, and
    samples > 1 checks that only the last sample takes the shortcut (its RNG state feeds the next sample)."""
    import copy
    s = copy.copy(get_scene("cornell"))
    m = s.materials.copy()
    m["emission"][0] = (0.3, 0.2, 0.1)
    m["emissionStrength"][0] = 1.5
    s.materials = m
    W, H = 48, 40
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("refs", [1, 0])
def test_stack_refs_match_oracle(gpu_ctx, kernel, refs):
    """Stack entries carrying (left, count) (default) or node indices: same frame, same counters. The hand-made
    BVH below has fat leaves (count 300 >= 255 index units) as deferred children: the packed form's fetch escape."""
    rng = np.random.default_rng(5)
    ntri = 200
    pos = (rng.random((ntri * 3, 3), dtype=np.float32) * 2.0 - 1.0).astype(np.float32)
    pos[:, 2] -= 3.0
    idx = np.arange(ntri * 3, dtype=np.uint32)
    lo0, hi0 = pos[:300].min(axis=0), pos[:300].max(axis=0)
    lo1, hi1 = pos[300:].min(axis=0), pos[300:].max(axis=0)
    nodes = np.zeros(3, dtype=wcpt._lib.NODE_DTYPE)
    nodes[0] = (np.minimum(lo0, lo1), np.maximum(hi0, hi1), 1, 0)
    nodes[1] = (lo0, hi0, 0, 300)
    nodes[2] = (lo1, hi1, 300, 300)
    fat = _with_mesh(get_scene("default"), wscene.HostBVH(pos, idx, nodes))
    gpu_ctx.set_option(wcpt._lib.OPTION_PACKED_REFS, refs)
    try:
        for s, (W, H) in ((get_scene("atrium"), (64, 40)), (get_scene("cornell"), (48, 32)), (fat, (48, 40))):
            img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=3, kernel=kernel)
            ref, rcnt = oracle.render_scene(s, W, H, max_bounce=3, threads=8)
            assert_close(img, ref)
            assert cnt == rcnt
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_PACKED_REFS, 1)


@pytest.mark.parametrize("refill", [1, 12, 20, 64])
def test_wavefront_refill_thresholds(gpu_ctx, refill):
    """The wavefront trace's refill threshold changes only the order rays are processed in."""
    s = get_scene("atrium")
    gpu_ctx.set_option(wcpt._lib.OPTION_WF_REFILL, refill)
    try:
        img, cnt = gpu_render(gpu_ctx, s, 80, 48, bounces=4, kernel=wcpt.KERNEL_WAVEFRONT)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_REFILL, wcpt._lib.DEFAULT_WF_REFILL)
    ref, rcnt = oracle.render_scene(s, 80, 48, max_bounce=4, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
def test_sah_bvh_frames(gpu_ctx, kernel):
    """The optional SAH tree through the same kernels: bit-exact against the oracle on the same tree, and equal to
    the midpoint tree's image except where triangles tie in t (a few pixels at most), with far fewer node visits."""
    mid = get_scene("atrium")
    if "atrium_sah" not in _scenes:
        _scenes["atrium_sah"] = wscene.generate("atrium", bvh="sah")
    sah = _scenes["atrium_sah"]
    W, H = 96, 54
    img, cnt = gpu_render(gpu_ctx, sah, W, H, bounces=4, kernel=kernel)
    ref, rcnt = oracle.render_scene(sah, W, H, max_bounce=4, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt
    img_mid, cnt_mid = gpu_render(gpu_ctx, mid, W, H, bounces=4, kernel=kernel)
    differ = (img.view(np.uint32) != img_mid.view(np.uint32)).any(axis=2).mean()
    assert differ <= 0.01, f"{differ:.4f} of pixels differ between SAH and midpoint trees"
    assert cnt["segments"] == cnt_mid["segments"] or differ > 0
    assert cnt["interior_visits"] < cnt_mid["interior_visits"]


# ---- randomized scenes ------------------------------------------------------------------------------------
def _random_scene(seed):
    """Random materials (metal and dielectric, emissive, rough), spheres (overlapping, camera possibly inside
    one), 1-2 triangle meshes of random size with the midpoint BVH, and a random camera."""
    rng = np.random.default_rng(seed)
    nm = int(rng.integers(1, 6))
    mats = np.zeros(nm, dtype=wcpt.MATERIAL_DTYPE)
    mats["type"] = rng.integers(0, 2, nm)
    mats["albedo"] = rng.random((nm, 3))
    mats["emission"] = rng.random((nm, 3))
    mats["emissionStrength"] = rng.random(nm) * rng.integers(0, 2, nm) * 4.0
    mats["roughness"] = rng.random(nm) * rng.integers(0, 2, nm)
    mats["absorption"] = rng.random((nm, 3))
    mats["absorptionStrength"] = rng.random(nm) * 2.0
    mats["ior"] = 1.0 + rng.random(nm) * 1.5
    ns = int(rng.integers(0, 7))
    sph = np.zeros(ns, dtype=wcpt.SPHERE_DTYPE)
    sph["position"] = (rng.random((ns, 3)) * 6.0 - 3.0).astype(np.float32)
    sph["radius"] = (0.2 + rng.random(ns) * 1.5).astype(np.float32)
    sph["material"] = rng.integers(0, nm, ns)
    meshes = []
    for _ in range(int(rng.integers(0, 3))):
        nt = int(rng.integers(1, 400))
        centers = rng.random((nt, 1, 3)) * 6.0 - 3.0
        pos = (centers + (rng.random((nt, 3, 3)) - 0.5) * rng.random() * 2.0).reshape(-1, 3).astype(np.float32)
        idx = np.arange(nt * 3, dtype=np.uint32)
        rng.shuffle(idx.reshape(-1, 3))
        meshes.append(wscene.bvh_build(wscene.HostMesh(pos, idx)))
    cam = wscene.make_camera(position=tuple((rng.random(3) * 6.0 - 3.0).tolist()), yaw=float(rng.random() * 360.0),
                             pitch=float(rng.random() * 120.0 - 60.0), fov=float(30.0 + rng.random() * 90.0))
    s = wscene.HostScene(f"random{seed}", mats, sph, cam)
    s.meshes = meshes
    return s, int(rng.integers(0, 7)), int(rng.integers(1, 4)), int(rng.integers(0, 50))


@pytest.mark.parametrize("seed", list(range(12)))
@pytest.mark.parametrize("kernel", KERNELS)
def test_random_scenes_match_oracle(gpu_ctx, seed, kernel):
    s, bounces, spp, frame = _random_scene(seed)
    W, H = 40, 28
    init = np.random.default_rng(seed + 100).random((H, W, 4)).astype(np.float32)
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=frame, init=init, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=frame, image=init, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("order", [0, 1, 3, 5])
@pytest.mark.parametrize("name,W,H,bounces,spp,rows", [
    ("cornell", 67, 45, 4, 3, None), ("atrium", 96, 54, 4, 1, None), ("cornell", 1920, 1080, 4, 1, 135),
    ("reference_init", 64, 72, 3, 2, None)])   # 8 x 9 tiles: a multiple of 8, tile rows not
def test_tile_orders_match_oracle(gpu_ctx, order, name, W, H, bounces, spp, rows):
    """WCPT_OPTION_MK_TILE_ORDER 0 (XCD bands), 1 (scattered), 3 and 5 (XCD bands striped by 1 and 4 tile rows) change only which
    wave renders which tile: every tile exactly once, same image and counters as the oracle."""
    s = get_scene(name)
    gpu_ctx.set_option(wcpt._lib.OPTION_MK_TILE_ORDER, order)
    try:
        img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=1, rows=rows,
                              init=np.zeros((rows or H, W, 4), np.float32))
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_MK_TILE_ORDER, 2)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=1, rows=rows, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt


@pytest.mark.parametrize("pipes", [1, 2, 3, 4])
@pytest.mark.parametrize("name,W,H,bounces,spp,frame,rows", [
    ("cornell", 67, 45, 4, 3, 0, None),     # ragged, several samples per pixel
    ("atrium", 96, 54, 4, 1, 2, None),
    ("default_dielectric", 48, 40, 3, 2, 7, None),
    ("atrium", 200, 120, 4, 1, 1, 40),      # a row block
    ("cornell", 24, 8, 2, 1, 0, None),      # 3 tiles: fewer tiles than pipelines at 4
])
def test_wavefront_pipelines_match_oracle(gpu_ctx, pipes, name, W, H, bounces, spp, frame, rows):
    """WCPT_OPTION_WF_PIPES = K: K wavefront pipelines on K streams (tile t in pipeline t % K) render exactly the
    oracle's image and count exactly its work."""
    s = get_scene(name)
    init = np.random.default_rng(9).uniform(0, 1, (rows or H, W, 4)).astype(np.float32)
    y0 = (H - rows) // 2 if rows else 0
    gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, pipes)
    try:
        img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=frame, y0=y0, rows=rows, init=init,
                              kernel=wcpt.KERNEL_WAVEFRONT)
        img2, _ = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=frame, y0=y0, rows=rows, init=init,
                             kernel=wcpt.KERNEL_WAVEFRONT)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, wcpt._lib.DEFAULT_WF_PIPES)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=frame, y0=y0, rows=rows,
                                    image=init, threads=8)
    assert_close(img, ref)
    assert np.array_equal(img.view(np.uint32), img2.view(np.uint32))
    assert cnt == rcnt


def test_wavefront_pipelines_full_frame(gpu_ctx):
    """1080p atrium frame: 2 and 4 pipelines give the bit-identical frame of one pipeline, and the stream join
    orders a following readback after every pipeline."""
    s = get_scene("atrium")
    W, H = 1920, 1080
    init = np.zeros((H, W, 4), np.float32)
    gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, 1)
    try:
        one, c1 = gpu_render(gpu_ctx, s, W, H, bounces=4, frame=0, init=init, kernel=wcpt.KERNEL_WAVEFRONT)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, wcpt._lib.DEFAULT_WF_PIPES)
    for k in (2, 4):
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, k)
        try:
            img, ck = gpu_render(gpu_ctx, s, W, H, bounces=4, frame=0, init=init, kernel=wcpt.KERNEL_WAVEFRONT)
        finally:
            gpu_ctx.set_option(wcpt._lib.OPTION_WF_PIPES, wcpt._lib.DEFAULT_WF_PIPES)
        assert np.array_equal(img.view(np.uint32), one.view(np.uint32))
        assert ck == c1


@pytest.mark.parametrize("fetch", [0, 1])
@pytest.mark.parametrize("name,W,H,bounces,spp,frame,rows", [
    ("atrium", 96, 54, 4, 1, 2, None),
    ("cornell", 67, 45, 4, 3, 0, None),
    ("default_dielectric", 48, 40, 3, 2, 7, None),
    ("atrium", 200, 120, 4, 2, 1, 40),      # a row block, two samples
])
def test_wavefront_fetch_rounds_match_oracle(gpu_ctx, fetch, name, W, H, bounces, spp, frame, rows):
    """WCPT_OPTION_WF_FETCH = 0 / 1: the fast-layout trace with two fetch rounds per iteration (a leaf descent tested in
    the same iteration) and with one (interior and leaf fetches together, the descent tested next iteration) renders
    exactly the oracle's image; auto picks one of them by queue length (small frames: one round)."""
    s = get_scene(name)
    init = np.random.default_rng(11).uniform(0, 1, (rows or H, W, 4)).astype(np.float32)
    y0 = (H - rows) // 2 if rows else 0
    gpu_ctx.set_option(wcpt._lib.OPTION_WF_FETCH, fetch)
    try:
        img, _ = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=spp, frame=frame, y0=y0, rows=rows, init=init,
                            kernel=wcpt.KERNEL_WAVEFRONT)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_FETCH, -1)
    ref, _ = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=frame, y0=y0, rows=rows,
                                 image=init, threads=8)
    assert_close(img, ref)


@pytest.mark.parametrize("persist", [0, 1])
@pytest.mark.parametrize("name,W,H,bounces,frame,rows", [
    ("atrium", 96, 54, 4, 2, None),
    ("cornell", 67, 45, 4, 0, None),
    ("default_dielectric", 48, 40, 3, 7, None),
    ("atrium", 200, 120, 4, 1, 40),      # a row block
    ("reference_init", 64, 48, 3, 0, None),
])
def test_wavefront_persist_matches_oracle(gpu_ctx, persist, name, W, H, bounces, frame, rows):
    """WCPT_OPTION_WF_PERSIST = 0 / 1: the per-bounce trace + shade launches and the path-persistent trace (each lane
    runs its path's segments one after another and shades between them) render exactly the oracle's image."""
    s = get_scene(name)
    init = np.random.default_rng(13).uniform(0, 1, (rows or H, W, 4)).astype(np.float32)
    y0 = (H - rows) // 2 if rows else 0
    gpu_ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, persist)
    try:
        img, _ = gpu_render(gpu_ctx, s, W, H, bounces=bounces, spp=1, frame=frame, y0=y0, rows=rows, init=init,
                            kernel=wcpt.KERNEL_WAVEFRONT)
    finally:
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, -1)
    ref, _ = oracle.render_scene(s, W, H, max_bounce=bounces, samples=1, frame=frame, y0=y0, rows=rows,
                                 image=init, threads=8)
    assert_close(img, ref)


def test_wavefront_persist_full_frame_and_block(gpu_ctx):
    """1080p atrium: the path-persistent trace forced on gives the bit-identical frame of the per-bounce launches, and
    so does a 135-row block (where it is the automatic choice); a bad option value is refused."""
    s = get_scene("atrium")
    W, H = 1920, 1080
    for rows, y0 in ((None, 0), (135, 540)):
        init = np.zeros((rows or H, W, 4), np.float32)
        out = []
        for persist in (0, 1):
            gpu_ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, persist)
            try:
                out.append(gpu_render(gpu_ctx, s, W, H, bounces=4, spp=1, frame=3, y0=y0, rows=rows, init=init,
                                      kernel=wcpt.KERNEL_WAVEFRONT)[0])
            finally:
                gpu_ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, -1)
        assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    with pytest.raises(wcpt.WcptError):
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_PERSIST, 2)


def test_wavefront_fetch_rounds_full_frame(gpu_ctx):
    """1080p atrium frame, 2 samples: one and two fetch rounds per trace iteration give the bit-identical frame, and a
    bad option value is refused."""
    s = get_scene("atrium")
    W, H = 1920, 1080
    init = np.zeros((H, W, 4), np.float32)
    out = []
    for fetch in (0, 1):
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_FETCH, fetch)
        try:
            out.append(gpu_render(gpu_ctx, s, W, H, bounces=4, spp=2, frame=3, init=init,
                                  kernel=wcpt.KERNEL_WAVEFRONT)[0])
        finally:
            gpu_ctx.set_option(wcpt._lib.OPTION_WF_FETCH, -1)
    assert np.array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    with pytest.raises(wcpt.WcptError):
        gpu_ctx.set_option(wcpt._lib.OPTION_WF_FETCH, 2)


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("channels", [3, 4, 8])
def test_gather_output_equals_image(gpu_ctx, kernel, channels):
    """wcpt_set_gather_output: the render writes each pixel of its row block into the payload buffer too: RGB or
    RGBA bit-identical to the accumulation image, or (8 = WCPT_PAYLOAD_DISPLAY_RGBA8) composite.comp's display value
    as RGBA8, bit-identical to the oracle's composite of the accumulated frame -- progressive frames, a row block."""
    s = get_scene("cornell")
    W, H = 96, 80
    y0, rows = row_block(H, 3, 1)
    dev = wcpt.DeviceScene(gpu_ctx, s)
    gpu_ctx.set_kernel(kernel)
    nbytes = rows * W * wcpt._lib.PAYLOAD_PIXEL_BYTES[channels]
    buf = gpu_ctx.buffer_from(np.full(nbytes // 4, -7.0, np.float32))
    try:
        gpu_ctx.create_screen(W, H)
        gpu_ctx.set_row_range(y0, rows)
        init = np.random.default_rng(2).uniform(0, 1, (rows, W, 4)).astype(np.float32)
        gpu_ctx.image_upload(init)
        for frame in (0, 1, 2):
            gpu_ctx.set_gather_output(gpu_ctx.buffer_address(buf), nbytes, channels)
            gpu_ctx.render(s.scene_data(W, H, max_bounce=4, frame=frame), *dev.addresses())
            gpu_ctx.sync()
            img = gpu_ctx.readback(rows)
            if channels == wcpt._lib.PAYLOAD_DISPLAY_RGBA8:
                got8 = np.frombuffer(gpu_ctx.buffer_download(buf, nbytes), np.uint8).reshape(rows, W, 4)
                assert np.array_equal(got8, oracle.composite(img)[1])
                continue
            got = np.frombuffer(gpu_ctx.buffer_download(buf, nbytes), np.float32).reshape(rows, W, channels)
            assert np.array_equal(got.view(np.uint32), img[..., :channels].view(np.uint32))
        # too small for the row block -> error, no launch
        gpu_ctx.set_gather_output(gpu_ctx.buffer_address(buf), nbytes - 4, channels)
        with pytest.raises(wcpt.WcptError):
            gpu_ctx.render(s.scene_data(W, H, max_bounce=4, frame=3), *dev.addresses())
    finally:
        gpu_ctx.set_gather_output(0, 0)
        gpu_ctx.set_row_range(0, 0)
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        gpu_ctx.buffer_free(buf)
        dev.free()


def test_vector_scalar_division_within_1_5_ulp(gpu_ctx):
    """GLSL vector / scalar (normalize, the sphere normal :145, target.xyz / target.w :301, result / samples :312) is
    defined in both the kernel and the oracle as v * RN(1/s) (pt_device.h operator/, oracle/pt_oracle.c div3s), one
    correctly rounded reciprocal and a multiply. Vulkan allows 2.5 ULP for GLSL division; this bounds the kernel's
    form against the exact quotient at 1.5 ULP (and so within 2 ULP of the correctly rounded quotient), so a drift of
    the definition on either side shows up here. Parity for those expressions is defined by this form."""
    rng = np.random.default_rng(16)
    n = 200000
    a = (rng.standard_normal(n) * 10.0 ** rng.uniform(-20, 20, n)).astype(np.float32)
    b = (rng.standard_normal(n) * 10.0 ** rng.uniform(-20, 20, n)).astype(np.float32)
    a[:6] = [1.0, 3.0, 1e-3, 7.0, -2.5, 0.1]
    b[:6] = [3.0, 7.0, 3.0, 1e30, 1.0, 0.3]
    got = gpu_ctx.selftest(16, a.view(np.uint32), b.view(np.uint32)).view(np.float32)
    with np.errstate(all="ignore"):
        form = (a * (np.float32(1.0) / b)).astype(np.float32)     # the oracle's div3s in numpy binary32
        exact = a.astype(np.float64) / b.astype(np.float64)
    assert np.array_equal(got.view(np.uint32), form.view(np.uint32))
    ok = np.isfinite(exact) & (np.abs(exact) > 1e-36) & (np.abs(exact) < 1e36)
    ulp = np.spacing(np.abs(exact[ok]).astype(np.float32)).astype(np.float64)
    err = np.abs(got[ok].astype(np.float64) - exact[ok]) / ulp
    assert ok.sum() > n * 0.9
    assert err.max() <= 1.5, f"max error {err.max():.3f} ULP"
    rn = exact[ok].astype(np.float32)
    assert np.abs(got[ok].view(np.int32).astype(np.int64) - rn.view(np.int32).astype(np.int64)).max() <= 2



# ---- the headline configs at full size (BASELINE.json configs 3-4, and the reference's own scene) -----------------
def _oracle_bands(s, W, H, bounces, spp, frames, bands, rows):
    """Oracle renders of row bands [y0, y0 + rows) of the progressive frames `frames` (accumulated in order)."""
    out = {}
    for y0 in bands:
        acc = None
        cnt = None
        for f in frames:
            acc, cnt = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=f, y0=y0, rows=rows,
                                           image=acc, threads=16)
        out[y0] = (acc, cnt)
    return out


@pytest.mark.parametrize("kernel", KERNELS)
def test_c3_full_frame_vs_oracle(gpu_ctx, kernel):
    """BASELINE config 3 (the 262k-triangle atrium, 1920x1080, 1 spp, 4 bounces) on both kernels -- the wavefront one
    is the headline c3 kernel -- against the oracle over the WHOLE frame: image bit-exact and every work counter
    equal (the reference's stack stays within its 32 entries: ref_stack_max <= 32, no overflowing segment)."""
    s = get_scene("atrium")
    W, H = 1920, 1080
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=4, frame=0, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=4, frame=0, threads=16)
    assert_close(img, ref)
    assert cnt == rcnt
    assert rcnt["ref_stack_overflow_segments"] == 0 and rcnt["ref_stack_max"] <= 32


@pytest.mark.parametrize("kernel", KERNELS)
def test_c4_bands_vs_oracle(gpu_ctx, kernel):
    """BASELINE config 4 (atrium, 3840x2160, 16 spp in one dispatch, 4 bounces: samples * (maxBounceCount + 1) = 80
    trace/shade iterations per wavefront pipeline) rendered as the 270-row blocks of the 8-GPU split: the top block,
    the block starting at row 1080 (a block boundary) and the bottom block, progressive frames 0 and 1, against the
    oracle on 8-row bands at the top, the boundary and the bottom of those blocks, with exact counters per band."""
    s = get_scene("atrium")
    W, H, spp, bounces = 3840, 2160, 16, 4
    bands = {0: 0, 1080: 1080, 2160 - 270: 2160 - 8}      # block y0 -> band y0 inside it
    for by0, band in bands.items():
        dev = wcpt.DeviceScene(gpu_ctx, s)
        gpu_ctx.set_kernel(kernel)
        try:
            gpu_ctx.create_screen(W, H)
            gpu_ctx.set_row_range(by0, 270)
            for f in (0, 1):
                gpu_ctx.render(s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f), *dev.addresses())
            gpu_ctx.sync()
            blk = gpu_ctx.readback(270)
            gpu_ctx.set_row_range(band, 8)
            cnt = gpu_ctx.render_counters(s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=1),
                                          *dev.addresses())
        finally:
            gpu_ctx.set_row_range(0, 0)
            gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
            dev.free()
        ref, rcnt = _oracle_bands(s, W, H, bounces, spp, (0, 1), [band], 8)[band]
        assert_close(blk[band - by0:band - by0 + 8], ref)
        assert cnt == rcnt
        assert rcnt["ref_stack_overflow_segments"] == 0


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", ["reference_init", "reference_init_glass"])
def test_reference_init_full_size_rows(gpu_ctx, kernel, name):
    """The reference's own scene at the headline size (1920x1080, its default maxBounceCount 3 and 1 spp, the editor's
    still-camera frames 1 then 3): oracle row bands, bit-exact, counters exact."""
    s = get_scene(name)
    W, H = 1920, 1080
    dev = wcpt.DeviceScene(gpu_ctx, s)
    gpu_ctx.set_kernel(kernel)
    try:
        gpu_ctx.create_screen(W, H)
        for f in (1, 3):
            gpu_ctx.render(s.scene_data(W, H, max_bounce=3, frame=f), *dev.addresses())
        gpu_ctx.sync()
        img = gpu_ctx.readback(H)
        cnt = gpu_ctx.render_counters(s.scene_data(W, H, max_bounce=3, frame=3), *dev.addresses())
    finally:
        gpu_ctx.set_kernel(wcpt.KERNEL_MEGAKERNEL)
        dev.free()
    for y0, (ref, _) in _oracle_bands(s, W, H, 3, 1, (1, 3), (0, 270, 536, 1072), 8).items():
        assert_close(img[y0:y0 + 8], ref)
    _, rcnt = oracle.render_scene(s, W, H, max_bounce=3, frame=3, threads=16)
    assert cnt == rcnt


@pytest.mark.parametrize("kernel", KERNELS)
def test_deeper_than_reference_stack_counted(gpu_ctx, kernel):
    """A BVH chain 40 levels deep (tests/deep_tree.py) that drives the reference's stack past its 32 entries
    (pathTracer.comp:151, undefined behaviour there): this implementation renders it with its 48-entry stack,
    bit-exact against the oracle, and the counting kernel reports the same overflowing segments and deepest stack."""
    from deep_tree import deep_chain_scene
    s = deep_chain_scene(get_scene("default"), levels=40)
    W, H = 48, 32
    img, cnt = gpu_render(gpu_ctx, s, W, H, bounces=2, kernel=kernel)
    ref, rcnt = oracle.render_scene(s, W, H, max_bounce=2, threads=8)
    assert_close(img, ref)
    assert cnt == rcnt
    assert rcnt["ref_stack_max"] == 41 and rcnt["ref_stack_overflow_segments"] > 0


@pytest.mark.parametrize("name,W,H,bounces,spp", [("cornell", 67, 45, 4, 2), ("reference_init", 96, 64, 3, 1)])
def test_cost_ordered_tiles_match_oracle(name, W, H, bounces, spp):
    """The default tile order becomes longest-first after the first render of a geometry (the renders record each
    tile's time; pt_kernels.hip cost_order_sort). Progressive frames through that order, then a row range and a resize
    (new geometries: back to the built-in order, then sorted again), all bit-exact against the oracle."""
    s = get_scene(name)
    with wcpt.Context(0) as ctx:
        dev = wcpt.DeviceScene(ctx, s)
        try:
            ctx.create_screen(W, H)
            acc = None
            for f in range(5):
                sd = s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f)
                ctx.render(sd, *dev.addresses())
                acc, _ = oracle.render_scene(s, W, H, sd=sd, image=acc, threads=8)
            ctx.sync()
            assert_close(ctx.readback(H), acc)
            ctx.set_row_range(8, 24)                  # a row block: another geometry
            blk = None
            for f in range(3):
                sd = s.scene_data(W, H, max_bounce=bounces, samples=spp, frame=f)
                ctx.render(sd, *dev.addresses())
                blk, _ = oracle.render_scene(s, W, H, sd=sd, y0=8, rows=24, image=blk, threads=8)
            ctx.sync()
            assert_close(ctx.readback(24), blk)
            ctx.set_row_range(0, 0)
            W2, H2 = W + 16, H - 9
            ctx.resize(W2, H2)
            acc = None
            for f in range(3):
                sd = s.scene_data(W2, H2, max_bounce=bounces, samples=spp, frame=f)
                ctx.render(sd, *dev.addresses())
                acc, _ = oracle.render_scene(s, W2, H2, sd=sd, image=acc, threads=8)
            ctx.sync()
            assert_close(ctx.readback(H2), acc)
        finally:
            dev.free()
