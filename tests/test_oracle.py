"""The CPU oracle pinned before it is trusted: known answers, hand-derived intersection cases,
libm accuracy against float64, and the committed golden images."""
import json
import math
import os

import numpy as np
import pytest

import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def test_pcg_hash_kat():
    kat = json.load(open(os.path.join(HERE, "golden", "kat.json")))
    for x, v in kat["pcg_hash"].items():
        assert oracle.pcg_hash(int(x)) == v
    # SURVEY.md §4 table
    assert oracle.pcg_hash(0) == 129708002 == 0x07BB2FE2
    assert oracle.pcg_hash(1) == 2831084092
    assert oracle.pcg_hash(2) == 2055130248
    assert oracle.pcg_hash(719393) == 1815429807
    assert oracle.pcg_hash(2073599) == 2921424543


def test_rand_stream_kat():
    """rand() overwrites the state with its output (Random.glsl:29-30): SURVEY.md §4 states and floats."""
    vals, states = oracle.rand_stream(oracle.pcg_hash(0), 4)
    assert states == [2354161293, 632039529, 839422272, 2779870596]
    assert np.allclose(vals, [0.54812092, 0.14715818, 0.19544323, 0.64723909], rtol=0, atol=5e-8)
    kat = json.load(open(os.path.join(HERE, "golden", "kat.json")))
    assert [e["state"] for e in kat["rand_from_pcg_hash_0"]] == states
    assert np.array_equal(vals, np.array([e["float"] for e in kat["rand_from_pcg_hash_0"]], np.float32))


def test_rand_can_return_one():
    """float(x)*2^-32 rounds to exactly 1.0 for x >= 2^32-128."""
    # find a state whose permutation output is >= 2^32 - 128 is expensive; check the arithmetic instead
    assert np.float32(np.float32(4294967295) * np.float32(2.0 ** -32)) == np.float32(1.0)


def _ulp_err(got, exact):
    got = np.float32(got)
    e32 = np.float32(exact)
    if e32 == 0:
        return 0.0 if got == 0 else float("inf")
    ulp = np.spacing(np.abs(e32))
    return abs(float(got) - exact) / float(ulp)


@pytest.mark.parametrize("name,fn,ref,lo,hi", [
    ("log", oracle.logf, math.log, 1e-38, 1.0),
    ("cos", oracle.cosf, math.cos, 0.0, 2 * math.pi),
    ("exp", oracle.expf, math.exp, -87.0, 0.0),
])
def test_libm_accuracy(name, fn, ref, lo, hi):
    rng = np.random.default_rng(11)
    if name == "log":
        xs = np.exp(rng.uniform(math.log(lo), 0.0, 4000)).astype(np.float32)
        xs = np.concatenate([xs, rng.uniform(0.0, 1.0, 4000).astype(np.float32)])
        xs = xs[xs > 0]
    else:
        xs = rng.uniform(lo, hi, 8000).astype(np.float32)
    worst = 0.0
    for x in xs:
        worst = max(worst, _ulp_err(fn(float(x)), ref(float(x))))
    assert worst <= 2.0, f"{name}: worst error {worst:.2f} ulp"


def test_libm_kernel_domains_equal_general():
    """The kernel's wcpt_logf_rand / wcpt_cosf_2pi return the general functions' bits on every rand() output they
    are called with (n * 2^-32, and 2*PI times it): checked on 2^32 / 251 values spread over the whole domain plus
    its ends."""
    assert oracle.lib.oracle_libm_domain_mismatches(0, 251) == 0
    assert oracle.lib.oracle_libm_domain_mismatches(0xFFFFFF00, 1) == 0
    assert oracle.lib.oracle_libm_domain_mismatches(0, 1 << 24) == 0


def test_libm_special_values():
    assert oracle.logf(0.0) == -np.inf
    assert oracle.logf(1.0) == 0.0
    assert np.isnan(oracle.logf(-1.0)) and np.isnan(oracle.logf(float("nan")))
    assert oracle.logf(float("inf")) == np.inf
    tiny = float(np.float32(1e-45))                                    # 2^-149, the smallest subnormal
    assert _ulp_err(oracle.logf(tiny), math.log(tiny)) <= 1.0
    assert oracle.cosf(0.0) == 1.0
    assert np.isnan(oracle.cosf(float("inf")))
    assert oracle.expf(0.0) == 1.0
    assert oracle.expf(-200.0) == 0.0 and oracle.expf(100.0) == np.inf
    assert 0.0 < oracle.expf(-100.0) < 1e-43                            # subnormal result


def test_ray_box_kat():
    """pathTracer.comp:97-108 with invDirection = 1/d (+-inf on zero components)."""
    t = oracle.ray_box([0, 0, -5], [0, 0, 1], [-1, -1, -1], [1, 1, 1])
    assert t.tolist() == [4.0, 6.0]
    # origin on the x = +1 slab plane: (1-1)*inf = NaN, minNum/maxNum drop it -> t1 = -inf, a miss
    t = oracle.ray_box([1, 0, -5], [0, 0, 1], [-1, -1, -1], [1, 1, 1])
    assert t[0] == 4.0 and t[1] == -np.inf
    # diagonal ray from inside: t0 < 0 < t1
    t = oracle.ray_box([0, 0, 0], np.array([1, 1, 1]) / np.sqrt(3), [-1, -1, -1], [1, 1, 1])
    assert t[0] < 0 < t[1]


def test_ray_sphere_kat():
    """Near root only (pathTracer.comp:141): rays starting inside a sphere miss it."""
    assert oracle.ray_sphere([0, 0, 0], [0, 0, -1], [0, 0, -3], 1.0) == 2.0
    assert oracle.ray_sphere([0, 0, -3], [0, 0, -1], [0, 0, -3], 1.0) == -1.0
    assert oracle.ray_sphere([0, 5, 0], [0, 0, -1], [0, 0, -3], 1.0) == -1.0   # disc < 0


def test_ray_triangle_kat():
    """Moller-Trumbore as written at pathTracer.comp:121-133 (no epsilon)."""
    a, b, c = [0, 0, 0], [1, 0, 0], [0, 1, 0]
    assert oracle.ray_triangle([0.25, 0.25, 1], [0, 0, -1], a, b, c) == 1.0
    assert oracle.ray_triangle([0.8, 0.8, 1], [0, 0, -1], a, b, c) == -1.0    # u + v > 1
    assert oracle.ray_triangle([0.25, 0.25, 1], [1, 0, 0], a, b, c) == -1.0   # parallel: inv = inf
    assert oracle.ray_triangle([0.25, 0.25, -1], [0, 0, -1], a, b, c) == -1.0  # behind the origin
    assert oracle.ray_triangle([0.0, 0.0, 1], [0, 0, -1], a, b, c) == 1.0     # on a vertex: u = v = 0 counts


def test_golden_images_reproduce():
    """The oracle, rebuilt here, reproduces the committed golden images bit for bit."""
    from golden_cases import CASES
    from wcpt import scene as wscene
    gold = np.load(os.path.join(HERE, "golden", "images.npz"))
    scenes = {}
    for key, (name, W, H, bounces, spp, frames) in CASES.items():
        s = scenes.setdefault(name, wscene.generate(name))
        acc = None
        for f in frames:
            acc, _ = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=f, image=acc, threads=8)
        assert np.array_equal(acc[..., :3], gold[key]), key


def test_render_counters_consistent():
    """Counter identities of the reference algorithm: pops = draws + 2*interior, segments bounded."""
    from wcpt import scene as wscene
    s = wscene.generate("cornell")
    img, c = oracle.render_scene(s, 64, 64, max_bounce=4, threads=4)
    assert c["pixels"] == 64 * 64
    assert c["pixels"] <= c["segments"] <= 5 * c["pixels"]
    assert c["node_pops"] == c["draw_fetches"] + 2 * c["interior_visits"]
    assert c["sphere_tests"] == len(s.spheres) * c["segments"]
    assert c["draw_fetches"] == c["segments"]
    assert np.all(img[..., 3] == 1.0)


def test_row_blocks_compose():
    """Oracle row blocks (global pixel indices) compose to the full frame exactly."""
    from wcpt import scene as wscene
    s = wscene.generate("default_dielectric")
    full, _ = oracle.render_scene(s, 40, 30, max_bounce=3)
    top, _ = oracle.render_scene(s, 40, 30, max_bounce=3, y0=0, rows=13)
    bot, _ = oracle.render_scene(s, 40, 30, max_bounce=3, y0=13, rows=17)
    assert np.array_equal(np.concatenate([top, bot]), full)


# ---- composite.comp (display step) ----------------------------------------------------------------------
def _composite_f64(img):
    """float64 restatement of composite.comp:3-54 (gamma 1/2.2 + PBR Neutral) for tolerance checks."""
    with np.errstate(divide="ignore", invalid="ignore"):
        return _composite_f64_body(img)


def _composite_f64_body(img):
    c = np.power(np.maximum(img[..., :3].astype(np.float64), 0.0), 1.0 / 2.2)
    x = c.min(axis=-1, keepdims=True)
    off = np.where(x < 0.08, x - 6.25 * x * x, 0.04)
    c = c - off
    peak = c.max(axis=-1, keepdims=True)
    sc = 0.8 - 0.04
    d = 1.0 - sc
    new_peak = 1.0 - d * d / (peak + d - sc)
    g = 1.0 - 1.0 / (0.15 * (peak - new_peak) + 1.0)
    comp = c * (new_peak / peak)
    comp = comp * (1.0 - g) + new_peak * g
    return np.where(peak < sc, c, comp)


def test_composite_oracle_vs_float64():
    rng = np.random.default_rng(3)
    img = np.ones((64, 48, 4), np.float32)
    img[..., :3] = (rng.random((64, 48, 3)) ** 3 * 8.0).astype(np.float32)
    img[0, 0, :3] = [0.0, 0.0, 0.0]
    img[0, 1, :3] = [1.0, 1.0, 1.0]
    img[0, 2, :3] = [100.0, 0.5, 0.0]
    out32, out8 = oracle.composite(img)
    ref = _composite_f64(img)
    assert np.all(out32[..., 3] == 1.0) and np.all(out8[..., 3] == 255)
    np.testing.assert_allclose(out32[..., :3], ref, rtol=2e-6, atol=2e-7)
    expect8 = np.where(out32[..., :3] > 0, np.floor(np.clip(out32[..., :3], 0, 1) * np.float32(255) + np.float32(0.5)), 0)
    assert np.array_equal(out8[..., :3], expect8.astype(np.uint8))


def test_composite_special_values():
    img = np.array([[np.nan, 0.5, 0.5, 1], [-1.0, 0.2, 0.2, 1], [np.inf, 0.0, 0.0, 1]], np.float32)
    out32, out8 = oracle.composite(img)
    assert out8.dtype == np.uint8 and out8.shape == (3, 4)
    assert np.all(out8[:, 3] == 255)
