"""ORACLE (test infrastructure only) — an independent float64 restatement of the reference path tracer in numpy.

Only tests/ import this module, as a second checker of oracle/pt_oracle.c. It restates, from the GLSL alone:
  /root/reference/src/shaders/pathTracer.comp:97-133   rayBoxIntersect, raySphereIntersect, rayTriangleIntersect
  /root/reference/src/shaders/pathTracer.comp:135-211  Intersect (sphere loop, per-draw BVH walk with nodeStack)
  /root/reference/src/shaders/pathTracer.comp:213-284  CalculateReflectance, ray_color, TraceRay
  /root/reference/src/shaders/pathTracer.comp:289-324  main (NDC -> primary ray, seed, samples, progressive mix)
  /root/reference/src/shaders/include/Random.glsl:10-56 pcg_hash, rand_pcg, rand, RandomValueNormalDistribution,
                                                         RandomDirection
and shares NO code or convention with pt_oracle.c / wcpt_libm.h / the HIP kernels: every real-valued expression is
evaluated in binary64 with numpy's libm log/cos/exp/sqrt and true division (GLSL `v / s` is a per-component divide
here, not v * (1/s)); min/max are IEEE minNum/maxNum (np.fmin/np.fmax). The only binary32 step kept is GLSL's
`float(x)` of the uint in rand (Random.glsl:31), which is a type conversion that defines the value, not arithmetic.

Purpose: the C oracle and the kernels are bit-exact with each other but share conventions (the libm,
v*RN(1/s)); a semantic slip common to both would pass every bit-exact test. This restatement catches such a slip:
tests/test_oracle_f64.py requires nearly all pixels to agree within 1e-4 and the work counters of every row
without a diverged pixel to be equal. Rays whose binary32 and binary64 decisions differ (a triangle edge, the
Fresnel draw, a tangent sphere) diverge chaotically; they are few and are counted, not hidden.

Vectorised over pixels: each segment traces all live paths together, each path walking its own stack in the
reference's order. Sizes are kept small (the tests use <= 64x48 frames).
"""
from __future__ import annotations

import numpy as np

K_INFINITY = float(np.float32(3.402823466e38))   # constants.glsl:6 (a float literal: FLT_MAX)
BIAS = 1e-5                                      # constants.glsl:5
PI = 3.14159265358979323846264338327950288       # constants.glsl:9
M_A, M_C, M_P = np.uint32(747796405), np.uint32(2891336453), np.uint32(277803737)
METAL = 0
STACK = 128                                      # the reference has 32 (:151); deeper use is counted, not clipped
_FT = np.float64    # the evaluation type; render(dtype=np.float32) re-evaluates the same statements in binary32


# ---- Random.glsl ------------------------------------------------------------------------------------------------
def _perm(state: np.ndarray) -> np.ndarray:
    """The PCG output permutation shared by pcg_hash and rand_pcg (Random.glsl:14-15, 23-24)."""
    with np.errstate(over="ignore"):
        word = ((state >> ((state >> np.uint32(28)) + np.uint32(4))) ^ state) * M_P
    return (word >> np.uint32(22)) ^ word


def pcg_hash(seed: np.ndarray) -> np.ndarray:
    """Random.glsl:10-16: one LCG step, then the permutation."""
    with np.errstate(over="ignore"):
        return _perm(np.asarray(seed, np.uint32) * M_A + M_C)


def rand(state: np.ndarray, mask: np.ndarray | None = None) -> np.ndarray:
    """Random.glsl:19-33: x = permutation of the OLD state (rand_pcg's LCG update is overwritten by `state = x`);
    returns float(x) * 2^-32 with float() the binary32 conversion. Updates `state` in place where mask is set."""
    x = _perm(state)
    if mask is None:
        state[:] = x
    else:
        state[mask] = x[mask]
    return x.astype(np.float32).astype(_FT) * 2.0 ** -32


def random_value_normal(state, mask):
    """Random.glsl:44-49: theta's rand is drawn before rho's."""
    theta = 2.0 * PI * rand(state, mask)
    with np.errstate(divide="ignore", invalid="ignore"):
        rho = np.sqrt(-2.0 * np.log(rand(state, mask)))
    return rho * np.cos(theta)


def random_direction(state, mask):
    """Random.glsl:51-57: normalize(vec3(x, y, z)), drawn x, y, z in order."""
    x = random_value_normal(state, mask)
    y = random_value_normal(state, mask)
    z = random_value_normal(state, mask)
    return _normalize(np.stack([x, y, z], axis=-1))


# ---- GLSL built-ins in binary64 ------------------------------------------------------------------------------------
def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - b[..., 1] * a[..., 2],
                     a[..., 2] * b[..., 0] - b[..., 2] * a[..., 0],
                     a[..., 0] * b[..., 1] - b[..., 0] * a[..., 1]], axis=-1)


def _normalize(v):
    with np.errstate(divide="ignore", invalid="ignore"):
        return v / np.sqrt(_dot(v, v))[..., None]


def _reflect(i, n):
    return i - 2.0 * _dot(n, i)[..., None] * n


def _refract(i, n, eta):
    """GLSL refract: k = 1 - eta^2 (1 - dot(N,I)^2); 0 when k < 0, else eta I - (eta dot(N,I) + sqrt(k)) N."""
    d = _dot(n, i)
    k = 1.0 - eta * eta * (1.0 - d * d)
    with np.errstate(invalid="ignore"):
        t = eta[..., None] * i - (eta * d + np.sqrt(np.maximum(k, 0.0)))[..., None] * n
    return np.where((k < 0.0)[..., None], 0.0, t)


def _sign(x):
    return np.sign(x)                       # GLSL sign(0) = 0


# ---- pathTracer.comp:97-133 -------------------------------------------------------------------------------------
def ray_box(o, inv, bmin, bmax):
    """rayBoxIntersect: slab distances, t0 = max of the three tmin, t1 = min of the three tmax (minNum/maxNum)."""
    with np.errstate(invalid="ignore"):
        tbot = (bmin - o) * inv
        ttop = (bmax - o) * inv
    tmin = np.fmin(ttop, tbot)
    tmax = np.fmax(ttop, tbot)
    t0 = np.fmax(np.fmax(tmin[..., 0], tmin[..., 1]), np.fmax(tmin[..., 0], tmin[..., 2]))
    t1 = np.fmin(np.fmin(tmax[..., 0], tmax[..., 1]), np.fmin(tmax[..., 0], tmax[..., 2]))
    return t0, t1


def ray_sphere_near(o, d, pos, radius):
    """raySphereIntersect(...).x: -b - sqrt(b^2 - c), or -1 when the discriminant is negative."""
    oc = o - pos
    b = _dot(oc, d)
    c = _dot(oc, oc) - radius * radius
    t = b * b - c
    with np.errstate(invalid="ignore"):
        return np.where(t < 0.0, -1.0, -b - np.sqrt(np.maximum(t, 0.0)))


def ray_triangle(o, d, a, b, c):
    """rayTriangleIntersect (Moller-Trumbore, :121-133): t when t > 0, u in [0,1], v >= 0, u + v <= 1, else -1."""
    e1 = b - a
    e2 = c - a
    oa = o - a
    p = _cross(d, e2)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / _dot(e1, p)
        q = _cross(oa, e1)
        u = _dot(oa, p) * inv
        v = _dot(d, q * inv[..., None])
        t = _dot(e2, q) * inv
    ok = (t > 0.0) & (u >= 0.0) & (u <= 1.0) & (v >= 0.0) & (u + v <= 1.0)
    return np.where(ok, t, -1.0)


# ---- pathTracer.comp:135-211 ------------------------------------------------------------------------------------
class _Draw:
    def __init__(self, positions, indices, nodes):
        self.v = np.asarray(positions, _FT).reshape(-1, 3)
        self.ix = np.asarray(indices, np.int64)
        n = np.asarray(nodes)
        self.bmin = np.asarray(n["min"], _FT)
        self.bmax = np.asarray(n["max"], _FT)
        self.left = np.asarray(n["leftNodeOrTriangleIndex"], np.int64)
        self.count = np.asarray(n["triangleCount"], np.int64)


def intersect(o, d, inv, spheres, draws, cnt):
    """Intersect for every ray of the batch. Returns (hit, t, p, normal, front, material); adds to the per-ray
    counters cnt[name] (the oracle's definitions: one segment per call, a sphere test per sphere, a node pop per
    popped stack entry, an interior visit per child-pair expansion, a triangle test per triangle, a draw fetch per
    draw command, a hit per segment that hits) and tracks the deepest stack (ref_stack_max, counted after pushes)."""
    n = o.shape[0]
    t = np.full(n, K_INFINITY, _FT)
    hit = np.zeros(n, bool)
    normal = np.zeros((n, 3), _FT)
    material = np.zeros(n, np.int64)
    cnt["segments"] += 1
    for s in spheres:
        pos = np.asarray(s["position"], _FT)
        r = _FT(s["radius"])
        ts = ray_sphere_near(o, d, pos, r)
        cnt["sphere_tests"] += 1
        upd = (ts > 0.0) & (ts < t)
        t = np.where(upd, ts, t)
        with np.errstate(over="ignore", invalid="ignore"):
            p = o + t[:, None] * d
            normal = np.where(upd[:, None], (p - pos) / r, normal)
        hit |= upd
        material = np.where(upd, int(s["material"]), material)
    over = np.zeros(n, bool)
    for dr in draws:
        cnt["draw_fetches"] += 1
        stack = np.zeros((n, STACK), np.int64)
        sp = np.ones(n, np.int64)                          # nodeStack[stackIndex++] = 0
        cnt["ref_stack_max"] = np.maximum(cnt["ref_stack_max"], 1)
        rows = np.arange(n)
        while True:
            act = np.nonzero(sp > 0)[0]
            if act.size == 0:
                break
            sp[act] -= 1
            node = stack[act, sp[act]]
            cnt["node_pops"][act] += 1
            t0, t1 = ray_box(o[act], inv[act], dr.bmin[node], dr.bmax[node])
            live = ~((t0 > t1) | (t1 < 0.0) | (t0 > t[act]))
            act, node = act[live], node[live]
            leaf = dr.count[node] > 0
            # leaves: triangles first + i, i += 3 while i < count, in order, strict < against the running rec.t
            la, ln = act[leaf], node[leaf]
            if la.size:
                first, count = dr.left[ln], dr.count[ln]
                i = 0
                while True:
                    m = i < count
                    if not m.any():
                        break
                    ra, f = la[m], first[m] + i
                    a = dr.v[dr.ix[f]]
                    b = dr.v[dr.ix[f + 1]]
                    c = dr.v[dr.ix[f + 2]]
                    tt = ray_triangle(o[ra], d[ra], a, b, c)
                    cnt["triangle_tests"][ra] += 1
                    upd = (tt != -1.0) & (tt < t[ra])
                    ru = ra[upd]
                    t[ru] = tt[upd]
                    normal[ru] = _normalize(_cross(b[upd] - a[upd], c[upd] - a[upd]))
                    hit[ru] = True
                    material[ru] = 0
                    i += 3
            # interior nodes: both children's boxes, the nearer (entry distance, or exit when behind) popped first
            ia, inode = act[~leaf], node[~leaf]
            if ia.size:
                cnt["interior_visits"][ia] += 1
                lc = dr.left[inode]
                rc = lc + 1
                l0, l1 = ray_box(o[ia], inv[ia], dr.bmin[lc], dr.bmax[lc])
                r0, r1 = ray_box(o[ia], inv[ia], dr.bmin[rc], dr.bmax[rc])
                ldist = np.where(l0 > 0.0, l0, l1)
                rdist = np.where(r0 > 0.0, r0, r1)
                near_left = ldist < rdist
                first_push = np.where(near_left, rc, lc)
                second_push = np.where(near_left, lc, rc)
                if (sp[ia] + 2 > STACK).any():
                    raise RuntimeError("pt_f64: traversal stack exceeded its 128 entries")
                stack[ia, sp[ia]] = first_push
                stack[ia, sp[ia] + 1] = second_push
                sp[ia] += 2
                over[ia] |= sp[ia] > 32                  # wrote nodeStack[32] or beyond
                cnt["ref_stack_max"][ia] = np.maximum(cnt["ref_stack_max"][ia], sp[ia])
        del rows
    cnt["ref_stack_overflow_segments"] += over
    cnt["hits"] += hit
    p = o + t[:, None] * d
    front = _dot(d, normal) < 0.0
    normal = np.where((hit & ~front)[:, None], -normal, normal)
    return hit, t, p, normal, front, material


# ---- pathTracer.comp:213-284 ------------------------------------------------------------------------------------
def reflectance(in_dir, normal, ior_a, ior_b):
    """CalculateReflectance (:213-234)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        ratio = ior_a / ior_b
        cos_in = -_dot(in_dir, normal)
        sin2 = ratio * ratio * (1.0 - cos_in * cos_in)
        cos_out = np.sqrt(np.maximum(1.0 - sin2, 0.0))
        den_perp = ior_a * cos_in + ior_b * cos_out
        den_par = ior_b * cos_in + ior_a * cos_out
        r_perp = ((ior_a * cos_in - ior_b * cos_out) / den_perp) ** 2
        r_par = ((ior_b * cos_in - ior_a * cos_out) / den_par) ** 2
        r = (r_perp + r_par) / 2.0
    r = np.where(np.fmin(den_perp, den_par) < 1e-8, 1.0, r)
    return np.where(sin2 >= 1.0, 1.0, r)


def ray_color(d):
    """Sky (:236-239): mix(vec3(0.5, 0.7, 1.0), vec3(1.0), 0.5 * (d.y + 1))."""
    a = 0.5 * (d[:, 1] + 1.0)
    base = np.array([0.5, 0.7, 1.0], _FT)
    return base * (1.0 - a)[:, None] + a[:, None]


def trace_ray(o, d, state, max_bounce, materials, spheres, draws, cnt):
    """TraceRay (:241-284) for a batch of rays: returns the radiance; updates the RNG states in place."""
    n = o.shape[0]
    o = o.copy()
    d = d.copy()
    with np.errstate(divide="ignore"):
        inv = 1.0 / d
    light = np.zeros((n, 3), _FT)
    trans = np.ones((n, 3), _FT)
    out = np.zeros((n, 3), _FT)
    alive = np.ones(n, bool)
    mat_type = np.asarray(materials["type"], np.int64)
    albedo = np.asarray(materials["albedo"], _FT)
    emission = np.asarray(materials["emission"], _FT)
    e_strength = np.asarray(materials["emissionStrength"], _FT)
    rough = np.asarray(materials["roughness"], _FT)
    absorption = np.asarray(materials["absorption"], _FT)
    a_strength = np.asarray(materials["absorptionStrength"], _FT)
    ior = np.asarray(materials["ior"], _FT)
    for _ in range(max_bounce + 1):
        idx = np.nonzero(alive)[0]
        if idx.size == 0:
            break
        sub = {k: np.zeros(idx.size, np.int64) for k in cnt}
        hit, t, p, nrm, front, mat = intersect(o[idx], d[idx], inv[idx], spheres, draws, sub)
        for k in cnt:
            cnt[k][idx] = np.maximum(cnt[k][idx], sub[k]) if k == "ref_stack_max" else cnt[k][idx] + sub[k]
        miss = idx[~hit]
        out[miss] = light[miss] + ray_color(d[miss]) * trans[miss]
        alive[miss] = False
        h = idx[hit]
        t, p, nrm, front, mat = t[hit], p[hit], nrm[hit], front[hit], mat[hit]
        light[h] += (emission[mat] * e_strength[mat][:, None]) * trans[h]
        metal = mat_type[mat] == METAL
        # metal (:256-262)
        hm = h[metal]
        if hm.size:
            mm = mat[metal]
            o[hm] = p[metal] + nrm[metal] * BIAS
            sel = np.zeros(n, bool)
            sel[hm] = True
            rd = random_direction(state, sel)[hm]
            d[hm] = _normalize(_reflect(d[hm], nrm[metal]) + rough[mm][:, None] * rd)
            with np.errstate(divide="ignore"):
                inv[hm] = 1.0 / d[hm]
            trans[hm] *= albedo[mm]
        # dielectric (:263-280)
        hd = h[~metal]
        if hd.size:
            md, nd, fd, td, pd = mat[~metal], nrm[~metal], front[~metal], t[~metal], p[~metal]
            eta_i = np.where(fd, 1.0, ior[md])
            eta_t = np.where(fd, ior[md], 1.0)
            prob = reflectance(d[hd], nd, eta_i, eta_t)
            R = _reflect(d[hd], nd)
            T = _refract(d[hd], nd, eta_i / eta_t)
            t_zero = (T[:, 0] == 0.0) & (T[:, 1] == 0.0) & (T[:, 2] == 0.0)
            sel = np.zeros(n, bool)
            sel[hd[~t_zero]] = True                      # `||` short-circuit: rand only when T != 0 (:273)
            r = rand(state, sel)[hd]
            follow = t_zero | (r <= prob)
            sel = np.zeros(n, bool)
            sel[hd] = True
            rd = random_direction(state, sel)[hd]
            nd_dir = _normalize(np.where(follow[:, None], R, T) + rough[md][:, None] * rd)
            d[hd] = nd_dir
            with np.errstate(divide="ignore"):
                inv[hd] = 1.0 / nd_dir
            absorb = ~follow & ~fd
            ha = hd[absorb]
            trans[ha] *= np.exp(-absorption[md[absorb]] * a_strength[md[absorb]][:, None] * td[absorb][:, None])
            o[hd] = pd + BIAS * nd * _sign(_dot(nd_dir, nd))[:, None]
    out[alive] = light[alive]                            # return totalLight after the last bounce (:283)
    return out


# ---- pathTracer.comp:289-324 ------------------------------------------------------------------------------------
def _mat4_mul(cols16, v):
    """GLSL mat4 * vec4 with the 16 floats of the scalar layout (column-major: column j = elements 4j..4j+3):
    ((c0 v.x + c1 v.y) + c2 v.z) + c3 v.w."""
    c = np.asarray(cols16, _FT).reshape(4, 4)
    return ((c[0] * v[:, 0:1] + c[1] * v[:, 1:2]) + c[2] * v[:, 2:3]) + c[3] * v[:, 3:4]


def render(sd, materials, spheres, meshes, width, height, y0=0, rows=None, image=None, dtype=np.float64):
    """Rows [y0, y0 + rows) of a width x height frame. Returns (rgba image, per-row counters dict of int64 arrays
    [rows]). `image` (float [rows, width, 4]) is the previous accumulation (imageLoad, :314). dtype np.float32
    evaluates the same statements in binary32 (numpy's per-operation rounding and its float32 libm): a control that
    separates precision effects from semantic ones (tests/test_oracle_f64.py)."""
    global _FT
    _FT = dtype
    rows = height - y0 if rows is None else rows
    sd = np.asarray(sd).reshape(())
    ys, xs = np.meshgrid(np.arange(y0, y0 + rows), np.arange(width), indexing="ij")
    xs, ys = xs.ravel(), ys.ravel()
    n = xs.size
    size = np.array([width, height], _FT)
    coord = np.stack([xs.astype(_FT) / size[0], ys.astype(_FT) / size[1]], axis=-1)
    coord = coord + (_FT(1.0) / size) * _FT(0.5)
    coord[:, 1] = 1.0 - coord[:, 1]
    coord = coord * 2.0 - 1.0
    one = np.ones(n, _FT)
    target = _mat4_mul(sd["inverseProjection"], np.stack([coord[:, 0], coord[:, 1], one, one], axis=-1))
    dcam = _normalize(target[:, :3] / target[:, 3:4])
    w4 = np.concatenate([dcam, np.zeros((n, 1), _FT)], axis=-1)
    direction = _normalize(_mat4_mul(sd["inverseView"], w4)[:, :3])
    origin = np.broadcast_to(np.asarray(sd["position"], _FT), (n, 3))
    frame = int(sd["renderedFramesCount"])
    with np.errstate(over="ignore"):
        pix = (xs.astype(np.uint32) + ys.astype(np.uint32) * np.uint32(width) + np.uint32(frame) * np.uint32(719393))
    state = pcg_hash(pix)
    mats = np.asarray(materials)
    sph = list(np.asarray(spheres)[: int(sd["sphereCount"])])
    draws = [_Draw(*m) for m in meshes[: int(sd["drawCommandCount"])]]
    names = ("pixels", "segments", "sphere_tests", "node_pops", "interior_visits", "triangle_tests", "hits",
             "draw_fetches", "ref_stack_overflow_segments", "ref_stack_max")
    cnt = {k: np.zeros(n, np.int64) for k in names}
    cnt["pixels"][:] = 1
    result = np.zeros((n, 3), _FT)
    samples = int(sd["samples"])
    for _ in range(samples):
        result += trace_ray(origin, direction, state, int(sd["maxBounceCount"]), mats, sph, draws, cnt)
    with np.errstate(divide="ignore", invalid="ignore"):
        result = result / _FT(samples)                   # samples == 0: 0/0 (:312)
    old = np.zeros((n, 3), _FT) if image is None else np.asarray(image, _FT).reshape(n, 4)[:, :3]
    weight = _FT(1.0) / _FT(frame + 1)
    acc = result if frame == 0 else old * (1.0 - weight) + result * weight
    out = np.concatenate([acc, np.ones((n, 1), _FT)], axis=-1).reshape(rows, width, 4)
    per_row = {k: (v.reshape(rows, width).max(axis=1) if k == "ref_stack_max" else v.reshape(rows, width).sum(axis=1))
               for k, v in cnt.items()}
    return out, per_row


def render_scene(scene, width, height, max_bounce=3, samples=1, frame=0, y0=0, rows=None, image=None,
                 dtype=np.float64):
    sd = scene.scene_data(width, height, max_bounce=max_bounce, samples=samples, frame=frame)
    meshes = [(m.positions, m.indices, m.nodes) for m in scene.meshes]
    return render(sd, scene.materials, scene.spheres, meshes, width, height, y0=y0, rows=rows, image=image,
                  dtype=dtype)
