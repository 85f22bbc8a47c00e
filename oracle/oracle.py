"""ORACLE (test infrastructure only) — ctypes wrapper of oracle/liboracle.so (oracle/pt_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and only as the
checker or the reported CPU baseline; the product (wc-path-tracer_amd/) never imports it.
Parity pinning status: see the header of pt_oracle.c and DESIGN.md §Parity.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# bench.py's cpu_baseline points this at its -O3 -march=native build of the same source (WCPT_ORACLE_LIB)
LIB_PATH = os.environ.get("WCPT_ORACLE_LIB", os.path.join(HERE, "liboracle.so"))

SCENE_DATA_ITEMSIZE = 164
WORK_FIELDS = ("pixels", "segments", "sphere_tests", "node_pops", "interior_visits", "triangle_tests",
               "hits", "draw_fetches")
REF_STACK_FIELDS = ("ref_stack_overflow_segments", "ref_stack_max")
COUNTER_FIELDS = WORK_FIELDS + REF_STACK_FIELDS


class _Counters(C.Structure):
    # wcpt_counters of include/wcpt.h: the 8 reference counters + 6 implementation diagnostics (left 0 here) + the
    # reference-stack fields (segments writing past uint nodeStack[32], deepest stack)
    _fields_ = ([(n, C.c_uint64) for n in WORK_FIELDS] + [(f"_diag{i}", C.c_uint64) for i in range(6)]
                + [(n, C.c_uint64) for n in REF_STACK_FIELDS])


class _Draw(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("indices", C.c_void_p), ("bvh", C.c_void_p)]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} missing: build it with `make -C oracle`")
    lib = C.CDLL(LIB_PATH)
    f = C.c_float
    lib.oracle_pcg_hash.restype = C.c_uint32
    lib.oracle_pcg_hash.argtypes = [C.c_uint32]
    lib.oracle_rand.restype = f
    lib.oracle_rand.argtypes = [C.POINTER(C.c_uint32)]
    lib.oracle_libm_domain_mismatches.restype = C.c_uint64
    lib.oracle_libm_domain_mismatches.argtypes = [C.c_uint32, C.c_uint32]
    for n in ("oracle_logf", "oracle_cosf", "oracle_expf", "oracle_logf_rand", "oracle_cosf_2pi"):
        getattr(lib, n).restype = f
        getattr(lib, n).argtypes = [f]
    lib.oracle_random_direction.restype = None
    lib.oracle_random_direction.argtypes = [C.POINTER(C.c_uint32), C.c_void_p]
    lib.oracle_ray_box.restype = None
    lib.oracle_ray_box.argtypes = [C.c_void_p] * 5
    lib.oracle_ray_sphere.restype = f
    lib.oracle_ray_sphere.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, f]
    lib.oracle_ray_triangle.restype = f
    lib.oracle_ray_triangle.argtypes = [C.c_void_p] * 5
    lib.oracle_render.restype = C.c_int
    lib.oracle_render.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                  C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(_Counters)]
    lib.oracle_composite.restype = None
    lib.oracle_composite.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]
    lib.oracle_bvh_build.restype = C.c_uint32
    lib.oracle_bvh_build.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]
    return lib


lib = _load()


def _f3(v):
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


def pcg_hash(x: int) -> int:
    return int(lib.oracle_pcg_hash(x & 0xFFFFFFFF))


def rand_stream(seed: int, n: int):
    """n successive rand() values from state `seed`; returns (floats, states after each draw)."""
    s = C.c_uint32(seed & 0xFFFFFFFF)
    vals, states = [], []
    for _ in range(n):
        vals.append(lib.oracle_rand(C.byref(s)))
        states.append(s.value)
    return np.array(vals, np.float32), states


def random_direction(seed: int):
    s = C.c_uint32(seed & 0xFFFFFFFF)
    out = np.zeros(3, np.float32)
    lib.oracle_random_direction(C.byref(s), out.ctypes.data)
    return out, s.value


def logf(x: float) -> np.float32:
    return np.float32(lib.oracle_logf(x))


def cosf(x: float) -> np.float32:
    return np.float32(lib.oracle_cosf(x))


def expf(x: float) -> np.float32:
    return np.float32(lib.oracle_expf(x))


def ray_box(o, d, bmin, bmax):
    out = np.zeros(2, np.float32)
    a = [_f3(o), _f3(d), _f3(bmin), _f3(bmax)]
    lib.oracle_ray_box(*[x.ctypes.data for x in a], out.ctypes.data)
    return out


def ray_sphere(o, d, c, r):
    a = [_f3(o), _f3(d), _f3(c)]
    return np.float32(lib.oracle_ray_sphere(*[x.ctypes.data for x in a], np.float32(r)))


def ray_triangle(o, d, a, b, c):
    arr = [_f3(o), _f3(d), _f3(a), _f3(b), _f3(c)]
    return np.float32(lib.oracle_ray_triangle(*[x.ctypes.data for x in arr]))


def bvh_build(positions: np.ndarray, indices: np.ndarray, node_dtype):
    """Oracle midpoint BVH (PathTracingRenderer.jai:147-217). Returns (nodes, permuted indices)."""
    pos = np.ascontiguousarray(positions, dtype=np.float32)
    idx = np.ascontiguousarray(indices, dtype=np.uint32).copy()
    max_nodes = max(1, 2 * (idx.size // 3))
    nodes = np.zeros(max_nodes, dtype=node_dtype)
    n = lib.oracle_bvh_build(pos.ctypes.data, idx.ctypes.data, idx.size, nodes.ctypes.data, max_nodes)
    if n == 0:
        raise RuntimeError("oracle BVH build overflow")
    return nodes[:n].copy(), idx


def render(sd: np.ndarray, materials: np.ndarray, spheres: np.ndarray, meshes, width: int, height: int,
           y0: int = 0, rows: int | None = None, image: np.ndarray | None = None, threads: int = 1):
    """Render rows [y0, y0+rows) of a width x height frame. `meshes` = list of (positions, indices, nodes)
    numpy arrays (one per draw command). `image` (float32 [rows, width, 4]) is read-modify-written like the
    reference's imageLoad/imageStore; a zero image is used when None. Returns (image, counters dict)."""
    rows = height - y0 if rows is None else rows
    sd = np.ascontiguousarray(sd)
    assert sd.dtype.itemsize == SCENE_DATA_ITEMSIZE
    mats = np.ascontiguousarray(materials)
    sph = np.ascontiguousarray(spheres)
    keep = []
    draws = (_Draw * max(1, len(meshes)))()
    for i, (pos, idx, nodes) in enumerate(meshes):
        p = np.ascontiguousarray(pos, dtype=np.float32)
        ix = np.ascontiguousarray(idx, dtype=np.uint32)
        nd = np.ascontiguousarray(nodes)
        keep += [p, ix, nd]
        draws[i] = _Draw(p.ctypes.data, ix.ctypes.data, nd.ctypes.data)
    if image is None:
        image = np.zeros((rows, width, 4), np.float32)
    else:
        image = np.ascontiguousarray(image, dtype=np.float32).copy()
        assert image.shape == (rows, width, 4)
    cnt = _Counters()
    rc = lib.oracle_render(sd.ctypes.data, mats.ctypes.data if mats.size else None,
                           sph.ctypes.data if sph.size else None, C.addressof(draws), image.ctypes.data,
                           width, height, y0, rows, threads, C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed with {rc}")
    return image, {n: int(getattr(cnt, n)) for n in COUNTER_FIELDS}


def render_scene(scene, width, height, max_bounce=3, samples=1, frame=0, y0=0, rows=None, image=None,
                 threads=1, sd=None):
    """Convenience: render a wcpt.scene.HostScene (data only is read from it)."""
    if sd is None:
        sd = scene.scene_data(width, height, max_bounce=max_bounce, samples=samples, frame=frame)
    meshes = [(m.positions, m.indices, m.nodes) for m in scene.meshes]
    return render(sd, scene.materials, scene.spheres, meshes, width, height, y0=y0, rows=rows, image=image,
                  threads=threads)


def composite(img: np.ndarray):
    """composite.comp (gamma 1/2.2 + PBR Neutral) of a float4 image: returns (rgba32f, rgba8)."""
    a = np.ascontiguousarray(img, dtype=np.float32)
    n = a.size // 4
    out32 = np.empty(a.shape, dtype=np.float32)
    out8 = np.empty(a.shape, dtype=np.uint8)
    lib.oracle_composite(a.ctypes.data, n, out32.ctypes.data, out8.ctypes.data)
    return out32, out8
