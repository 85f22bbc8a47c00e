"""ctypes binding of libwcpt.so (the C-ABI declared in include/wcpt.h).

The shared library is built in-tree (``make -C wc-path-tracer_amd``) and lives next to this package. There
is no fallback: if the library is missing, importing :mod:`wcpt` raises, so nothing can silently run a
non-HIP path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(PKG_DIR), "libwcpt.so")
# Kernel-variant experiments (tools/ab_build.sh) point this at another in-tree build of the same sources.
LIB_PATH = os.environ.get("WCPT_LIBRARY", LIB_PATH)

WCPT_SUCCESS = 0
ERRORS = {
    -1: "WCPT_ERROR_OUT_OF_HOST_MEMORY",
    -2: "WCPT_ERROR_OUT_OF_DEVICE_MEMORY",
    -3: "WCPT_ERROR_INITIALIZATION_FAILED",
    -4: "WCPT_ERROR_DEVICE_LOST",
    -13: "WCPT_ERROR_UNKNOWN",
    -1000: "WCPT_ERROR_INVALID_ARGUMENT",
    -1001: "WCPT_ERROR_INVALID_HANDLE",
    -1002: "WCPT_ERROR_STACK_OVERFLOW",
    -1003: "WCPT_ERROR_NO_SCREEN",
    -1004: "WCPT_ERROR_PARSE",
}
WCPT_ERROR_INVALID_ARGUMENT = -1000
WCPT_ERROR_INVALID_HANDLE = -1001
WCPT_ERROR_STACK_OVERFLOW = -1002
WCPT_ERROR_NO_SCREEN = -1003

MATERIAL_METAL = 0
MATERIAL_DIELECTRIC = 1

KERNEL_MEGAKERNEL = 0
KERNEL_WAVEFRONT = 2
KERNEL_AUTO = 1

OPTION_STACK = 1
OPTION_DIAGNOSTICS = 2
OPTION_SORT_RAYS = 3
OPTION_WF_STACK = 4
OPTION_TRIANGLE_CACHE = 5
OPTION_PAIR_RECORDS = 6
OPTION_PACKED_REFS = 7
OPTION_WF_REFILL = 8
DEFAULT_WF_REFILL = 20  # wcpt_runtime.hip
OPTION_MK_TILE_ORDER = 9
OPTION_WF_PIPES = 10
OPTION_PROFILE_REGION = 11
OPTION_WF_FETCH = 12
OPTION_WF_PERSIST = 13
OPTION_GATHER_FRAME_ROWS = 14
OPTION_FRAME_OVERLAP = 15
DEFAULT_WF_PIPES = 0  # wcpt_runtime.hip: by queue length (2 or 3)

# gather payload formats (wcpt_set_gather_output, wcpt_group_set_output)
PAYLOAD_RGB32F = 3
PAYLOAD_RGBA32F = 4
PAYLOAD_DISPLAY_RGBA8 = 8
PAYLOAD_PIXEL_BYTES = {PAYLOAD_RGB32F: 12, PAYLOAD_RGBA32F: 16, PAYLOAD_DISPLAY_RGBA8: 4}

# ---- POD types (byte layouts of include/wcpt.h == the reference's GLSL scalar layouts) -------------------
SCENE_DATA_DTYPE = np.dtype([
    ("inverseProjection", "<f4", (16,)), ("inverseView", "<f4", (16,)), ("position", "<f4", (3,)),
    ("maxBounceCount", "<u4"), ("samples", "<u4"), ("sphereCount", "<u4"), ("drawCommandCount", "<u4"),
    ("renderedFramesCount", "<u4"), ("boxID", "<u4")])
MATERIAL_DTYPE = np.dtype([
    ("type", "<u4"), ("albedo", "<f4", (3,)), ("emission", "<f4", (3,)), ("emissionStrength", "<f4"),
    ("metallic", "<f4"), ("roughness", "<f4"), ("absorption", "<f4", (3,)), ("absorptionStrength", "<f4"),
    ("ior", "<f4")])
SPHERE_DTYPE = np.dtype([("position", "<f4", (3,)), ("radius", "<f4"), ("material", "<u4")])
NODE_DTYPE = np.dtype([("min", "<f4", (3,)), ("max", "<f4", (3,)), ("leftNodeOrTriangleIndex", "<u4"),
                       ("triangleCount", "<u4")])
DRAW_COMMAND_DTYPE = np.dtype([("vertexBuffer", "<u8"), ("indexBuffer", "<u8"), ("bvhBuffer", "<u8"),
                               ("indexCount", "<u4"), ("_pad", "<u4")])
WORK_FIELDS = ("pixels", "segments", "sphere_tests", "node_pops", "interior_visits", "triangle_tests",
               "hits", "draw_fetches")
DIAG_FIELDS = ("wave_interior_steps", "lane_interior_steps", "wave_triangle_steps", "lane_triangle_steps",
               "wave_segment_steps", "lane_segment_steps")
# the reference's uint nodeStack[32] (pathTracer.comp:151): segments that write past it, and its deepest use (a max)
REF_STACK_FIELDS = ("ref_stack_overflow_segments", "ref_stack_max")
COUNTER_FIELDS = WORK_FIELDS + REF_STACK_FIELDS
# multi-device groups (wcpt_group_*)
GROUP_TRANSPORT_RCCL = 0
GROUP_TRANSPORT_COPY = 1
GROUP_TRANSPORT_DIRECT = 2
GROUP_UNIQUE_ID_BYTES = 128
GROUP_OPTION_OVERLAP = 1
GROUP_OPTION_THREADS = 2
GROUP_OPTION_TIMEOUT_MS = 3
GROUP_OPTION_ROW_STRIPE = 4
ABI_VERSION = 4
assert SCENE_DATA_DTYPE.itemsize == 164 and MATERIAL_DTYPE.itemsize == 60 and SPHERE_DTYPE.itemsize == 20
assert NODE_DTYPE.itemsize == 32 and DRAW_COMMAND_DTYPE.itemsize == 32


class Counters(C.Structure):
    """wcpt_counters (include/wcpt.h): the 8 work counters, 6 SIMD diagnostics, the 2 reference-stack fields."""
    _fields_ = [(n, C.c_uint64) for n in WORK_FIELDS + DIAG_FIELDS + REF_STACK_FIELDS]

    def as_dict(self, diagnostics: bool = False):
        names = COUNTER_FIELDS + (DIAG_FIELDS if diagnostics else ())
        return {n: int(getattr(self, n)) for n in names}


class Mesh(C.Structure):
    _fields_ = [("positions", C.POINTER(C.c_float)), ("vertex_count", C.c_uint32),
                ("indices", C.POINTER(C.c_uint32)), ("index_count", C.c_uint32)]


class Camera(C.Structure):
    """PathTracingRenderer.jai:6-20 (matrices column-major, as the shader reads them)."""
    _fields_ = [("position", C.c_float * 3), ("direction", C.c_float * 3), ("yaw", C.c_float),
                ("pitch", C.c_float), ("fov", C.c_float), ("projection", C.c_float * 16),
                ("view", C.c_float * 16), ("inverseProjection", C.c_float * 16),
                ("inverseView", C.c_float * 16)]


class GroupInfo(C.Structure):
    """wcpt_group_info (include/wcpt.h)."""
    _fields_ = [(n, C.c_int32) for n in ("nranks", "local_ranks", "first_local_rank", "root", "transport", "overlap",
                                         "distinct_devices", "broken")] + [("frames", C.c_uint64),
                                                                           ("issue_threads", C.c_int32),
                                                                           ("_pad", C.c_int32)]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class SceneC(C.Structure):
    _fields_ = [("mesh", Mesh), ("materials", C.c_void_p), ("material_count", C.c_uint32),
                ("spheres", C.c_void_p), ("sphere_count", C.c_uint32), ("camera", Camera)]


_p = C.c_void_p
_u32 = C.c_uint32
_u64 = C.c_uint64
_i = C.c_int

_PROTOTYPES = {
    "wcpt_abi_version": (_i, []),
    "wcpt_build_id": (C.c_char_p, []),
    "wcpt_device_count": (_i, [C.POINTER(_i)]),
    "wcpt_last_kernel": (_i, [_p, C.POINTER(_i)]),
    "wcpt_device_pci_bus_id": (_i, [_i, C.c_char_p, _i]),
    "wcpt_create": (_i, [_i, C.POINTER(_p)]),
    "wcpt_destroy": (_i, [_p]),
    "wcpt_last_error": (C.c_char_p, [_p]),
    "wcpt_set_stream": (_i, [_p, _p]),
    "wcpt_set_kernel": (_i, [_p, _i]),
    "wcpt_set_option": (_i, [_p, _i, _i]),
    "wcpt_buffer_alloc": (_i, [_p, _u64, C.POINTER(_u64)]),
    "wcpt_buffer_upload": (_i, [_p, _u64, _p, _u64, _u64]),
    "wcpt_buffer_download": (_i, [_p, _u64, _p, _u64, _u64]),
    "wcpt_buffer_size": (_i, [_p, _u64, C.POINTER(_u64)]),
    "wcpt_buffer_device_address": (_u64, [_p, _u64]),
    "wcpt_buffer_free": (_i, [_p, _u64]),
    "wcpt_create_screen": (_i, [_p, _u32, _u32]),
    "wcpt_resize": (_i, [_p, _u32, _u32]),
    "wcpt_set_row_range": (_i, [_p, _u32, _u32]),
    "wcpt_set_row_stripes": (_i, [_p, _u32, _u32, _u32, _u32]),
    "wcpt_image_device_ptr": (_u64, [_p]),
    "wcpt_set_external_image": (_i, [_p, _u64, _u64]),
    "wcpt_set_gather_output": (_i, [_p, _u64, _u64, _u32]),
    "wcpt_readback": (_i, [_p, _p, _u64]),
    "wcpt_image_upload": (_i, [_p, _p, _u64]),
    "wcpt_composite": (_i, [_p, _u64, _i]),
    "wcpt_render": (_i, [_p, _p, _u64, _u64, _u64]),
    "wcpt_sync": (_i, [_p]),
    "wcpt_render_counters": (_i, [_p, _p, _u64, _u64, _u64, C.POINTER(Counters)]),
    "wcpt_read_diagnostics": (_i, [_p, C.POINTER(C.c_uint64), _u32]),
    "wcpt_profile_begin": (_i, [_p]),
    "wcpt_profile_end": (_i, [_p, C.POINTER(C.c_double), C.POINTER(_u32)]),
    "wcpt_obj_parse": (_i, [C.c_char_p, _u64, C.POINTER(Mesh)]),
    "wcpt_obj_load": (_i, [C.c_char_p, C.POINTER(Mesh)]),
    "wcpt_mesh_free": (None, [C.POINTER(Mesh)]),
    "wcpt_bvh_build": (_i, [_p, _u32, _p, _u32, _p, _u32, C.POINTER(_u32)]),
    "wcpt_bvh_build_sah": (_i, [_p, _u32, _p, _u32, _p, _u32, C.POINTER(_u32)]),
    "wcpt_camera_update": (_i, [C.POINTER(Camera), C.c_float]),
    "wcpt_scene_generate": (_i, [C.c_char_p, _u32, C.POINTER(SceneC)]),
    "wcpt_scene_free": (None, [C.POINTER(SceneC)]),
    "wcpt_mesh_to_obj": (_i, [C.POINTER(Mesh), C.POINTER(C.c_void_p), C.POINTER(_u64)]),
    "wcpt_string_free": (None, [C.c_void_p]),
    "wcpt_selftest_device": (_i, [_p, _i, _p, _p, _p, _u32]),
    "wcpt_runtime_version": (_i, [C.POINTER(_i)]),
    "wcpt_row_block": (_i, [_u32, _u32, _u32, C.POINTER(_u32), C.POINTER(_u32)]),
    "wcpt_row_stripes": (_i, [_u32, _u32, _u32, _u32, C.POINTER(_u32), C.POINTER(_u32)]),
    "wcpt_group_create": (_i, [C.POINTER(_i), _i, _i, C.POINTER(_p)]),
    "wcpt_group_destroy": (_i, [_p]),
    "wcpt_group_context": (_p, [_p, _i]),
    "wcpt_group_create_screen": (_i, [_p, _u32, _u32]),
    "wcpt_group_set_output": (_i, [_p, _i, _u64, _u64]),
    "wcpt_group_render": (_i, [_p, _p, C.POINTER(_u64), C.POINTER(_u64), C.POINTER(_u64)]),
    "wcpt_group_sync": (_i, [_p]),
    "wcpt_group_create_ex": (_i, [C.POINTER(_i), _i, _i, _i, C.POINTER(_p)]),
    "wcpt_group_unique_id": (_i, [C.POINTER(C.c_uint8)]),
    "wcpt_group_create_rank": (_i, [_i, _i, _i, _i, C.POINTER(C.c_uint8), C.POINTER(_p)]),
    "wcpt_group_set_option": (_i, [_p, _i, _i]),
    "wcpt_group_info_get": (_i, [_p, C.POINTER(GroupInfo)]),
}

EXPORTED_SYMBOLS = tuple(_PROTOTYPES)


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libwcpt.so not found at {LIB_PATH}: build it with `make -C wc-path-tracer_amd` "
            "(or __graft_entry__.build()). There is no non-HIP fallback.")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in _PROTOTYPES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


class WcptError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"{ERRORS.get(code, code)}: {message}")
        self.code = code


def check(rc: int, ctx=None):
    if rc != WCPT_SUCCESS:
        msg = lib.wcpt_last_error(ctx)
        raise WcptError(rc, msg.decode(errors="replace") if msg else "")
    return rc


def ptr(a: np.ndarray) -> int:
    """Raw address of a C-contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data
