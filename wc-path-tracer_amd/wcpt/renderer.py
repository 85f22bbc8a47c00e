"""Device context and the host-side mirror of the reference renderer, over the C-ABI (libwcpt.so).

:class:`Context` is a thin 1:1 wrapper of the C entry points. :class:`PathTracingRenderer` mirrors the Jai
procedures of src/PathTracingRenderer.jai (Init :272, CreateScreen :345, Resize :393, Render :399,
UpdateMaterials :459, Deinit :473, PushMaterial :492) with the same names, fields and frame-counter
sequencing, so that a test reads like driving the reference editor (src/editor.jai:60-80,155-158).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import (COUNTER_FIELDS, DRAW_COMMAND_DTYPE, GROUP_OPTION_ROW_STRIPE, GROUP_TRANSPORT_RCCL,
                   GROUP_UNIQUE_ID_BYTES, OPTION_DIAGNOSTICS,
                   MATERIAL_DTYPE, SCENE_DATA_DTYPE, SPHERE_DTYPE, Camera, Counters, GroupInfo, WcptError, check, lib, ptr)
from . import scene as _scene


class Context:
    """One HIP device context (one stream). Not thread-safe, like the reference's single render thread."""

    def __init__(self, device: int = 0, _handle=None):
        self.owned = _handle is None
        if _handle is None:
            h = C.c_void_p()
            check(lib.wcpt_create(device, C.byref(h)))
            _handle = h
        self.h = _handle
        self.device = device

    @classmethod
    def borrowed(cls, handle, device: int) -> "Context":
        """A context owned by someone else (a Group's rank context): close() leaves it alone."""
        return cls(device, _handle=C.c_void_p(handle))

    # -- lifetime -----------------------------------------------------------------------------------
    def close(self):
        if self.h and self.owned:
            lib.wcpt_destroy(self.h)
        self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        return check(rc, self.h)

    # -- configuration -------------------------------------------------------------------------------
    def set_kernel(self, variant: int):
        self._chk(lib.wcpt_set_kernel(self.h, variant))

    def last_kernel(self) -> int:
        """The variant the last render ran (WCPT_KERNEL_AUTO resolved per render)."""
        v = C.c_int()
        self._chk(lib.wcpt_last_kernel(self.h, C.byref(v)))
        return v.value

    def set_option(self, option: int, value: int):
        self._chk(lib.wcpt_set_option(self.h, option, value))

    def set_stream(self, stream_handle: int | None):
        self._chk(lib.wcpt_set_stream(self.h, stream_handle or None))

    # -- buffers ---------------------------------------------------------------------------------------
    def buffer_alloc(self, nbytes: int) -> int:
        out = C.c_uint64()
        self._chk(lib.wcpt_buffer_alloc(self.h, nbytes, C.byref(out)))
        return out.value

    def buffer_upload(self, buf: int, arr: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(arr)
        self._chk(lib.wcpt_buffer_upload(self.h, buf, ptr(a) if a.nbytes else None, a.nbytes, offset))

    def buffer_download(self, buf: int, nbytes: int, offset: int = 0) -> bytes:
        out = np.empty(nbytes, np.uint8)
        self._chk(lib.wcpt_buffer_download(self.h, buf, ptr(out), nbytes, offset))
        return out.tobytes()

    def buffer_size(self, buf: int) -> int:
        out = C.c_uint64()
        self._chk(lib.wcpt_buffer_size(self.h, buf, C.byref(out)))
        return out.value

    def buffer_address(self, buf: int) -> int:
        a = lib.wcpt_buffer_device_address(self.h, buf)
        if a == 0 and self.buffer_size(buf) > 0:
            raise WcptError(-1001, lib.wcpt_last_error(self.h).decode())
        return a

    def buffer_free(self, buf: int):
        self._chk(lib.wcpt_buffer_free(self.h, buf))

    def buffer_from(self, arr: np.ndarray) -> int:
        a = np.ascontiguousarray(arr)
        b = self.buffer_alloc(max(a.nbytes, 0))
        if a.nbytes:
            self.buffer_upload(b, a)
        return b

    # -- image ----------------------------------------------------------------------------------------
    def create_screen(self, width: int, height: int):
        self._chk(lib.wcpt_create_screen(self.h, width, height))
        self.width, self.height = width, height

    def resize(self, width: int, height: int):
        self._chk(lib.wcpt_resize(self.h, width, height))
        self.width, self.height = width, height

    def set_row_range(self, y0: int, rows: int):
        self._chk(lib.wcpt_set_row_range(self.h, y0, rows))

    def set_row_stripes(self, y_first: int, rows: int, stripe: int, period: int):
        """Interleaved stripes (wcpt_set_row_stripes): `rows` rows, stripes of `stripe` rows every `period` rows from
        frame row y_first, stored back to back."""
        self._chk(lib.wcpt_set_row_stripes(self.h, y_first, rows, stripe, period))

    def set_external_image(self, device_ptr: int, nbytes: int):
        self._chk(lib.wcpt_set_external_image(self.h, device_ptr, nbytes))

    def set_gather_output(self, device_ptr: int, nbytes: int, channels: int = 3):
        """The render also writes each pixel into its payload at device_ptr (0 = off): channels = 3 / 4 (float RGB /
        RGBA of the accumulation) or 8 (PAYLOAD_DISPLAY_RGBA8: composite.comp's display value as RGBA8)."""
        self._chk(lib.wcpt_set_gather_output(self.h, device_ptr, nbytes, channels))

    def image_ptr(self) -> int:
        return lib.wcpt_image_device_ptr(self.h)

    def readback(self, rows: int | None = None) -> np.ndarray:
        rows = self.height if rows is None else rows
        out = np.empty((rows, self.width, 4), np.float32)
        self._chk(lib.wcpt_readback(self.h, ptr(out), out.nbytes))
        return out

    def image_upload(self, img: np.ndarray):
        a = np.ascontiguousarray(img, dtype=np.float32)
        self._chk(lib.wcpt_image_upload(self.h, ptr(a), a.nbytes))

    # -- dispatch ---------------------------------------------------------------------------------------
    def composite(self, dst: int, rgba8: bool = False):
        """composite.comp into device memory at `dst` (asynchronous)."""
        self._chk(lib.wcpt_composite(self.h, dst, 1 if rgba8 else 0))

    def render(self, sd: np.ndarray, materials: int, spheres: int, draws: int):
        sd = np.ascontiguousarray(sd, dtype=SCENE_DATA_DTYPE)
        self._chk(lib.wcpt_render(self.h, ptr(sd), materials, spheres, draws))

    def sync(self):
        self._chk(lib.wcpt_sync(self.h))

    def render_counters(self, sd: np.ndarray, materials: int, spheres: int, draws: int,
                        diagnostics: bool = False) -> dict:
        """Reference-algorithm work counters of one frame (COUNTER_FIELDS); with diagnostics=True also the
        implementation's SIMD-efficiency step counters (DIAG_FIELDS)."""
        sd = np.ascontiguousarray(sd, dtype=SCENE_DATA_DTYPE)
        c = Counters()
        self._chk(lib.wcpt_set_option(self.h, OPTION_DIAGNOSTICS, 1 if diagnostics else 0))
        try:
            self._chk(lib.wcpt_render_counters(self.h, ptr(sd), materials, spheres, draws, C.byref(c)))
        finally:
            lib.wcpt_set_option(self.h, OPTION_DIAGNOSTICS, 0)
        return c.as_dict(diagnostics)

    def read_diagnostics(self) -> list:
        out = (C.c_uint64 * 8)()
        self._chk(lib.wcpt_read_diagnostics(self.h, out, 8))
        return [int(v) for v in out]

    def profile_begin(self):
        self._chk(lib.wcpt_profile_begin(self.h))

    def profile_end(self):
        ms, n = C.c_double(), C.c_uint32()
        self._chk(lib.wcpt_profile_end(self.h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def selftest(self, fn: int, x: np.ndarray, x2: np.ndarray | None = None) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.uint32)
        per = {1: 4, 7: 3}.get(fn, 1)
        out = np.empty(x.size * per, np.uint32)
        x2p = None
        if x2 is not None:
            x2 = np.ascontiguousarray(x2, dtype=np.uint32)
            x2p = ptr(x2)
        self._chk(lib.wcpt_selftest_device(self.h, fn, ptr(x), x2p, ptr(out), x.size))
        return out


class DeviceScene:
    """A HostScene resident in device buffers: the six DBufferManagers of PathTracingRenderer.jai:110-117."""

    def __init__(self, ctx: Context, scene: "_scene.HostScene"):
        self.ctx = ctx
        self.scene = scene
        self.buffers = []
        self.materials = self._buf(scene.materials)
        self.spheres = self._buf(scene.spheres)
        draws = np.zeros(len(scene.meshes), dtype=DRAW_COMMAND_DTYPE)
        for i, m in enumerate(scene.meshes):
            draws[i] = (self._buf(m.positions), self._buf(m.indices), self._buf(m.nodes), m.indices.size, 0)
        self.draws = self._buf(draws)

    def _buf(self, arr: np.ndarray) -> int:
        b = self.ctx.buffer_from(arr)
        self.buffers.append(b)
        return self.ctx.buffer_address(b)

    def addresses(self):
        return self.materials, self.spheres, self.draws

    def free(self):
        for b in self.buffers:
            self.ctx.buffer_free(b)
        self.buffers = []


def group_unique_id() -> bytes:
    """wcpt_group_unique_id: the 128-byte RCCL id the root's process hands to every process of a rank group."""
    buf = (C.c_uint8 * GROUP_UNIQUE_ID_BYTES)()
    check(lib.wcpt_group_unique_id(buf))
    return bytes(buf)


class Group:
    """One frame on several devices (include/wcpt.h wcpt_group_*): rank r renders rows
    [r*H/N, (r+1)*H/N) on its device, and a set output gathers every frame's blocks to the root.

    ``Group(devices, root, transport)`` holds every rank in this process (one host thread, like the reference's
    host); ``Group.rank(device, nranks, rank, root, uid)`` holds one rank of a one-process-per-device group. The
    local ranks are ``self.ranks``; ``context(r)`` is rank r's context (None for a rank of another process)."""

    def __init__(self, devices=None, root: int = 0, transport: int = GROUP_TRANSPORT_RCCL, _rank=None):
        h = C.c_void_p()
        if _rank is None:
            devs = (C.c_int * len(devices))(*devices)
            check(lib.wcpt_group_create_ex(devs, len(devices), root, transport, C.byref(h)))
            self.ranks = list(range(len(devices)))
            self.devices = list(devices)
            self.nranks = len(devices)
        else:
            device, nranks, rank, uid = _rank
            idp = None
            if uid is not None:
                assert len(uid) == GROUP_UNIQUE_ID_BYTES
                idp = (C.c_uint8 * GROUP_UNIQUE_ID_BYTES).from_buffer_copy(uid)
            check(lib.wcpt_group_create_rank(device, nranks, rank, root, idp, C.byref(h)))
            self.ranks = [rank]
            self.devices = [device]
            self.nranks = nranks
        self.h = h
        self.root = root
        self._ctx = {r: Context.borrowed(lib.wcpt_group_context(h, r), d) for r, d in zip(self.ranks, self.devices)}
        self.contexts = [self._ctx[r] for r in self.ranks]

    @classmethod
    def rank(cls, device: int, nranks: int, rank: int, root: int = 0, uid: bytes | None = None) -> "Group":
        return cls(root=root, _rank=(device, nranks, rank, uid))

    def close(self):
        if self.h:
            for c in self.contexts:
                c.h = None
            lib.wcpt_group_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def context(self, rank: int) -> Context | None:
        return self._ctx.get(rank)

    def set_option(self, option: int, value: int):
        check(lib.wcpt_group_set_option(self.h, option, value))
        if option == GROUP_OPTION_ROW_STRIPE:
            self.stripe = value
            if getattr(self, "width", None):
                self._set_rows()

    def info(self) -> dict:
        out = GroupInfo()
        check(lib.wcpt_group_info_get(self.h, C.byref(out)))
        return out.as_dict()

    def create_screen(self, width: int, height: int):
        check(lib.wcpt_group_create_screen(self.h, width, height))
        self.width, self.height = width, height
        self._set_rows()

    def _set_rows(self):
        from .dist import row_stripes
        for r, c in self._ctx.items():   # a rank's context holds only its rows (a block, or interleaved stripes)
            c.width, c.height = self.width, row_stripes(self.height, self.nranks, r, getattr(self, "stripe", 0))[1]

    def set_output(self, fmt: int, dst: int, nbytes: int):
        check(lib.wcpt_group_set_output(self.h, fmt, dst, nbytes))

    def render(self, sd: np.ndarray, materials, spheres, draws):
        """materials / spheres / draws: one device address per local rank, in rank order."""
        n = len(self.ranks)
        sd = np.ascontiguousarray(sd, dtype=SCENE_DATA_DTYPE)
        arr = [(C.c_uint64 * n)(*[int(v) for v in a]) for a in (materials, spheres, draws)]
        check(lib.wcpt_group_render(self.h, ptr(sd), *arr))

    def sync(self):
        check(lib.wcpt_group_sync(self.h))


class PathTracingRenderer:
    """Host mirror of ``PathTracingRenderer`` (src/PathTracingRenderer.jai:92-123) over the C-ABI."""

    def __init__(self, device: int = 0):
        self.renderSize = (0, 0)
        self.samples = 1                 # :119
        self.maxBounceCount = 3          # :120
        self.renderedFramesCount = 0     # :121
        self.boxID = 0                   # :122
        self.materials = np.zeros(0, dtype=MATERIAL_DTYPE)
        self.spheres = np.zeros(0, dtype=SPHERE_DTYPE)
        self.meshes = []
        self.ctx = Context(device)
        self._mat_buf = self._sph_buf = self._draw_buf = None
        self._mesh_bufs = []

    # Init :272-343 — LoadModel + materials/spheres + UpdateMaterials
    def Init(self, model_path: str | None = None, scene: "_scene.HostScene | None" = None):
        if scene is None:
            scene = _scene.generate("default")
            if model_path is not None:
                scene.meshes = [_scene.bvh_build(_scene.obj_load(model_path))]
        self.materials = scene.materials.copy()
        self.spheres = scene.spheres.copy()
        self.meshes = list(scene.meshes)
        self.LoadModel()
        self.UpdateMaterials()

    # LoadModel :219-270 — vertex/index/BVH uploads + one DrawCommand per mesh
    def LoadModel(self):
        draws = np.zeros(len(self.meshes), dtype=DRAW_COMMAND_DTYPE)
        for i, m in enumerate(self.meshes):
            vb, ib, nb = (self.ctx.buffer_from(m.positions), self.ctx.buffer_from(m.indices),
                          self.ctx.buffer_from(m.nodes))
            self._mesh_bufs += [vb, ib, nb]
            draws[i] = (self.ctx.buffer_address(vb), self.ctx.buffer_address(ib), self.ctx.buffer_address(nb),
                        m.indices.size, 0)
        if self._draw_buf is None:
            self._draw_buf = self.ctx.buffer_alloc(0)
        self.ctx.buffer_upload(self._draw_buf, draws)

    # PushMaterial :492-496
    def PushMaterial(self) -> int:
        m = np.zeros(1, dtype=MATERIAL_DTYPE)
        m["absorptionStrength"] = 1.0
        m["ior"] = 1.0
        self.materials = np.concatenate([self.materials, m])
        return len(self.materials) - 1

    # UpdateMaterials :459-471 — re-upload materials and spheres (grow-on-demand)
    def UpdateMaterials(self):
        if self._mat_buf is None:
            self._mat_buf = self.ctx.buffer_alloc(0)
            self._sph_buf = self.ctx.buffer_alloc(0)
        self.ctx.buffer_upload(self._mat_buf, self.materials)
        self.ctx.buffer_upload(self._sph_buf, self.spheres)

    # CreateScreen :345-385
    def CreateScreen(self, size):
        w, h = int(size[0]), int(size[1])
        self.renderSize = (w, h)
        self.ctx.create_screen(w, h)

    # Resize :393-397
    def Resize(self, size):
        self.CreateScreen(size)
        self.renderedFramesCount = 0

    def scene_data(self, camera: Camera) -> np.ndarray:
        """SceneData as Render fills it (:410-422); the camera's matrices must be up to date (Update :22)."""
        sd = np.zeros((), dtype=SCENE_DATA_DTYPE)
        sd["inverseProjection"] = np.ctypeslib.as_array(camera.inverseProjection)
        sd["inverseView"] = np.ctypeslib.as_array(camera.inverseView)
        sd["position"] = np.ctypeslib.as_array(camera.position)
        sd["maxBounceCount"] = self.maxBounceCount
        sd["samples"] = self.samples
        sd["sphereCount"] = len(self.spheres)
        sd["drawCommandCount"] = len(self.meshes)
        sd["renderedFramesCount"] = self.renderedFramesCount
        sd["boxID"] = self.boxID
        return sd

    # Render :399-457
    def Render(self, camera: Camera):
        sd = self.scene_data(camera)
        self.renderedFramesCount += 1    # :423 (the editor adds its own +1 when the camera is still)
        self.ctx.render(sd, self.ctx.buffer_address(self._mat_buf), self.ctx.buffer_address(self._sph_buf),
                        self.ctx.buffer_address(self._draw_buf))

    def Readback(self) -> np.ndarray:
        return self.ctx.readback()

    # Deinit :473-490
    def Deinit(self):
        for b in self._mesh_bufs:
            self.ctx.buffer_free(b)
        self._mesh_bufs = []
        for b in (self._mat_buf, self._sph_buf, self._draw_buf):
            if b is not None:
                self.ctx.buffer_free(b)
        self._mat_buf = self._sph_buf = self._draw_buf = None
        self.ctx.close()


class Editor:
    """The editor's per-frame protocol around the renderer (src/editor.jai:118-158), for frame sequencing:

    - camera input: ``moved`` resets ``renderedFramesCount`` to 0, otherwise the editor adds 1 (:149-152);
    - UpdateEditor (:154-158): camera Update (aspect of the viewport), UpdateMaterials, Render, which uploads
      SceneData with the current count and adds its own 1 (PathTracingRenderer.jai:423).

    So while the camera is still the shader sees every second frame number (1, 3, 5, ... from start-up; 0, 2,
    4, ... after a move), and the progressive ``mix`` weights follow that sequence. ``frame`` returns the
    count the dispatch used.
    """

    def __init__(self, renderer: PathTracingRenderer, camera: Camera):
        self.renderer = renderer
        self.camera = camera

    def frame(self, moved: bool = False) -> int:
        r = self.renderer
        if moved:
            r.renderedFramesCount = 0
        else:
            r.renderedFramesCount += 1
        w, h = r.renderSize
        cam = _scene.update_camera(self.camera, w / h)
        r.UpdateMaterials()
        used = r.renderedFramesCount
        r.Render(cam)
        return used


__all__ = ["Context", "DeviceScene", "Group", "group_unique_id", "PathTracingRenderer", "Editor", "COUNTER_FIELDS"]
