"""Host-side scene inputs: OBJ loading, BVH building, camera, synthetic scenes (all through libwcpt.so).

Mirrors ``LoadModel`` (src/PathTracingRenderer.jai:219-270): OBJ -> unique vertices + fan-triangulated
indices (src/ModelLoader.jai:60-141) -> midpoint BVH with BVH-permuted indices (:147-217, :228-233).
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field

import numpy as np

from ._lib import (MATERIAL_DTYPE, NODE_DTYPE, SCENE_DATA_DTYPE, SPHERE_DTYPE, Camera, Mesh, SceneC, check,
                   lib, ptr)


@dataclass
class HostMesh:
    positions: np.ndarray          # float32 [V, 3]
    indices: np.ndarray            # uint32 [I]

    @property
    def triangle_count(self) -> int:
        return int(self.indices.size // 3)


@dataclass
class HostBVH:
    positions: np.ndarray          # float32 [V, 3]
    indices: np.ndarray            # uint32 [I], BVH-permuted
    nodes: np.ndarray              # NODE_DTYPE [N]

    def depth(self) -> int:
        """Number of node levels (root = 1)."""
        best, stack = 0, [(0, 1)]
        while stack:
            i, d = stack.pop()
            best = max(best, d)
            n = self.nodes[i]
            if n["triangleCount"] == 0:
                left = int(n["leftNodeOrTriangleIndex"])
                stack.append((left, d + 1))
                stack.append((left + 1, d + 1))
        return best


@dataclass
class HostScene:
    name: str
    materials: np.ndarray          # MATERIAL_DTYPE [M]
    spheres: np.ndarray            # SPHERE_DTYPE [S]
    camera: Camera
    meshes: list = field(default_factory=list)   # list[HostBVH], one per draw command

    def scene_data(self, width: int, height: int, max_bounce: int = 3, samples: int = 1, frame: int = 0,
                   camera: Camera | None = None) -> np.ndarray:
        """SceneData for a frame, as Render fills it (PathTracingRenderer.jai:410-422)."""
        cam = camera if camera is not None else self.camera
        cam = update_camera(cam, width / height)
        sd = np.zeros((), dtype=SCENE_DATA_DTYPE)
        sd["inverseProjection"] = np.ctypeslib.as_array(cam.inverseProjection)
        sd["inverseView"] = np.ctypeslib.as_array(cam.inverseView)
        sd["position"] = np.ctypeslib.as_array(cam.position)
        sd["maxBounceCount"] = max_bounce
        sd["samples"] = samples
        sd["sphereCount"] = len(self.spheres)
        sd["drawCommandCount"] = len(self.meshes)
        sd["renderedFramesCount"] = frame
        return sd


def _mesh_from_c(m: Mesh) -> HostMesh:
    pos = np.ctypeslib.as_array(m.positions, shape=(m.vertex_count * 3,)).copy() if m.vertex_count else \
        np.zeros(0, np.float32)
    idx = np.ctypeslib.as_array(m.indices, shape=(m.index_count,)).copy() if m.index_count else \
        np.zeros(0, np.uint32)
    return HostMesh(pos.astype(np.float32).reshape(-1, 3), idx.astype(np.uint32))


def obj_parse(text: str | bytes) -> HostMesh:
    data = text.encode() if isinstance(text, str) else text
    m = Mesh()
    check(lib.wcpt_obj_parse(data, len(data), C.byref(m)))
    try:
        return _mesh_from_c(m)
    finally:
        lib.wcpt_mesh_free(C.byref(m))


def obj_load(path: str) -> HostMesh:
    m = Mesh()
    check(lib.wcpt_obj_load(path.encode(), C.byref(m)))
    try:
        return _mesh_from_c(m)
    finally:
        lib.wcpt_mesh_free(C.byref(m))


def mesh_to_obj(mesh: HostMesh) -> bytes:
    pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
    idx = np.ascontiguousarray(mesh.indices, dtype=np.uint32)
    m = Mesh(pos.ctypes.data_as(C.POINTER(C.c_float)), pos.shape[0], idx.ctypes.data_as(C.POINTER(C.c_uint32)),
             idx.size)
    out, n = C.c_void_p(), C.c_uint64()
    check(lib.wcpt_mesh_to_obj(C.byref(m), C.byref(out), C.byref(n)))
    try:
        return C.string_at(out, n.value)
    finally:
        lib.wcpt_string_free(out)


def bvh_build(mesh: HostMesh, builder: str = "midpoint") -> HostBVH:
    """Midpoint BVH (PathTracingRenderer.jai:147-217, the reference's) or, with builder="sah", the optional
    binned-SAH builder; returns the permuted index buffer with it."""
    if builder not in ("midpoint", "sah"):
        raise ValueError(f"unknown BVH builder {builder!r}")
    pos = np.ascontiguousarray(mesh.positions, dtype=np.float32)
    idx = np.ascontiguousarray(mesh.indices, dtype=np.uint32).copy()
    max_nodes = max(1, 2 * (idx.size // 3))
    nodes = np.zeros(max_nodes, dtype=NODE_DTYPE)
    used = C.c_uint32()
    fn = lib.wcpt_bvh_build if builder == "midpoint" else lib.wcpt_bvh_build_sah
    check(fn(ptr(pos), pos.shape[0], ptr(idx), idx.size, ptr(nodes), max_nodes, C.byref(used)))
    return HostBVH(pos, idx, nodes[: used.value].copy())


def update_camera(cam: Camera, aspect: float) -> Camera:
    c = Camera()
    C.pointer(c)[0] = cam
    check(lib.wcpt_camera_update(C.byref(c), float(aspect)))
    return c


def make_camera(position=(0.0, 0.0, 0.0), yaw=0.0, pitch=0.0, fov=90.0) -> Camera:
    c = Camera()
    c.position[:] = list(position)
    c.yaw, c.pitch, c.fov = yaw, pitch, fov
    return c


ASSETS_DIR = os.environ.get("WCPT_ASSETS", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                          "assets"))
# The reference's own input: run_tree/data/assets/models/mushroom.obj, loaded by LoadModel
# (PathTracingRenderer.jai:220); a copy of that mesh data ships with the package.
MUSHROOM_OBJ = os.path.join(ASSETS_DIR, "mushroom.obj")
REFERENCE_SCENES = ("reference_init", "reference_init_glass")


def reference_init(glass_dielectric: bool = False, obj_path: str | None = None, bvh: str = "midpoint") -> HostScene:
    """The scene the reference renders after Init (PathTracingRenderer.jai:272-343):

    - LoadModel (:219-243): mushroom.obj through parse_obj_file (ModelLoader.jai:60-141) and the midpoint BVH
      (:147-217) as one draw command (:251-256);
    - the 4 materials and 4 spheres of :322-339 (every material METAL: SetDielectric never sets `type`, :78-82; all
      triangles use material 0, the "glass" one, pathTracer.comp:175);
    - the editor's start camera (editor.jai:25: a default Camera, :6-13): origin, yaw = pitch = 0 (looking along +x),
      fov 90 -- which puts the camera inside the mushroom's bounding box.

    glass_dielectric=True sets material 0's type to DIELECTRIC (the editor's material
    panel can), so the mushroom and the glass sphere refract (ior 1.5, roughness 0.07)."""
    scene = generate("default")
    scene.name = "reference_init_glass" if glass_dielectric else "reference_init"
    if glass_dielectric:
        m = scene.materials.copy()
        m["type"][0] = 1
        scene.materials = m
    scene.meshes = [bvh_build(obj_load(obj_path or MUSHROOM_OBJ), bvh)]
    scene.camera = make_camera(position=(0.0, 0.0, 0.0), yaw=0.0, pitch=0.0, fov=90.0)
    return scene


def generate(name: str, seed: int = 0, via_obj: bool = True, bvh: str = "midpoint") -> HostScene:
    """Synthetic scene -> HostScene. With via_obj the mesh goes through OBJ text and the loader, like
    LoadModel's parse_obj_file (the atrium is the Sponza-scale OBJ of configs 3-5). "reference_init" and
    "reference_init_glass" are the reference's own Init scene (reference_init)."""
    if name in REFERENCE_SCENES:
        return reference_init(glass_dielectric=name.endswith("_glass"), bvh=bvh)
    s = SceneC()
    check(lib.wcpt_scene_generate(name.encode(), seed, C.byref(s)))
    try:
        mats = np.frombuffer(C.string_at(s.materials, s.material_count * MATERIAL_DTYPE.itemsize),
                             dtype=MATERIAL_DTYPE).copy()
        sph = np.frombuffer(C.string_at(s.spheres, s.sphere_count * SPHERE_DTYPE.itemsize),
                            dtype=SPHERE_DTYPE).copy()
        cam = Camera()
        C.pointer(cam)[0] = s.camera
        mesh = _mesh_from_c(s.mesh)
    finally:
        lib.wcpt_scene_free(C.byref(s))
    scene = HostScene(name, mats, sph, cam)
    if mesh.indices.size:
        if via_obj:
            mesh = obj_parse(mesh_to_obj(mesh))
        scene.meshes.append(bvh_build(mesh, bvh))
    return scene


def scene_from_obj(path: str, base: str = "default") -> HostScene:
    """The reference's Init (PathTracingRenderer.jai:272-343): an OBJ model + the default materials/spheres."""
    scene = generate(base)
    scene.name = f"{base}+{path}"
    scene.meshes = [bvh_build(obj_load(path))]
    return scene
