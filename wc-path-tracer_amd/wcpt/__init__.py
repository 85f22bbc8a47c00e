"""wcpt — MI355X-native path-tracing compute path (drop-in for pathTracer.comp of myri4/WC-Path-tracer).

The compute lives in libwcpt.so (hand-written HIP for gfx950 behind the C-ABI of include/wcpt.h); this
package is the Python host mirror used by tests and the benchmark.
"""
from ._lib import (COUNTER_FIELDS, DRAW_COMMAND_DTYPE, EXPORTED_SYMBOLS, KERNEL_AUTO, KERNEL_MEGAKERNEL,
                   KERNEL_WAVEFRONT, LIB_PATH, MATERIAL_DIELECTRIC, MATERIAL_DTYPE, MATERIAL_METAL, NODE_DTYPE,
                   SCENE_DATA_DTYPE, SPHERE_DTYPE, Camera, WcptError, lib)
from .renderer import Context, DeviceScene, Editor, Group, PathTracingRenderer, group_unique_id
from . import scene
from . import _lib

__all__ = [
    "COUNTER_FIELDS", "DRAW_COMMAND_DTYPE", "EXPORTED_SYMBOLS", "KERNEL_AUTO", "KERNEL_MEGAKERNEL",
    "KERNEL_WAVEFRONT", "LIB_PATH", "MATERIAL_DIELECTRIC", "MATERIAL_DTYPE", "MATERIAL_METAL", "NODE_DTYPE",
    "SCENE_DATA_DTYPE", "SPHERE_DTYPE", "Camera", "WcptError", "lib", "Context", "DeviceScene",
    "PathTracingRenderer", "Editor", "Group", "group_unique_id", "scene", "device_count", "device_pci_bus_id", "runtime_version", "build_id",
]


def device_count() -> int:
    import ctypes as C
    n = C.c_int()
    lib.wcpt_device_count(C.byref(n))
    return n.value


def device_pci_bus_id(device: int) -> str:
    """wcpt_device_pci_bus_id: the GPU's PCI bus id, the same in every process whatever its device ordinals."""
    import ctypes as C
    buf = C.create_string_buffer(64)
    _lib.check(lib.wcpt_device_pci_bus_id(device, buf, 64))
    return buf.value.decode()


def build_id() -> str:
    """wcpt_build_id: hash of the library's sources and compile flags (profiles record the build they measured)."""
    return lib.wcpt_build_id().decode()


def runtime_version() -> int:
    """hipRuntimeGetVersion of the HIP runtime libwcpt.so is bound to (e.g. 70226090 = ROCm 7.2)."""
    import ctypes as C
    v = C.c_int()
    _lib.check(lib.wcpt_runtime_version(C.byref(v)))
    return v.value
