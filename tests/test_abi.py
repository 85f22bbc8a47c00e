"""The C-ABI surface (no GPU compute): the library loads, exports every symbol include/wcpt.h declares, keeps the
reference byte layouts, and fails with error codes (never aborts) when no device is present."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import wcpt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "wcpt.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wcpt_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported():
    names = declared_functions()
    assert len(names) >= 30
    lib = C.CDLL(wcpt.LIB_PATH)
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(wcpt.EXPORTED_SYMBOLS), set(names) ^ set(wcpt.EXPORTED_SYMBOLS)


def test_abi_version():
    assert wcpt.lib.wcpt_abi_version() == wcpt._lib.ABI_VERSION == 4


def test_option_and_kernel_constants_match_header():
    """The Python mirror's option / kernel numbers are the header's (renumbering one side breaks callers)."""
    text = open(HEADER).read()
    options = dict(re.findall(r"#define WCPT_OPTION_(\w+)\s+(\d+)", text))
    assert len(options) >= 9
    for name, value in options.items():
        assert getattr(wcpt._lib, "OPTION_" + name) == int(value), name
    assert len(set(options.values())) == len(options), "duplicate option numbers"
    kernels = dict(re.findall(r"#define WCPT_KERNEL_(\w+)\s+(\d+)", text))
    for name, value in kernels.items():
        assert getattr(wcpt, "KERNEL_" + name) == int(value), name


def test_layouts_match_reference():
    """GLSL scalar layouts (pathTracer.comp:10-95) == Jai structs (PathTracingRenderer.jai:38-140)."""
    sd = wcpt.SCENE_DATA_DTYPE
    assert sd.itemsize == 164
    assert [sd.fields[n][1] for n in ("inverseProjection", "inverseView", "position", "maxBounceCount",
                                      "samples", "sphereCount", "drawCommandCount", "renderedFramesCount",
                                      "boxID")] == [0, 64, 128, 140, 144, 148, 152, 156, 160]
    m = wcpt.MATERIAL_DTYPE
    assert m.itemsize == 60
    assert [m.fields[n][1] for n in m.names] == [0, 4, 16, 28, 32, 36, 40, 52, 56]
    assert wcpt.SPHERE_DTYPE.itemsize == 20 and wcpt.NODE_DTYPE.itemsize == 32
    assert wcpt.DRAW_COMMAND_DTYPE.itemsize == 32
    assert [wcpt.DRAW_COMMAND_DTYPE.fields[n][1] for n in wcpt.DRAW_COMMAND_DTYPE.names] == [0, 8, 16, 24, 28]


def test_header_compiles_as_c_with_layout_asserts(tmp_path):
    src = tmp_path / "t.c"
    src.write_text(f'''#include "{HEADER}"
#include <stddef.h>
_Static_assert(sizeof(wcpt_scene_data) == 164, "SceneData");
_Static_assert(offsetof(wcpt_scene_data, renderedFramesCount) == 156, "frames");
_Static_assert(sizeof(wcpt_material) == 60, "Material");
_Static_assert(offsetof(wcpt_material, ior) == 56, "ior");
_Static_assert(sizeof(wcpt_sphere) == 20, "Sphere");
_Static_assert(sizeof(wcpt_node) == 32, "Node");
_Static_assert(sizeof(wcpt_draw_command) == 32, "DrawCommand");
_Static_assert(sizeof(wcpt_counters) == 16 * 8, "counters (ABI 2)");
_Static_assert(offsetof(wcpt_counters, ref_stack_overflow_segments) == 14 * 8, "reference-stack fields last");
_Static_assert(WCPT_PAYLOAD_RGB32F == 3 && WCPT_PAYLOAD_RGBA32F == 4 && WCPT_PAYLOAD_DISPLAY_RGBA8 == 8, "payloads");
int main(void) {{ return 0; }}
''')
    rc = os.system(f"gcc -std=c99 -Wall -Werror -c {src} -o {tmp_path / 't.o'}")
    assert rc == 0


@pytest.mark.skipif(wcpt.device_count() > 0, reason="checks the no-device error path")
def test_no_device_errors_cleanly():
    h = C.c_void_p()
    rc = wcpt.lib.wcpt_create(0, C.byref(h))
    assert rc == -3 and not h.value                         # WCPT_ERROR_INITIALIZATION_FAILED
    assert b"no HIP device" in wcpt.lib.wcpt_last_error(None)
    with pytest.raises(wcpt.WcptError):
        wcpt.Context(0)


def test_null_handles_rejected():
    assert wcpt.lib.wcpt_render(None, None, 0, 0, 0) == -1001
    assert wcpt.lib.wcpt_sync(None) == -1001
    assert wcpt.lib.wcpt_set_gather_output(None, 0, 0, 3) == -1001
    assert wcpt.lib.wcpt_buffer_device_address(None, 1) == 0
    assert wcpt.lib.wcpt_destroy(None) == 0
    n = C.c_int(-1)
    assert wcpt.lib.wcpt_device_count(C.byref(n)) == 0 and n.value >= 0


def test_python_package_fails_loudly_without_library(tmp_path):
    """No silent fallback: importing the package with the .so missing raises."""
    import shutil
    import subprocess
    import sys
    pkg = tmp_path / "pkg"
    shutil.copytree(os.path.join(ROOT, "wc-path-tracer_amd", "wcpt"), pkg / "wcpt")
    r = subprocess.run([sys.executable, "-c", "import wcpt"], cwd=pkg, capture_output=True, text=True)
    assert r.returncode != 0 and "libwcpt.so not found" in r.stderr


def test_counters_struct_matches_header():
    assert C.sizeof(wcpt._lib.Counters) == 128
    assert wcpt._lib.Counters.ref_stack_overflow_segments.offset == 14 * 8
    assert wcpt.COUNTER_FIELDS[-2:] == ("ref_stack_overflow_segments", "ref_stack_max")


def test_group_entry_points_reject_bad_arguments():
    """wcpt_group_*: argument checks come before any device work, and nothing aborts without a device."""
    lib = wcpt.lib
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 1)
    assert lib.wcpt_group_create(devs, 2, 0, None) == -1000
    assert lib.wcpt_group_create(None, 1, 0, C.byref(h)) == -1000
    assert lib.wcpt_group_create(devs, 0, 0, C.byref(h)) == -1000
    assert lib.wcpt_group_create(devs, 2, 2, C.byref(h)) == -1000     # root outside the group
    assert lib.wcpt_group_destroy(None) == 0
    assert lib.wcpt_group_context(None, 0) is None
    assert lib.wcpt_group_create_screen(None, 8, 8) == -1001
    assert lib.wcpt_group_set_output(None, 4, 0, 0) == -1001
    assert lib.wcpt_group_sync(None) == -1001
    assert lib.wcpt_group_create_ex(devs, 2, 0, 7, C.byref(h)) == -1000  # unknown transport
    assert lib.wcpt_group_create_rank(0, 2, 2, 0, None, C.byref(h)) == -1000  # rank outside the group
    assert lib.wcpt_group_create_rank(0, 2, 1, 0, None, C.byref(h)) == -1000  # N > 1 needs the unique id
    assert lib.wcpt_group_create_rank(0, 2, 0, 3, None, C.byref(h)) == -1000  # root outside the group
    assert lib.wcpt_group_set_option(None, 1, 1) == -1001
    assert lib.wcpt_group_info_get(None, None) == -1001
    assert lib.wcpt_group_render(None, None, None, None, None) == -1001
    if wcpt.device_count() == 0:
        assert lib.wcpt_group_create(devs, 1, 0, C.byref(h)) == -3     # WCPT_ERROR_INITIALIZATION_FAILED
        assert lib.wcpt_group_create_ex(devs, 2, 0, 1, C.byref(h)) == -3
        assert lib.wcpt_group_create_rank(0, 1, 0, 0, None, C.byref(h)) == -3
        assert not h.value
        with pytest.raises(wcpt.WcptError):
            wcpt.Group([0])


def test_group_constants_match_header():
    """Transport / option numbers and the info struct of the group API are the header's."""
    text = open(HEADER).read()
    for name, value in re.findall(r"#define WCPT_GROUP_(\w+?)\s+(\d+)", text):
        assert getattr(wcpt._lib, "GROUP_" + name) == int(value), name
    fields = re.search(r"typedef struct wcpt_group_info \{(.*?)\} wcpt_group_info;", text, re.S).group(1)
    fields = re.sub(r"/\*.*?\*/", "", fields, flags=re.S)
    names = re.findall(r"(?:int32_t|uint64_t)\s+(\w+);", fields)
    assert names == [n for n, _ in wcpt._lib.GroupInfo._fields_]
    assert C.sizeof(wcpt._lib.GroupInfo) == 8 * 4 + 8 + 8


def test_runtime_version_reported():
    v = wcpt.runtime_version()
    assert v >= 70000000, v   # ROCm 7.x HIP runtime (hipRuntimeGetVersion works without a device)
