"""Host code under the sanitizers ("race detection / sanitizers: -fsanitize=address on the host side"):
the product's host utilities (wc-path-tracer_amd/host/wcpt_host.cpp -- OBJ loader, midpoint and SAH BVH builders,
camera, scene generators) are compiled here with AddressSanitizer and UndefinedBehaviorSanitizer into a standalone
driver (tests/host_asan_driver.cpp) and run over the reference's mesh, malformed and random OBJ text, random and
degenerate triangle soups, node arrays too small for the tree, and every scene generator. A sanitizer report aborts
the driver (-fno-sanitize-recover); its own structural checks fail it with exit code 1. CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_host_utilities_clean_under_asan_and_ubsan(tmp_path):
    exe = tmp_path / "host_asan_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", "-ffp-contract=off",
           os.path.join(ROOT, "tests", "host_asan_driver.cpp"),
           os.path.join(ROOT, "wc-path-tracer_amd", "host", "wcpt_host.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([str(exe), os.path.join(ROOT, "wc-path-tracer_amd", "assets", "mushroom.obj")],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert "0 failed checks" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr
