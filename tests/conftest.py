import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "wc-path-tracer_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP path of libwcpt.so)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def _have_gpu():
    try:
        import wcpt
        return wcpt.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx():
    import wcpt
    if not _have_gpu():
        pytest.fail("no HIP device visible: -m gpu tests must run on an MI355X box")
    ctx = wcpt.Context(0)
    yield ctx
    ctx.close()
