import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libANN.so")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture(scope="session")
def gpu():
    """The product library on a real device; a missing library or device is a test failure, not a skip."""
    import tiler_amd
    try:  # torch's HIP runtime first (tests that hand torch-allocated HBM to libANN.so need it; bench.py's order)
        import torch
        torch.cuda.init()
    except Exception:
        pass
    lib = tiler_amd.load()
    rc = lib.tiler_init(0)
    assert rc == 0, f"tiler_init failed: {tiler_amd.last_error()}"
    return tiler_amd
