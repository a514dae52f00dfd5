import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DRAGON = os.path.join(ROOT, "data", "dragon.ply")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def dragon():
    from oracle import oracle
    return oracle.load_ply(DRAGON)


@pytest.fixture(scope="session")
def ctx():
    """The GPU context.  Fails (does not skip) when the HIP library or device is missing."""
    import simpleraytracing_amd as xrt
    c = xrt.Context(int(os.environ.get("XRT_DEVICE", "0")))
    yield c
    c.close()


def bits(a):
    a = np.ascontiguousarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a
