import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libarslam_lm.so)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def lm():
    """The HIP library; GPU tests fail loudly (no fallback) if it or the GPU is missing."""
    from ar_slam_amd import build, lm as L
    build.build()
    assert L.device_count() > 0, "no HIP device visible: GPU tests need an MI355X"
    return L
