"""Shared fixtures.  `gpu`-marked tests need an MI355X (run via gpurun); the rest run on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import __graft_entry__ as graft  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: full-size configurations")


@pytest.fixture(scope="session")
def orc():
    """CPU oracle (test infrastructure)."""
    return graft.load_oracle()


@pytest.fixture(scope="session")
def pkg():
    """The product package (vrdd_amd); libvr.so must be built."""
    return graft.load_package()


@pytest.fixture(scope="session")
def gpu(pkg):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test run without a HIP device")
    torch.cuda.set_device(0)
    pkg._lib.load()
    return torch.device("cuda", 0)


class _Tuning:
    """vr_set_tuning knobs for one test (kernel-path overrides, occupancy caps,
    layouts); the library reads no environment, so tests set them explicitly"""

    def __init__(self, pkg):
        self.pkg = pkg

    def set(self, key, value):
        self.pkg.set_tuning(key, value)

    def clear(self, key):
        self.pkg.set_tuning(key, None)


@pytest.fixture
def tune(pkg):
    """Tuning knobs, all cleared when the test ends."""
    pkg.clear_tuning()
    yield _Tuning(pkg)
    pkg.clear_tuning()
