import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "a2cat-vn-pytorch_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); runs on the GPU box")


def _lib_path():
    return os.path.join(PKG, "vnav", "_lib", "libvnav.so")


@pytest.fixture(scope="session")
def built_lib():
    """Build libvnav.so in-tree if it is missing (hipcc cross-compiles for gfx950)."""
    if not os.path.exists(_lib_path()):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, stdout=subprocess.DEVNULL)
    return _lib_path()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

    return load
