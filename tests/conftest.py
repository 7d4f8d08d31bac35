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


_TRACE = {"n": 0}


@pytest.fixture(autouse=True)
def _trace_marker(request):
    """VN_TRACE_TESTS=<file>: before each GPU test, record its node id (line k of the file)
    and launch vn_trace_marker(k) so a rocprofv3 kernel trace of the run splits per test
    (tools/test_kernel_map.py). Off unless the variable is set."""
    path = os.environ.get("VN_TRACE_TESTS")
    if not path or request.node.get_closest_marker("gpu") is None:
        yield
        return
    import torch
    from vnav import _lib
    torch.cuda.synchronize()
    _TRACE["n"] += 1
    with open(path, "a") as f:
        f.write("%d\t%s\n" % (_TRACE["n"], request.node.nodeid))
    _lib.check(_lib.load().vn_trace_marker(_TRACE["n"], _lib.stream_ptr(torch.device("cuda", 0))),
               "vn_trace_marker")
    torch.cuda.synchronize()
    yield
    torch.cuda.synchronize()
