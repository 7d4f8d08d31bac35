"""libvnav.so loads and exports every symbol declared in include/vnav.h. CPU only
(no compute calls: the container has no GPU)."""
import ctypes
import os
import re

from conftest import REPO


def declared_symbols():
    text = open(os.path.join(REPO, "include", "vnav.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(vn_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ("vn_create", "vn_destroy", "vn_reset", "vn_step", "vn_set_schedule", "vn_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol(built_lib):
    import torch  # noqa: F401  (shares torch's HIP runtime, as the product does)
    lib = ctypes.CDLL(built_lib)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_ctypes_signatures_cover_header(built_lib):
    from vnav import _lib
    lib = _lib.load()
    syms = declared_symbols()
    assert set(_lib.SIGNATURES) <= set(syms)
    assert lib.vn_version().decode().startswith("vnav")
    # error path without a device: NULL ctx is rejected with a message
    assert lib.vn_step(None, None, None, None, None, None, None, None) != 0
    assert "NULL" in _lib.last_error()
