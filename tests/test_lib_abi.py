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


def test_recurrent_policy_layout(built_lib):
    """VN_POLICY_LSTM appends W_cat [2048][xcat] (W_ih | pad | W_hh), b_ih, b_hh to the flat
    parameters (host-side layout only: no device call)."""
    from vnav import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    n, a = ctypes.c_int64(), ctypes.c_int64()
    assert lib.vn_policy_create_ex(84, 84, 4, 0, ctypes.byref(h)) == 0
    assert lib.vn_policy_info(h, ctypes.byref(n), ctypes.byref(a), None) == 0
    base = n.value
    assert base == 239397
    assert lib.vn_policy_lstm_info(h, (ctypes.c_int64 * 8)()) != 0  # feed-forward policy has no core
    lib.vn_policy_destroy(h)
    assert lib.vn_policy_create_ex(84, 84, 4, 1, ctypes.byref(h)) == 0
    info = (ctypes.c_int64 * 8)()
    assert lib.vn_policy_lstm_info(h, info) == 0
    lin, xoff, xcat = 512 + 4 + 1, 520, 1032
    assert list(info) == [base, base + 2048 * xcat, base + 2048 * xcat + 2048, xcat, xoff, lin, 512, 0]
    assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
    assert n.value == base + 2048 * xcat + 4096
    lib.vn_policy_destroy(h)
    assert lib.vn_policy_create_ex(84, 84, 4, 16, ctypes.byref(h)) != 0  # unknown flag


def test_unreal_policy_layout(built_lib):
    """VN_POLICY_UNREAL appends, 16-byte aligned, pc_base W [2592][512], b [2592], W1 [32][4][4][64],
    b1 [64], W2 [64][4][4][8], b2 [8], rp W [3][3 FCIN], b [4] (goal.py:94-119); with
    VN_POLICY_BIGHOUSE bignet.py:77-96's one deconv per branch: W1 [32][4][4][8], b1 [8], no
    W2 / b2, rp W [3][3 * 1568]."""
    from vnav import _lib
    lib = _lib.load()
    for hw, fcin in ((84, 288), (174, 2592)):
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        assert lib.vn_policy_create_ex(hw, hw, 4, 1, ctypes.byref(h)) == 0
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        base = n.value
        assert lib.vn_policy_unreal_info(h, (ctypes.c_int64 * 8)()) != 0
        lib.vn_policy_destroy(h)
        assert lib.vn_policy_create_ex(hw, hw, 4, 1 | 8, ctypes.byref(h)) == 0
        info = (ctypes.c_int64 * 8)()
        assert lib.vn_policy_unreal_info(h, info) == 0
        o = (base + 3) // 4 * 4
        sizes = (2592 * 512, 2592, 32 * 16 * 64, 64, 64 * 16 * 8, 8, 3 * 3 * fcin, 4)
        want = [o + sum(sizes[:i]) for i in range(8)]
        assert list(info) == want and all(v % 4 == 0 for v in info)
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        assert n.value == want[-1] + 4
        lib.vn_policy_destroy(h)
    for flags in (4, 4 | 1):
        assert lib.vn_policy_create_ex(84, 84, 4, flags, ctypes.byref(h)) == 0
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        base = n.value
        lib.vn_policy_destroy(h)
        assert lib.vn_policy_create_ex(84, 84, 4, flags | 8, ctypes.byref(h)) == 0
        assert lib.vn_policy_unreal_info(h, info) == 0
        o = (base + 3) // 4 * 4
        sizes = (2592 * 512, 2592, 32 * 16 * 8, 8, 0, 0, 3 * 3 * 1568, 4)
        want = [o + sum(sizes[:i]) for i in range(8)]
        assert list(info) == want and all(v % 4 == 0 for v in info)
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        assert n.value == want[-1] + 4
        lib.vn_policy_destroy(h)
    assert lib.vn_policy_create_ex(84, 84, 4, 4 | 2 | 8, ctypes.byref(h)) != 0  # no aux heads on BigHouseModel


def test_aux_policy_layout(built_lib):
    """VN_POLICY_AUX appends the deconv heads (W1 [32][4][4][48], b1, W2 [48][4][4][8], b2);
    maps 3x3 -> 8x8 -> 18x18 at 84x84 and 9x9 -> 20x20 -> 42x42 at 174x174 (goal.py:150-170)."""
    from vnav import _lib
    lib = _lib.load()
    for hw, base, a_hw, p_hw in ((84, 239397, 8, 18), (174, None, 20, 42)):
        h = ctypes.c_void_p()
        n = ctypes.c_int64()
        assert lib.vn_policy_create_ex(hw, hw, 4, 0, ctypes.byref(h)) == 0
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        plain = n.value
        lib.vn_policy_destroy(h)
        if base is not None:
            assert plain == base
        assert lib.vn_policy_create_ex(hw, hw, 4, 2, ctypes.byref(h)) == 0
        info = (ctypes.c_int64 * 8)()
        assert lib.vn_policy_aux_info(h, info) == 0
        w1 = plain
        assert list(info) == [w1, w1 + 24576, w1 + 24576 + 48, w1 + 24576 + 48 + 6144, a_hw, a_hw, p_hw, p_hw]
        assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
        assert n.value == plain + 24576 + 48 + 6144 + 8
        lib.vn_policy_destroy(h)


def test_bighouse_policy_layout(built_lib):
    """VN_POLICY_BIGHOUSE: BigHouseModel's trunk (bignet.py:28-41) + heads = 863365 parameters
    (the count of the reference module's conv_base/conv_merge/critic/policy_logits), the LSTM
    appended as for the goal net; 84x84 only, no aux heads."""
    from vnav import _lib
    lib = _lib.load()
    h = ctypes.c_void_p()
    n = ctypes.c_int64()
    assert lib.vn_policy_create_ex(84, 84, 4, 4, ctypes.byref(h)) == 0
    assert lib.vn_policy_info(h, ctypes.byref(n), None, None) == 0
    assert n.value == 863365
    lib.vn_policy_destroy(h)
    assert lib.vn_policy_create_ex(84, 84, 4, 5, ctypes.byref(h)) == 0
    info = (ctypes.c_int64 * 8)()
    assert lib.vn_policy_lstm_info(h, info) == 0
    assert info[0] == 863365 and info[5] == 512 + 4 + 1
    lib.vn_policy_destroy(h)
    assert lib.vn_policy_create_ex(174, 174, 4, 4, ctypes.byref(h)) != 0  # Linear(7*7*32) fixes 84x84
    assert lib.vn_policy_create_ex(84, 84, 4, 6, ctypes.byref(h)) != 0    # no aux heads on BigHouse
