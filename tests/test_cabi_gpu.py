"""The C ABI driven the way a foreign host binds it: plain ctypes on
libvnav.so with its own struct definition and raw device pointers — no vnav Python layer —
stepping a golden reference trajectory bit-exactly (cached.py:74-99 goldens)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import REPO
from oracle.frames import synth_frames

pytestmark = pytest.mark.gpu


class vn_scene_desc(ctypes.Structure):  # include/vnav.h, as a maintainer would write it
    _fields_ = [("n_states", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("channels", ctypes.c_int32), ("graph", ctypes.POINTER(ctypes.c_int64)),
                ("spd", ctypes.POINTER(ctypes.c_int64)), ("observations", ctypes.POINTER(ctypes.c_uint8)),
                ("reward_goal", ctypes.c_float), ("reward_step", ctypes.c_float),
                ("reward_collision", ctypes.c_float), ("terminal_obs", ctypes.c_int32),
                ("synth_id", ctypes.c_uint32), ("companion", ctypes.POINTER(ctypes.c_uint8))]


def test_raw_ctypes_binding_replays_golden(golden):
    lib = ctypes.CDLL(os.path.join(REPO, "a2cat-vn-pytorch_amd", "vnav", "_lib", "libvnav.so"))
    vp = ctypes.c_void_p
    lib.vn_create.argtypes = [ctypes.POINTER(vn_scene_desc), ctypes.c_int, ctypes.c_int, ctypes.c_uint64, ctypes.c_int,
                              ctypes.POINTER(vp)]
    lib.vn_step.argtypes = [vp] * 8
    lib.vn_reset.argtypes = [vp, vp, vp]
    lib.vn_set_schedule.argtypes = [vp, vp, ctypes.c_int]
    lib.vn_set_autoreset.argtypes = [vp, ctypes.c_int]
    lib.vn_set_max_episode_steps.argtypes = [vp, ctypes.c_int]
    lib.vn_observe.argtypes = [vp] * 5
    lib.vn_destroy.argtypes = [vp]

    h = golden("h5_scenes.npz")
    d = golden("cached_env.npz")
    p = "c3_"
    k = int(d[p + "meta"][0])
    graph = np.ascontiguousarray(h["graph%d" % k], dtype=np.int64)
    spd = np.ascontiguousarray(h["spd%d" % k], dtype=np.int64)
    frames = np.ascontiguousarray(synth_frames(100 + k, np.arange(len(graph)), (84, 84, 3)))
    desc = vn_scene_desc(len(graph), 84, 84, 3, graph.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                         spd.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                         frames.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), 1.0, -0.0, 0.0, 0, 0, None)
    ctx = vp()
    torch.cuda.init()
    assert lib.vn_create(ctypes.byref(desc), 1, 1, 2, 0, ctypes.byref(ctx)) == 0
    try:
        assert lib.vn_set_autoreset(ctx, 0) == 0 and lib.vn_set_max_episode_steps(ctx, 0) == 0
        sched = torch.as_tensor(d[p + "resets"][1:].astype(np.int32), device="cuda").contiguous()
        assert lib.vn_set_schedule(ctx, vp(sched.data_ptr()), sched.shape[0]) == 0
        stream = vp(torch.cuda.current_stream().cuda_stream)
        assert lib.vn_reset(ctx, None, stream) == 0
        a = torch.zeros(1, dtype=torch.int32, device="cuda")
        img = torch.empty((1, 84, 84, 3), dtype=torch.uint8, device="cuda")
        goal = torch.empty_like(img)
        reward = torch.empty(1, dtype=torch.float32, device="cuda")
        done = torch.empty(1, dtype=torch.uint8, device="cuda")
        state = torch.empty(1, dtype=torch.int32, device="cuda")
        for t, act in enumerate(d[p + "actions"]):
            a.fill_(int(act))
            assert lib.vn_step(ctx, vp(a.data_ptr()), vp(img.data_ptr()), vp(goal.data_ptr()), vp(reward.data_ptr()),
                               vp(done.data_ptr()), vp(state.data_ptr()), stream) == 0
            torch.cuda.current_stream().synchronize()
            assert state.item() == d[p + "states"][t], t
            assert reward.cpu().numpy().view(np.uint32)[0] == d[p + "reward_bits"][t], t
            assert bool(done.item()) == bool(d[p + "dones"][t]), t
            assert np.array_equal(img[0].cpu().numpy(), frames[d[p + "img_idx"][t]]), t
            assert np.array_equal(goal[0].cpu().numpy(), frames[d[p + "goal_idx"][t]]), t
    finally:
        assert lib.vn_destroy(ctx) == 0
