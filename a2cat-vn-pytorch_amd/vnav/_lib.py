"""ctypes binding of libvnav.so (the C ABI declared in include/vnav.h).

torch is imported first on purpose: libvnav.so links libamdhip64.so.7 by soname, and
torch's bundled runtime must be the one already mapped so that both share one HIP
runtime (one set of device pointers and streams). There is no CPU fallback: if the
library is missing every entry point raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libvnav.so")

c_int = ctypes.c_int
c_int32 = ctypes.c_int32
c_int64 = ctypes.c_int64
c_uint32 = ctypes.c_uint32
c_uint64 = ctypes.c_uint64
c_float = ctypes.c_float
c_double = ctypes.c_double
c_void_p = ctypes.c_void_p
c_size_t = ctypes.c_size_t
P = ctypes.POINTER


class SceneDesc(ctypes.Structure):
    _fields_ = [
        ("n_states", c_int32),
        ("height", c_int32),
        ("width", c_int32),
        ("channels", c_int32),
        ("graph", P(c_int64)),
        ("spd", P(c_int64)),
        ("observations", P(ctypes.c_uint8)),
        ("reward_goal", c_float),
        ("reward_step", c_float),
        ("reward_collision", c_float),
        ("terminal_obs", c_int32),
        ("synth_id", c_uint32),
        ("companion", P(ctypes.c_uint8)),
    ]


class A2CStep(ctypes.Structure):
    """vn_a2c_step (include/vnav.h)."""
    _fields_ = [
        ("policy_out", c_void_p),
        ("num_actions", c_int),
        ("seed", c_uint64),
        ("counter_base_dev", c_void_p),
        ("counter", c_uint64),
        ("actions", c_void_p),
        ("prev_action", c_void_p),
        ("prev_reward", c_void_p),
        ("prev_mask", c_void_p),
        ("lra_next", c_void_p),
        ("mask_next", c_void_p),
        ("episode_stats_env", c_void_p),
        ("head_weight", c_void_p),
        ("head_bias", c_void_p),
        ("head_input", c_void_p),
        ("head_out", c_void_p),
    ]


class GoalRuns(ctypes.Structure):
    """vn_goal_runs (include/vnav.h)."""
    _fields_ = [
        ("goal_list", c_void_p),
        ("goal_count", c_void_p),
        ("goal_delta", c_void_p),
        ("run_length", c_void_p),
        ("num_envs", c_int),
    ]


class ReplaySeg(ctypes.Structure):
    """vn_replay_seg (include/vnav.h)."""
    _fields_ = [
        ("src", c_void_p),
        ("src_ld", c_int64),
        ("ring", c_void_p),
        ("cur", c_void_p),
        ("slot_elems", c_int64),
        ("rows", c_int),
        ("cols", c_int),
        ("elem_bytes", c_int),
        ("pad_", c_int),
    ]


# name -> (restype, argtypes). Every symbol here is declared in include/vnav.h.
SIGNATURES = {
    "vn_version": (ctypes.c_char_p, []),
    "vn_last_error": (c_int, [ctypes.c_char_p, c_size_t]),
    "vn_create": (c_int, [P(SceneDesc), c_int, c_int, c_uint64, c_int, P(c_void_p)]),
    "vn_destroy": (c_int, [c_void_p]),
    "vn_reset": (c_int, [c_void_p, c_void_p, c_void_p]),
    "vn_observe": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_set_info_buffers": (c_int, [c_void_p] + [c_void_p] * 6),
    "vn_set_schedule": (c_int, [c_void_p, c_void_p, c_int]),
    "vn_set_tasks": (c_int, [c_void_p, P(c_int32), c_int]),
    "vn_set_env_scenes": (c_int, [c_void_p, P(c_int32)]),
    "vn_set_max_episode_steps": (c_int, [c_void_p, c_int]),
    "vn_set_curriculum": (c_int, [c_void_p, c_double, c_int, c_double]),
    "vn_set_curriculum_scenes": (c_int, [c_void_p, c_double, c_void_p, c_void_p]),
    "vn_set_autoreset": (c_int, [c_void_p, c_int]),
    "vn_random_actions": (c_int, [c_void_p, c_void_p, c_uint64, c_void_p]),
    "vn_get_state": (c_int, [c_void_p, c_void_p, c_void_p]),
    "vn_set_state": (c_int, [c_void_p, c_void_p, c_void_p]),
    "vn_get_episode_returns": (c_int, [c_void_p, c_void_p, c_void_p]),
    "vn_set_episode_returns": (c_int, [c_void_p, c_void_p, c_void_p]),
    "vn_frame_arena": (c_int, [c_void_p, P(c_void_p), P(c_int64), P(c_int64)]),
    "vn_scene_row_base": (c_int, [c_void_p, c_int, P(c_int64)]),
    "vn_error_flags_sync": (c_int, [c_void_p, P(c_uint32), c_int]),
    "vn_num_envs": (c_int, [c_void_p]),
    "vn_gather_rows": (c_int, [c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p]),
    "vn_step_a2c": (c_int, [c_void_p, P(A2CStep), c_void_p, c_void_p, c_void_p, c_void_p]),
}

SIGNATURES.update({
    "vn_policy_create": (c_int, [c_int, c_int, c_int, P(c_void_p)]),
    "vn_policy_destroy": (c_int, [c_void_p]),
    "vn_policy_info": (c_int, [c_void_p, P(c_int64), P(c_int64),
                                      P(c_int64)]),
    "vn_policy_workspace_floats": (c_int, [c_void_p, c_int64, P(c_int64)]),
    "vn_policy_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int,
                                         c_void_p, c_int64, c_int64, c_void_p,
                                         c_void_p]),
    "vn_policy_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int,
                                          c_void_p, c_int64, c_void_p, c_void_p,
                                          c_void_p, c_void_p]),
    "vn_policy_create_ex": (c_int, [c_int, c_int, c_int, c_int, P(c_void_p)]),
    "vn_policy_lstm_info": (c_int, [c_void_p, P(c_int64)]),
    "vn_lstm_workspace_floats": (c_int, [c_void_p, c_int, c_int, P(c_int64)]),
    "vn_lstm_forward_step": (c_int, [c_void_p, c_void_p, c_int] + [c_void_p] * 10 + [c_void_p]),
    "vn_policy_heads": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "vn_lstm_backward": (c_int, [c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 11 + [c_void_p]),
    "vn_policy_backward_trunk": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p,
                                         c_void_p, c_void_p, c_void_p]),
    "vn_policy_aux_info": (c_int, [c_void_p, P(c_int64)]),
    "vn_aux_workspace_floats": (c_int, [c_void_p, P(c_int64)]),
    "vn_aux_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "vn_aux_target_table": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64, c_void_p, c_void_p]),
    "vn_aux_loss_grad": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_float, c_void_p, c_void_p, c_void_p]),
    "vn_aux_forward_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                                         c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_aux_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "vn_policy_unreal_info": (c_int, [c_void_p, P(c_int64)]),
    "vn_pc_workspace_floats": (c_int, [c_void_p, P(c_int64)]),
    "vn_pc_forward": (c_int, [c_void_p] * 3 + [c_int] + [c_void_p] * 6),
    "vn_pc_backward": (c_int, [c_void_p] * 3 + [c_int] + [c_void_p] * 6 + [c_int, c_void_p, c_void_p]),
    "vn_rp_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "vn_rp_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_void_p]),
    "vn_lstm_backward_ex": (c_int, [c_void_p, c_void_p, c_int, c_int] + [c_void_p] * 9 + [c_int] + [c_void_p] * 4),
    "vn_unreal_pc_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int, c_void_p,
                                       c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, c_void_p, c_void_p]),
    "vn_unreal_pc_loss_grad_ex": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_int,
                                          c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_float, c_void_p,
                                          c_void_p]),
    "vn_unreal_rp_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_void_p,
                                       c_void_p, c_void_p]),
    "vn_unreal_rp_scatter": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "vn_unreal_gather": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    "vn_unreal_vr_grad": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p,
                                  c_void_p]),
    "vn_policy_backward_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_policy_sample": (c_int, [c_void_p, c_int, c_int, c_uint64, c_uint64,
                                        c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "vn_policy_greedy": (c_int, [c_void_p, c_int, c_int, c_void_p,
                                        c_void_p]),
    "vn_a2c_returns": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int,
                                      c_int, c_float, c_void_p, c_void_p]),
    "vn_a2c_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int,
                                        c_float, c_float, c_void_p, c_void_p,
                                        c_void_p]),
    "vn_a2c_step_post": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_grad_norm": (c_int, [c_void_p, c_int64, c_float, c_float, c_void_p,
                                    c_void_p, c_void_p]),
    "vn_grad_norm_join": (c_int, [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_void_p, c_int64, c_int64,
                                  c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "vn_replay_push_draw": (c_int, [P(ReplaySeg), c_int, c_void_p, c_int, c_uint64, c_void_p]),
    "vn_rmsprop_step": (c_int, [c_void_p, c_void_p, c_void_p, c_int64,
                                       c_float, c_void_p, c_float, c_float,
                                       c_float, c_void_p]),
    "vn_a2c_schedule": (c_int, [c_void_p, c_void_p, c_double, c_double, c_int64, c_int, c_void_p]),
    "vn_a2c_metrics": (c_int, [c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_a2c_metrics_ex": (c_int, [c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_void_p, c_void_p]),
    "vn_a2c_rollout_begin":(c_int, [c_void_p, c_void_p, c_double, c_double, c_int64, c_int, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                     c_void_p, c_void_p]),
    "vn_policy_sample_dev": (c_int, [c_void_p, c_int, c_int, c_uint64, c_void_p, c_uint64, c_void_p, c_void_p,
                                     c_void_p, c_void_p, c_void_p]),
    "vn_trace_marker": (c_int, [c_int, c_void_p]),
    "vn_policy_goal_runs_supported": (c_int, [c_void_p, c_int, P(c_int)]),
    "vn_policy_forward_goals": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_int64, c_void_p,
                                        P(GoalRuns), c_void_p]),
    "vn_policy_backward_goals": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_void_p, P(GoalRuns), c_void_p]),
    "vn_goal_runs_step": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_goal_runs_rollout": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "vn_a2c_episode_stats": (c_int, [c_void_p, c_int, c_void_p, c_void_p]),
    "vn_rmsprop_step_dev": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p, c_void_p, c_float,
                                    c_float, c_void_p]),
})

_lib = None


class VnavError(RuntimeError):
    pass


def load():
    """Load libvnav.so (raises if it has not been built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VnavError("libvnav.so not found at %s — build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                        "(hipcc --offload-arch=gfx950)" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def last_error():
    buf = ctypes.create_string_buffer(1024)
    load().vn_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise VnavError("%s failed (%d): %s" % (what, rc, last_error()))
    return rc


def ptr(t):
    """Raw device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return c_void_p(t.data_ptr())


def stream_ptr(device):
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)
