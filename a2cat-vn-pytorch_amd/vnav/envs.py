"""VectorEnv — the batched cached-scene environment on one GPU.

Drop-in for the deep_rl ``SubprocVecEnv`` of THORDiscreteCachedEnv / THORCachedEnv
processes (experiments/thor_cached_auxiliary.py:58-71): ``reset()``, ``step(actions)``
with baselines-style auto-reset, ``call_unwrapped('set_complexity', x)`` and
``set_hardness``. Every env lives on the device; a step is one HIP launch
(``vn_step`` in libvnav.so) — there is no per-env process, pipe or host copy.

Observations are the tuple ``(image, goal)`` of uint8 ``[E,H,W,C]`` device tensors (the
raw cached frames, cached.py:59-60 / gym_thor_cached.py:52-53). The reference
wrapper chain TransposeImage + ScaledFloatFrame is ``to_float_chw`` below; the policy
kernels consume the uint8 frames directly and fuse that conversion.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from .scenes import Scene

ST_FIELDS = ("scene", "state", "goal", "obs_state", "elapsed", "episode", "sched_pos")


def to_float_chw(frames):
    """TransposeImage + ScaledFloatFrame: uint8 [...,H,W,C] -> float32 [...,C,H,W] / 255."""
    return frames.permute(*range(frames.dim() - 3), -1, -3, -2).to(torch.float32) / 255.0


class VectorEnv:
    num_actions = 4  # THORDiscreteCachedEnv.get_action_size (cached.py:66-68)

    def __init__(self, scenes, num_envs, seed=0, device=None, max_episode_steps=900, tasks=None,
                 env_scenes=None, autoreset=True, aux_observations=False):
        if isinstance(scenes, Scene):
            scenes = [scenes]
        if not scenes:
            raise ValueError("VectorEnv needs at least one scene")
        if not torch.cuda.is_available():
            raise _lib.VnavError("VectorEnv requires a ROCm GPU (no CPU fallback)")
        self.lib = _lib.load()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.scenes = list(scenes)
        self.num_envs = int(num_envs)
        self.seed = int(seed)
        self.frame_shape = tuple(self.scenes[0].frame_shape)
        descs = (_lib.SceneDesc * len(self.scenes))()
        self._keep = []
        for i, s in enumerate(self.scenes):
            d = descs[i]
            d.n_states = s.n_states
            d.height, d.width, d.channels = s.frame_shape
            d.graph = s.graph.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            d.spd = s.spd.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            if s.observations is not None:
                d.observations = s.observations.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            d.reward_goal, d.reward_step, d.reward_collision = s.rewards
            d.terminal_obs = s.terminal_obs
            if s.companion is not None:
                d.companion = s.companion.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
            d.synth_id = s.synth_id
            self._keep.append(s)
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _lib.check(self.lib.vn_create(descs, len(self.scenes), self.num_envs,
                                          ctypes.c_uint64(self.seed & (2**64 - 1)),
                                          self.device.index, ctypes.byref(handle)), "vn_create")
        self._ctx = handle
        # bumped by every call that replaces the kernels' per-ctx configuration (tables,
        # schedules, limits): a captured hipGraph holds the old launch arguments and must be
        # recaptured (A2CTrainer checks it before each replay)
        self.config_generation = 0
        self._out_cache = None
        E = self.num_envs
        kw = dict(device=self.device)
        self._info = dict(
            ep_return=torch.zeros(E, dtype=torch.float32, **kw),
            ep_length=torch.zeros(E, dtype=torch.int32, **kw),
            terminal_state=torch.zeros(E, dtype=torch.int32, **kw),
            truncated=torch.zeros(E, dtype=torch.uint8, **kw),
            img_row=torch.zeros(E, dtype=torch.int32, **kw),
            goal_row=torch.zeros(E, dtype=torch.int32, **kw),
        )
        self.set_row_outputs(None, None)
        self.set_max_episode_steps(max_episode_steps)
        if not autoreset:
            _lib.check(self.lib.vn_set_autoreset(self._ctx, 0), "vn_set_autoreset")
        if env_scenes is not None:
            self.set_env_scenes(env_scenes)
        if tasks is None and all(s.goals for s in self.scenes):
            # the scenes' own fixed goal lists (OrientedGraphEnv goals, MazeGraph goal)
            tasks = [(i, g) for i, s in enumerate(self.scenes) for g in s.goals]
        if tasks:
            self.set_tasks(tasks)
        self.complexity = None
        self._schedule = None
        self.aux_arena = None
        if all(s.depth is not None and s.segmentation is not None for s in self.scenes):
            self.aux_arena = self._build_aux_arena()
        self.aux_observations = bool(aux_observations)
        if self.aux_observations and self.aux_arena is None:
            raise ValueError("aux_observations needs depth + segmentation on every scene")

    def _build_aux_arena(self):
        """Depth [rows,H,W,1] and segmentation [rows,H,W,3] uint8 on the device, indexed by
        the frame arena's rows (so info img_row / goal_row address them too)."""
        _, _, rows, bases = self.frame_arena()
        H, W = self.frame_shape[:2]
        depth = torch.zeros((rows, H, W, 1), dtype=torch.uint8, device=self.device)
        seg = torch.zeros((rows, H, W, 3), dtype=torch.uint8, device=self.device)
        for s, b in zip(self.scenes, bases):
            depth[b:b + s.n_states].copy_(torch.from_numpy(s.depth))
            seg[b:b + s.n_states].copy_(torch.from_numpy(s.segmentation))
        return depth, seg

    def _gather_aux(self):
        """(depth, segmentation, goal segmentation) of the current observation by row."""
        depth, seg = self.aux_arena
        E = self.num_envs
        out = []
        for src, rows in ((depth, self._info["img_row"]), (seg, self._info["img_row"]), (seg, self._info["goal_row"])):
            dst = torch.empty((E,) + tuple(src.shape[1:]), dtype=torch.uint8, device=self.device)
            _lib.check(self.lib.vn_gather_rows(_lib.ptr(src), int(src[0].numel()), _lib.ptr(rows), E, _lib.ptr(dst),
                                               self._stream()), "vn_gather_rows")
            out.append(dst)
        return tuple(out)

    # -- configuration -------------------------------------------------------
    def set_max_episode_steps(self, n):
        self.config_generation += 1
        _lib.check(self.lib.vn_set_max_episode_steps(self._ctx, int(n or 0)), "vn_set_max_episode_steps")

    def set_tasks(self, tasks):
        """tasks: [(scene_index, goal_state or -1)] sampled uniformly at each reset."""
        arr = np.ascontiguousarray(np.asarray(tasks, dtype=np.int32).reshape(-1, 2))
        self.config_generation += 1
        _lib.check(self.lib.vn_set_tasks(self._ctx, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(arr)),
                   "vn_set_tasks")

    def set_env_scenes(self, env_scenes):
        arr = np.ascontiguousarray(np.asarray(env_scenes, dtype=np.int32))
        if arr.shape != (self.num_envs,):
            raise ValueError("env_scenes must have one entry per env")
        self.config_generation += 1
        _lib.check(self.lib.vn_set_env_scenes(self._ctx, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))),
                   "vn_set_env_scenes")

    def set_schedule(self, schedule):
        """Exact-replay test mode: schedule [E, L, 2] int32 (start, goal) per reset."""
        self.config_generation += 1
        if schedule is None:
            _lib.check(self.lib.vn_set_schedule(self._ctx, None, 0), "vn_set_schedule")
            self._schedule = None
            return
        sched = torch.as_tensor(schedule, dtype=torch.int32).to(self.device).contiguous()
        if sched.dim() != 3 or sched.shape[0] != self.num_envs or sched.shape[2] != 2:
            raise ValueError("schedule must be [num_envs, L, 2]")
        torch.cuda.synchronize(self.device)
        _lib.check(self.lib.vn_set_schedule(self._ctx, _lib.ptr(sched), sched.shape[1]), "vn_set_schedule")
        self._schedule = sched

    def set_complexity(self, complexity=None, mode=None, offset=None):
        """Curriculum hook (graph/env.py:98-99, environments/gym_graph/graph.py:40-52,
        experiments/thor_cached_auxiliary.py:68-70): subsequent resets draw starts near the
        goal on the device (vn_set_curriculum); None switches back to uniform starts.
        mode/offset default to each scene's own semantics (Scene.curriculum)."""
        self.complexity = complexity
        self.config_generation += 1
        if complexity is None:
            _lib.check(self.lib.vn_set_curriculum(self._ctx, 0.0, 0, 0.0), "vn_set_curriculum")
            return
        modes = np.array([s.curriculum[0] if mode is None else int(mode) for s in self.scenes], dtype=np.int32)
        offs = np.array([s.curriculum[1] if offset is None else float(offset) for s in self.scenes], dtype=np.float64)
        _lib.check(self.lib.vn_set_curriculum_scenes(self._ctx, float(complexity), modes.ctypes.data_as(ctypes.c_void_p),
                                                     offs.ctypes.data_as(ctypes.c_void_p)), "vn_set_curriculum_scenes")

    set_hardness = set_complexity

    def call_unwrapped(self, name, *args, **kwargs):
        return getattr(self, name)(*args, **kwargs)

    # -- gym VecEnv API -------------------------------------------------------
    def _stream(self):
        return _lib.stream_ptr(self.device)

    def set_row_outputs(self, img_rows, goal_rows):
        """Where the next steps write the arena rows of the frames they emit: int32 [E] device
        tensors (e.g. the trainer's per-step rollout slots, so no copy follows each step), or
        None for this env's own info["img_row"] / info["goal_row"]."""
        i = self._info
        if img_rows is None:
            img_rows, goal_rows = i["img_row"], i["goal_row"]
        self._check_out("img_rows", img_rows, torch.int32, self.num_envs)
        self._check_out("goal_rows", goal_rows, torch.int32, self.num_envs)
        _lib.check(self.lib.vn_set_info_buffers(self._ctx, _lib.ptr(i["ep_return"]), _lib.ptr(i["ep_length"]),
                                                _lib.ptr(i["terminal_state"]), _lib.ptr(i["truncated"]),
                                                _lib.ptr(img_rows), _lib.ptr(goal_rows)), "vn_set_info_buffers")

    def _check_out(self, name, t, dtype, numel):
        """Caller-owned output buffers are written by the kernel through raw pointers: refuse
        anything the launch would write past or misread (wrong device, dtype, size, layout)."""
        if t is None:
            return
        if not isinstance(t, torch.Tensor) or t.device != self.device:
            raise ValueError("%s must be a tensor on %s" % (name, self.device))
        if t.dtype != dtype or not t.is_contiguous() or t.numel() != numel:
            raise ValueError("%s must be a contiguous %s tensor of %d elements (got %s, %d, contiguous=%s)"
                             % (name, dtype, numel, t.dtype, t.numel(), t.is_contiguous()))

    def _check_frames_out(self, img, goal):
        F = int(np.prod(self.frame_shape))
        self._check_out("image", img, torch.uint8, self.num_envs * F)
        self._check_out("goal", goal, torch.uint8, self.num_envs * F)

    def _frames(self):
        shape = (self.num_envs,) + self.frame_shape
        return (torch.empty(shape, dtype=torch.uint8, device=self.device),
                torch.empty(shape, dtype=torch.uint8, device=self.device))

    def reset(self, mask=None):
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.int32).contiguous()
            if m.shape != (self.num_envs,):
                raise ValueError("reset mask must have shape [num_envs]")
        _lib.check(self.lib.vn_reset(self._ctx, _lib.ptr(m), self._stream()), "vn_reset")
        return self.observe()

    def observe(self, out=None, gather=True):
        """Current (image, goal) frames; gather=False only refreshes info img_row/goal_row."""
        if not gather:
            _lib.check(self.lib.vn_observe(self._ctx, None, None, None, self._stream()), "vn_observe")
            return None, None
        img, goal = out if out is not None else self._frames()
        self._check_frames_out(img, goal)
        _lib.check(self.lib.vn_observe(self._ctx, _lib.ptr(img), _lib.ptr(goal), None, self._stream()), "vn_observe")
        if self.aux_observations:
            return (img, goal) + self._gather_aux()
        return img, goal

    def step(self, actions, out=None, gather=True):
        """actions: int32 [E] device tensor (other integer dtypes are converted).
        Returns ((image, goal), reward f32 [E], done bool [E], info dict of [E] tensors).
        Without ``out`` every returned tensor is fresh, info included (a caller may keep step
        t's results while stepping on). ``out`` = dict of preallocated outputs (image, goal,
        reward, done, state) to write in place: the fast path, where nothing is allocated or
        copied per step and info's tensors (ep_return, ep_length, terminal_state, truncated,
        img_row, goal_row) are the env's own buffers, overwritten by the next step like the
        ``out`` buffers. ``gather=False`` skips the frame copy
        (index-only step: info img_row / goal_row address the frames in the scene cache)."""
        if type(actions) is torch.Tensor and actions.dtype == torch.int32 and actions.device == self.device \
                and actions.shape == (self.num_envs,) and actions.is_contiguous():
            a = actions
        else:
            a = torch.as_tensor(actions, device=self.device)
            if a.dtype != torch.int32:
                a = a.to(torch.int32)
            a = a.contiguous()
            if a.shape != (self.num_envs,):
                raise ValueError("actions must have shape [num_envs]")
        if out is not None and gather:
            # the same caller-owned buffers as the previous call: validated then, pointers cached.
            # The key also holds each buffer's current data_ptr and size, so a tensor that was
            # resize_()d or set_() to other storage since is validated again
            bufs = (out["image"], out["goal"], out.get("reward"), out.get("done"), out.get("state"))
            c = self._out_cache
            if c is not None and all(x is y for x, y in zip(bufs, c[0])) and \
                    c[2] == tuple((t.data_ptr(), t.numel()) if t is not None else None for t in bufs):
                P = c[1]
                _lib.check(self.lib.vn_step(self._ctx, _lib.ptr(a), P[0], P[1], P[2], P[3], P[4], self._stream()),
                           "vn_step")
                info = dict(self._info)
                info["state"] = bufs[4]
                if self.aux_observations:
                    return (bufs[0], bufs[1]) + self._gather_aux(), bufs[2], bufs[3], info
                return (bufs[0], bufs[1]), bufs[2], bufs[3], info
        if out is None:
            img, goal = self._frames() if gather else (None, None)
            reward = torch.empty(self.num_envs, dtype=torch.float32, device=self.device)
            done = torch.empty(self.num_envs, dtype=torch.bool, device=self.device)
            state = torch.empty(self.num_envs, dtype=torch.int32, device=self.device)
        else:
            img, goal = (out["image"], out["goal"]) if gather else (None, None)
            reward, done, state = out.get("reward"), out.get("done"), out.get("state")
            self._check_frames_out(img, goal)
            self._check_out("reward", reward, torch.float32, self.num_envs)
            self._check_out("done", done, torch.bool, self.num_envs)
            self._check_out("state", state, torch.int32, self.num_envs)
            if gather:
                bufs = (img, goal, reward, done, state)
                self._out_cache = (bufs, tuple(_lib.ptr(t) for t in bufs),
                                   tuple((t.data_ptr(), t.numel()) if t is not None else None for t in bufs))
        _lib.check(self.lib.vn_step(self._ctx, _lib.ptr(a), _lib.ptr(img), _lib.ptr(goal), _lib.ptr(reward),
                                    _lib.ptr(done), _lib.ptr(state), self._stream()), "vn_step")
        # fresh info tensors unless the caller chose the in-place path (out=...)
        info = {k: v.clone() for k, v in self._info.items()} if out is None else dict(self._info)
        info["state"] = state
        if self.aux_observations and gather:
            return (img, goal) + self._gather_aux(), reward, done, info
        return (img, goal), reward, done, info

    def step_a2c(self, a2c, reward, done, state):
        """The trainer's rollout step (vn_step_a2c): the actions are sampled in the step from
        the policy outputs named by ``a2c`` (a prepared _lib.A2CStep whose buffers the caller
        keeps alive), index-only, with the per-step bookkeeping fused. reward / done / state
        are the caller's [E] buffers (checked once by the caller)."""
        _lib.check(self.lib.vn_step_a2c(self._ctx, ctypes.byref(a2c), _lib.ptr(reward), _lib.ptr(done),
                                        _lib.ptr(state), self._stream()), "vn_step_a2c")

    def random_actions(self, step, out=None):
        out = torch.empty(self.num_envs, dtype=torch.int32, device=self.device) if out is None else out
        _lib.check(self.lib.vn_random_actions(self._ctx, _lib.ptr(out), ctypes.c_uint64(int(step)), self._stream()),
                   "vn_random_actions")
        return out

    # -- state / checkpoint ----------------------------------------------------
    def get_state(self):
        buf = torch.empty((len(ST_FIELDS), self.num_envs), dtype=torch.int32, device=self.device)
        _lib.check(self.lib.vn_get_state(self._ctx, _lib.ptr(buf), self._stream()), "vn_get_state")
        return buf

    def set_state(self, buf):
        """Restore get_state()'s [len(ST_FIELDS), num_envs] int32 table (checked before the
        device copy: a table of another env count would be read past or misaligned)."""
        buf = torch.as_tensor(buf)
        if tuple(buf.shape) != (len(ST_FIELDS), self.num_envs):
            raise ValueError("env state must be [%d, %d] (this env), got %s"
                             % (len(ST_FIELDS), self.num_envs, tuple(buf.shape)))
        buf = buf.to(device=self.device, dtype=torch.int32).contiguous()
        _lib.check(self.lib.vn_set_state(self._ctx, _lib.ptr(buf), self._stream()), "vn_set_state")

    def get_episode_returns(self):
        """Running return of every env's unfinished episode ([E] f32, device)."""
        buf = torch.empty(self.num_envs, dtype=torch.float32, device=self.device)
        _lib.check(self.lib.vn_get_episode_returns(self._ctx, _lib.ptr(buf), self._stream()),
                   "vn_get_episode_returns")
        return buf

    def set_episode_returns(self, buf):
        buf = torch.as_tensor(buf)
        if tuple(buf.shape) != (self.num_envs,):
            raise ValueError("episode returns must be [%d] (this env), got %s" % (self.num_envs, tuple(buf.shape)))
        buf = buf.to(device=self.device, dtype=torch.float32).contiguous()
        _lib.check(self.lib.vn_set_episode_returns(self._ctx, _lib.ptr(buf), self._stream()),
                   "vn_set_episode_returns")

    def frame_arena(self):
        """(arena uint8 tensor view [rows, H, W, C] over the scene cache, row bases per scene)."""
        p, fb, rows = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        _lib.check(self.lib.vn_frame_arena(self._ctx, ctypes.byref(p), ctypes.byref(fb), ctypes.byref(rows)),
                   "vn_frame_arena")
        bases = []
        for k in range(len(self.scenes)):
            b = ctypes.c_int64()
            _lib.check(self.lib.vn_scene_row_base(self._ctx, k, ctypes.byref(b)), "vn_scene_row_base")
            bases.append(b.value)
        return p.value, fb.value, rows.value, bases

    def error_flags(self, clear=True):
        f = ctypes.c_uint32()
        _lib.check(self.lib.vn_error_flags_sync(self._ctx, ctypes.byref(f), int(clear)), "vn_error_flags_sync")
        return f.value

    def close(self):
        if getattr(self, "_ctx", None):
            self.lib.vn_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# gym-style registry mirroring environments.make ids (environments/__init__.py:2,
# environments/gym_ai2thor/__init__.py:45-49, environments/gym_graph/__init__.py:18-27)
REGISTRY = {
    "CachedThor-v0": dict(max_episode_steps=900),
    "AuxiliaryGraph-v0": dict(max_episode_steps=900, aux_observations=True),
    "OrientedGraph-v0": dict(max_episode_steps=900),
}


def make(id, scenes, num_envs, **kwargs):
    if id not in REGISTRY:
        raise KeyError("unknown env id %r (known: %s)" % (id, sorted(REGISTRY)))
    opts = dict(REGISTRY[id])
    opts.update(kwargs)
    return VectorEnv(scenes, num_envs, **opts)


class CachedThorEnv:
    """One gym-style env over the same kernel: the single-env surface of
    THORDiscreteCachedEnv (environments/gym_ai2thor/envs/cached.py:10-99) under gym's
    TimeLimit, for callers that drive one env at a time (gym.make + a hand-written loop,
    test-time episodes). ``reset() -> (image, goal)``; ``step(a) -> (obs, reward, done,
    info)`` with no auto-reset: on a terminal step the previous observation is returned
    (cached.py:90-96) and the caller resets, as with the reference. Frames are float64 in
    [0, 1], HWC, as ``_preprocess_frame`` returns at equal size (cached.py:62-64; resize
    offline with tools/h5_to_npz.py --size). Every call synchronises with the device; the
    batched ``VectorEnv`` is the fast path."""

    def __init__(self, scene, seed=0, device=None, max_episode_steps=900, float_frames=True):
        self._env = VectorEnv([scene], 1, seed=seed, device=device, max_episode_steps=max_episode_steps,
                              autoreset=False)
        self.float_frames = bool(float_frames)
        self.action_size = VectorEnv.num_actions  # get_action_size (cached.py:66-68)
        self.max_episode_steps = max_episode_steps

    def _obs(self, img, goal):
        img, goal = img[0].cpu().numpy(), goal[0].cpu().numpy()
        if self.float_frames:
            return img.astype(np.float64) / 255.0, goal.astype(np.float64) / 255.0
        return img, goal

    def reset(self):
        return self._obs(*self._env.reset())

    def step(self, action):
        (img, goal), reward, done, info = self._env.step(torch.tensor([int(action)], dtype=torch.int32))
        info_out = {}
        if bool(info["truncated"][0].item()):
            info_out["TimeLimit.truncated"] = True  # gym's TimeLimit (environments/gym_ai2thor/__init__.py:48)
        return self._obs(img, goal), float(reward[0].item()), bool(done[0].item()), info_out

    @property
    def state(self):
        """(state, goal) indices of the env (cached.py: self.state, self.goal)."""
        st = self._env.get_state().cpu().numpy()
        return int(st[ST_FIELDS.index("state"), 0]), int(st[ST_FIELDS.index("goal"), 0])

    def set_schedule(self, starts_goals):
        """Exact replay: the (start, goal) pairs the following resets take, in order."""
        self._env.set_schedule(np.asarray(starts_goals, dtype=np.int32)[None])

    def set_complexity(self, complexity=None):
        self._env.set_complexity(complexity)

    def close(self):
        self._env.close()
