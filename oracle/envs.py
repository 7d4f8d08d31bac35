"""Env restatements (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

CachedEnvOracle        THORDiscreteCachedEnv (environments/gym_ai2thor/envs/cached.py:10-99)
python_random_sampler  its reset sampler _get_random_start_goal_tuple (cached.py:38-45):
                       goal from the seeded instance, start from the module-global
                       ``random`` (modelled by a second Random instance)
VectorEnvOracle        the engine's batched contract: cached.py step semantics, gym
                       TimeLimit (environments/gym_ai2thor/__init__.py:45-49), baselines
                       auto-reset, Philox resets (DESIGN.md "RNG streams"), tasks
                       (gym_thor_cached.py:45-50) and replay schedules
SimpleGraphEnvOracle   graph/env.py:73-143 (maze, config C1) + MazeGraph.render
                       (graph/maze_graph.py:20-24)
sample_initial_position graph/util.py:88-117 (np.random global stream)
"""
import random

import numpy as np

from . import philox
from .graph import DIRS, enumerate_positions, is_valid_state, maze_render

FLAG_BAD_ACTION = 1
FLAG_RESET_EXHAUSTED = 2
FLAG_BAD_SCHEDULE = 4
START_ATTEMPTS = 1024


class CachedEnvOracle:
    """Frame *indices* stand in for frames: obs = (image_state, goal_state); the
    reference returns observations[idx] (resized; identity at equal size)."""

    reward_configuration = (1.0, 0.0, 0.0)  # cached.py:70-72

    def __init__(self, graph, spd, sampler):
        self.graph = np.asarray(graph)
        self.spd = np.asarray(spd)
        self.sampler = sampler
        self.reset()  # cached.py:36

    def reset(self):
        self.state, self.goal = self.sampler()
        self.last_state = (self.state, self.goal)
        return self.last_state

    def step(self, action):
        collided = False
        nxt = int(self.graph[self.state][action])
        if nxt != -1:
            self.state = nxt
        else:
            collided = True
        terminal = self.goal == self.state
        reward = -self.reward_configuration[1]
        if terminal:
            reward = self.reward_configuration[0]
        if collided:
            reward = self.reward_configuration[2]
        state = (self.state, self.goal) if not terminal else self.last_state
        self.last_state = state
        return state, reward, terminal, {}


def python_random_sampler(n, spd, rand_seed, global_seed):
    own = random.Random(rand_seed)
    glob = random.Random(global_seed)

    def sample():
        goal = own.randrange(n)
        while True:
            s = glob.randrange(n)
            if spd[s][goal] > 0:
                return s, goal

    return sample


class VectorEnvOracle:
    """scenes: list of dict(graph [N,4], spd [N,N], rewards=(goal, step, collision),
    terminal_obs=0|1). Rows are global arena rows (scene row base + state)."""

    def __init__(self, scenes, n_envs, seed, max_steps=900, autoreset=True, env_scene=None,
                 tasks=None):
        self.scenes = scenes
        self.n_envs = n_envs
        self.k0, self.k1 = philox.seed_key(seed)
        self.max_steps = max_steps
        self.autoreset = autoreset
        self.sizes = np.array([len(s["graph"]) for s in scenes], dtype=np.int64)
        self.row_base = np.concatenate([[0], np.cumsum(self.sizes)[:-1]]).astype(np.int64)
        self.graph = np.concatenate([np.asarray(s["graph"], dtype=np.int64) for s in scenes])
        self.rewards = np.array([s["rewards"] for s in scenes], dtype=np.float32)
        self.terminal_obs = np.array([s.get("terminal_obs", 0) for s in scenes], dtype=bool)
        self.env_scene = (np.arange(n_envs) % len(scenes)) if env_scene is None else np.asarray(env_scene)
        self.tasks = None if not tasks else np.asarray(tasks, dtype=np.int64)
        self.schedule = None
        self.cur_mode, self.cur_c, self.cur_offset = 0, 0.0, 0.0
        z = lambda: np.zeros(n_envs, dtype=np.int64)  # noqa: E731
        self.scene, self.state, self.goal, self.obs_state = z(), z(), z(), z()
        self.elapsed, self.episode, self.sched_pos = z(), z(), z()
        self.ep_ret = np.zeros(n_envs, dtype=np.float32)
        self.flags = 0
        self.reset()

    def set_curriculum(self, complexity, mode, offset):
        """The engine's curriculum draw (restated from DESIGN.md "Curriculum"): per goal,
        states sorted stably by spd; near = 0 < spd <= floor(opt), far = spd > opt."""
        n = len(self.scenes)
        self.cur_c = float(complexity)
        self.cur_modes = [int(m) for m in (mode if np.ndim(mode) else [mode] * n)]
        self.cur_offsets = [float(o) for o in (offset if np.ndim(offset) else [offset] * n)]
        self.cur_mode = int(any(self.cur_modes))

    def _curriculum_start(self, e, k, sc, g):
        spd = np.asarray(self.scenes[sc]["spd"])
        n = spd.shape[0]
        maxd = int(spd.max())
        col = np.clip(spd[:, g], -1, maxd)
        order = np.argsort(col, kind="stable")
        if not self.cur_modes[sc]:
            return None
        opt = self.cur_c * (maxd + self.cur_offsets[sc]) + 1.0  # Python floats, as the reference
        oi = min(max(int(np.floor(opt)), 0), maxd)
        lo = int((col <= 0).sum())
        hi = int((col <= oi).sum())
        rx, ry, _, _ = philox.philox4x32_10(e, k, 0, philox.STREAM_START, self.k0, self.k1)
        use_far = (self.cur_modes[sc] == 2 and int(ry) >= 3865470566 and hi < n) or hi <= lo
        b0, b1 = (hi, n) if use_far else (lo, hi)
        if b1 <= b0:
            return None
        return int(order[b0 + int(philox.uniform_below(rx, b1 - b0))])

    def set_schedule(self, schedule):
        """schedule [n_envs, L, 2] of (start, goal)."""
        self.schedule = None if schedule is None else np.asarray(schedule, dtype=np.int64)
        self.sched_pos[:] = 0

    def _reset_env(self, e):
        k = int(self.episode[e])
        sp = int(self.sched_pos[e])
        if self.schedule is not None and sp < self.schedule.shape[1]:
            sc = int(self.env_scene[e])
            n = int(self.sizes[sc])
            s, g = (int(v) for v in self.schedule[e, sp])
            if not (0 <= s < n and 0 <= g < n):
                self.flags |= FLAG_BAD_SCHEDULE
                s, g = min(max(s, 0), n - 1), min(max(g, 0), n - 1)
            self.sched_pos[e] = sp + 1
        else:
            sc, g = self._draw_goal(e, k)
            s = self._curriculum_start(e, k, sc, g) if self.cur_mode > 0 else None
            if s is None:
                s = self._rejection_start(e, k, sc, g)
        self.scene[e], self.state[e], self.goal[e] = sc, s, g
        self.obs_state[e] = s
        self.elapsed[e] = 0
        self.ep_ret[e] = 0.0
        self.episode[e] = k + 1

    def _draw_goal(self, e, k):
        rx, ry, _, _ = philox.philox4x32_10(e, k, 0, philox.STREAM_GOAL, self.k0, self.k1)
        if self.tasks is not None:
            t = int(philox.uniform_below(rx, len(self.tasks)))
            sc, g = int(self.tasks[t, 0]), int(self.tasks[t, 1])
            if g < 0:
                g = int(philox.uniform_below(ry, self.sizes[sc]))
        else:
            sc = int(self.env_scene[e])
            g = int(philox.uniform_below(rx, self.sizes[sc]))
        return sc, g

    def _rejection_start(self, e, k, sc, g):
        """cached.py:41-44 over Philox attempts: first candidate with spd[s][g] > 0."""
        n = int(self.sizes[sc])
        att = np.arange(START_ATTEMPTS)
        r = philox.philox4x32_10(e, k, att, philox.STREAM_START, self.k0, self.k1)[0]
        cand = philox.uniform_below(r, n)
        ok = np.asarray(self.scenes[sc]["spd"])[cand, g] > 0
        if ok.any():
            return int(cand[int(np.argmax(ok))])
        self.flags |= FLAG_RESET_EXHAUSTED
        return int(cand[0])

    def reset(self, mask=None):
        for e in range(self.n_envs):
            if mask is None or mask[e]:
                self._reset_env(e)

    def observe(self):
        return dict(img_row=self.row_base[self.scene] + self.obs_state,
                    goal_row=self.row_base[self.scene] + self.goal, state=self.state.copy())

    def step(self, actions):
        a = np.asarray(actions, dtype=np.int64)
        sc = self.scene
        bad = (a < 0) | (a > 3)
        if bad.any():
            self.flags |= FLAG_BAD_ACTION
        nxt = np.full(self.n_envs, -1, dtype=np.int64)
        ok = ~bad
        nxt[ok] = self.graph[self.row_base[sc[ok]] + self.state[ok], a[ok]]
        collided = nxt == -1
        s = np.where(collided, self.state, nxt)
        terminal = s == self.goal
        rw = self.rewards[sc]
        reward = rw[:, 1].copy()
        reward[terminal] = rw[terminal, 0]
        reward[collided] = rw[collided, 2]
        emit_current = (~terminal) | self.terminal_obs[sc]
        self.obs_state = np.where(emit_current, s, self.obs_state)
        self.state = s
        self.elapsed = self.elapsed + 1
        limit = (self.elapsed >= self.max_steps) if self.max_steps > 0 else np.zeros(self.n_envs, bool)
        done = terminal | limit
        ret = (self.ep_ret + reward).astype(np.float32)
        info = dict(ep_return=ret.copy(), ep_length=self.elapsed.copy(),
                    terminal_state=self.obs_state.copy(), truncated=limit & ~terminal)
        self.ep_ret = ret
        if self.autoreset:
            for e in np.nonzero(done)[0]:
                self._reset_env(int(e))
        out = self.observe()
        out.update(reward=reward.astype(np.float32), done=done, **info)
        return out


class SimpleGraphEnvOracle:
    """graph/env.py:73-143 with MazeGraph rendering; start supplied by the caller."""

    def __init__(self, maze, goal, rewards=(1.0, 0.0, 0.0)):
        self.maze = np.asarray(maze)
        self.goal = tuple(goal)
        self.rewards = rewards
        self.state = None

    def reset(self, start):
        self.state = tuple(start)
        return self.observe(self.state)

    def observe(self, state):
        # GridWorldScene.dtype is uint8 (graph/core.py:25-27) -> divide by 255 (graph/env.py:110-115)
        return maze_render(self.maze, state, self.goal).astype(np.float32) / 255.0

    def step(self, action):
        dx, dy = DIRS[action]
        nstate = (self.state[0] + dx, self.state[1] + dy)
        if not is_valid_state(self.maze, nstate):
            return self.observe(self.state), self.rewards[2], False, dict(state=self.state)
        self.state = nstate
        if self.state[:2] == self.goal:
            return self.observe(self.state), self.rewards[0], True, dict(state=self.state, win=True)
        return self.observe(self.state), self.rewards[1], False, dict(state=self.state)


def sample_initial_position(maze, distances, goal, optimal_distance=None, rng=np.random):
    """graph/util.py:88-117 over distances[x,y,gx,gy] (np.random global stream)."""
    potentials, dists = [], []
    for position in enumerate_positions(maze):
        d = distances[position + tuple(goal)]
        if d > 0:
            potentials.append(position)
            dists.append(d)
    if optimal_distance is None:
        x = None
        while x is None or potentials[x] == tuple(goal):
            x = rng.choice(np.arange(len(potentials)))
    else:
        dists = np.array(dists)
        positive = dists <= optimal_distance
        negative = dists > optimal_distance
        sum_negative = np.sum(negative)
        if sum_negative == 0:
            weights = positive / np.sum(positive)
        else:
            positive = 0.9 * positive / np.sum(positive)
            negative = 0.1 * negative / sum_negative
            weights = positive + negative
        x = None
        while x is None or potentials[x] == tuple(goal):
            x = rng.choice(np.arange(len(potentials)), p=weights)
    return potentials[x]


def compute_rotation_steps(optimal_actions, goal, state):
    """graph/util.py:82-86."""
    optimal_action = optimal_actions[tuple(state[:2]) + tuple(goal[:2])]
    rot_steps = np.array(list(map(lambda x: (state[2] - (goal[2] + x)) % 4, np.where(optimal_action))))
    rot_steps[rot_steps == 3] = 1
    return np.min(rot_steps)


def sample_initial_state(maze, distances, optimal_actions, goal, optimal_distance=None, rng=np.random):
    """graph/util.py:119-143 (np.random global stream)."""
    potentials, dists = [], []
    for position in enumerate_positions(maze):
        d = distances[position + tuple(goal[:2])]
        if d > 0:
            for i in range(4):
                state = position + (i,)
                potentials.append(state)
                dists.append(d + compute_rotation_steps(optimal_actions, goal, state))
    if optimal_distance is None:
        x = rng.choice(np.arange(len(potentials)))
    else:
        dists = np.array(dists)
        positive = dists <= optimal_distance
        weights = positive / np.sum(positive)
        x = rng.choice(np.arange(len(potentials)), p=weights)
    return potentials[x]


class MultiSceneResetOracle:
    """THORCachedEnv.reset / _sample_start (environments/gym_thor_cached.py:37-50):
    (scene, goal) = rnd.choice(tasks); start = rnd.randrange(N) until spd[start][goal] > 0."""

    def __init__(self, tasks, scenes, rnd):
        self.tasks = tasks
        self.scenes = scenes  # scene key -> dict(spd=..)
        self.rnd = rnd

    def reset(self):
        scene, goal = self.rnd.choice(self.tasks)
        spd = self.scenes[scene]["spd"]
        n = len(spd)
        while True:
            s = self.rnd.randrange(n)
            if spd[s][goal] > 0:
                return scene, goal, s
