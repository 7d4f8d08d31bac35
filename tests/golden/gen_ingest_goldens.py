"""Golden vectors for scene ingestion from the REFERENCE code.

Run ONLY in the build container (the reference tree is not on the GPU box):
    /opt/conda/bin/python3.9 tests/golden/gen_ingest_goldens.py
(Anaconda 3.9 has h5py and scikit-image, which the reference's cached env needs.)

1. OrientedGraphEnv (environments/gym_graph/graph.py:9-93) on a ThorGridWorld
   (graph/thor_graph.py:5-18) pickled by the reference's own dump_graph (graph/util.py:40-65)
   and read back by its load_graph (:69-79): seeded resets (goal from ``random``, start from
   ``np.random`` via sample_initial_state) and seeded steps, recorded as (x, y, r) states,
   reward bits, done flags and the emitted frame's state id; then the start support of
   set_complexity(c) for several c (draws of the reference sampler).
2. THORDiscreteCachedEnv (environments/gym_ai2thor/envs/cached.py) with image_size 84x84 on
   a 100x100 h5 scene written by save_graph_as_h5: the skimage anti-aliased resize output
   the reference feeds its model (_preprocess_frame, cached.py:62-64) for a few states.
Frames are synthetic; every output is data (inputs + expected outputs) in ingest.npz.
"""
import importlib
import importlib.util
import os
import random
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "stubs"), REF, REPO]

np.int = int
np.float = float
np.bool = bool

import graph.util as gutil  # noqa: E402
from graph.thor_graph import ThorGridWorld  # noqa: E402

gutil.create_resnet = lambda: (lambda observation: np.zeros(2048, dtype=np.float32))


def import_oriented_env():
    """environments.gym_graph.graph without running environments/__init__.py (it imports
    every env family and requests): bare parent packages pointing at the reference dirs."""
    for name, rel in (("environments", "environments"), ("environments.gym_graph", "environments/gym_graph")):
        if name not in sys.modules:
            m = types.ModuleType(name)
            m.__path__ = [os.path.join(REF, rel)]
            sys.modules[name] = m
    return importlib.import_module("environments.gym_graph.graph")


def oriented_frames(maze, hw=(84, 84)):
    """[X, Y, 4, H, W, 3] uint8: channel 0 = state id (point*4 + r), 1 = x, 2 = y (plus a
    fixed ramp so frames are not constant). The observation is the tuple render() returns
    (graph/thor_graph.py:15-33): (rgb, third-person rgb)."""
    X, Y = maze.shape
    obs = np.zeros((X, Y, 4) + hw + (3,), dtype=np.uint8)
    ramp = (np.arange(hw[0])[:, None] + np.arange(hw[1])[None, :]) % 7
    for i, (x, y) in enumerate(gutil.enumerate_positions(maze)):
        for r in range(4):
            obs[x, y, r, :, :, 0] = i * 4 + r
            obs[x, y, r, :, :, 1] = 10 * x + ramp
            obs[x, y, r, :, :, 2] = 10 * y + r
    return obs


def oriented_goldens(tmp):
    rng = np.random.RandomState(21)
    maze = rng.rand(5, 6) > 0.25
    maze[0, 0] = maze[4, 5] = maze[2, 3] = True
    obs = oriented_frames(maze)
    tp = obs.copy()
    tp[..., 0] = 255 - tp[..., 0]  # third-person frames: channel 0 = 255 - state id
    small = np.zeros(maze.shape + (4, 2, 2, 1), dtype=np.uint8)
    g = ThorGridWorld(maze, obs, small, small, tp, small, small)
    goals = [(0, 0, 1), (4, 5, 3), (2, 3, 0)]
    g.goals = goals
    path = os.path.join(tmp, "grid.pkl")
    try:
        with open(path, "wb") as f:
            gutil.dump_graph(g, f)
    except SystemExit:  # dump_graph ends with exit() (graph/util.py:67) after writing the pickle
        pass
    mod = import_oriented_env()
    env = mod.OrientedGraphEnv(graph_file=path, goals=list(goals), screen_size=(84, 84))
    out = {"o_maze": maze, "o_goals": np.array(goals, dtype=np.int32),
           "o_largest": np.array([env.largest_distance])}
    random.seed(4)
    np.random.seed(4)
    arng = np.random.RandomState(5)
    actions = arng.randint(0, 4, size=6000)
    starts, goals_at, states, rbits, dones, frame_ids = [], [], [], [], [], []
    ob = env.reset()
    starts.append(env.state)
    goals_at.append(env.goal)
    first_frame = (int(ob[0][0, 0, 0]), int(ob[1][0, 0, 0]))
    for a in actions:
        ob, rew, done, info = env.step(int(a))
        states.append(env.state)
        rbits.append(np.float32(rew).view(np.uint32))
        dones.append(done)
        frame_ids.append((int(ob[0][0, 0, 0]), int(ob[1][0, 0, 0])))  # (rgb, third-person) ids
        if done:
            env.reset()
            starts.append(env.state)
            goals_at.append(env.goal)
    out.update(o_actions=actions.astype(np.int32), o_starts=np.array(starts, dtype=np.int32),
               o_goal_seq=np.array(goals_at, dtype=np.int32), o_states=np.array(states, dtype=np.int32),
               o_reward_bits=np.array(rbits, dtype=np.uint32), o_dones=np.array(dones),
               o_frame_ids=np.array(frame_ids, dtype=np.int32), o_first_frame=np.array(first_frame))
    # set_complexity start support (graph.py:47-52): many reference draws per (c, goal)
    cs = [0.05, 0.2, 0.5, 1.0]
    support = np.zeros((len(cs), len(goals), maze.size * 4), dtype=bool)
    for i, c in enumerate(cs):
        env.set_complexity(c)
        for j, goal in enumerate(goals):
            np.random.seed(100 + i * 10 + j)
            opt = c * (env.largest_distance + 4 - 1) + 1
            for _ in range(4000):
                s = gutil.sample_initial_state(env.graph, goal, optimal_distance=opt)
                support[i, j, (s[0] * maze.shape[1] + s[1]) * 4 + s[2]] = True
    out["o_complexities"] = np.array(cs)
    out["o_support_xyr"] = support  # index (x * Y + y) * 4 + r
    return out


def resize_goldens(tmp):
    spec = importlib.util.spec_from_file_location("ref_cached", os.path.join(REF, "environments/gym_ai2thor/envs/cached.py"))
    cached_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cached_mod)
    maze = np.ones((2, 1), dtype=bool)
    rng = np.random.RandomState(8)
    frames = rng.randint(0, 256, size=(8, 100, 100, 3)).astype(np.uint8)
    # smooth half + noisy half so both the anti-aliasing and the interpolation matter
    yy, xx = np.mgrid[0:100, 0:100]
    frames[:, :50] = ((np.sin(xx[:50, :, None] / 3.0 + np.arange(8)[:, None, None, None] / 2.0) + 1) * 127.5
                      ).astype(np.uint8)[:, :, :, :1].repeat(3, axis=3)[:, :50]

    class Grid:
        def __init__(self):
            self.maze = maze
            self.graph = None

        @property
        def observation_shape(self):
            return (100, 100, 3)

        def render(self, location, rotation):
            return frames[list(gutil.enumerate_positions(maze)).index(tuple(location)) * 4 + rotation]

    path = os.path.join(tmp, "big.h5")
    gutil.save_graph_as_h5(Grid(), path)
    env = cached_mod.THORDiscreteCachedEnv(h5_file_path=path, image_size=(84, 84), rand_seed=1)
    pick = [0, 5]
    pre = np.stack([env._preprocess_frame(frames[i]) for i in pick]).astype(np.float32)
    import h5py
    with h5py.File(path, "r") as f:
        graph, spd = f["graph"][()], f["shortest_path_distance"][()]
    return {"r_frames": frames, "r_graph": graph, "r_spd": spd, "r_pick": np.array(pick),
            "r_expected": pre}


def main():
    with tempfile.TemporaryDirectory() as tmp:
        out = oriented_goldens(tmp)
        out.update(resize_goldens(tmp))
    np.savez_compressed(os.path.join(HERE, "ingest.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
