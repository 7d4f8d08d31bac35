"""Generate env / graph golden vectors by running the REFERENCE code in this container.

Run ONLY in the build container (the reference tree is not on the GPU box):
    /opt/conda/bin/python3.9 tests/golden/gen_env_goldens.py
(Anaconda 3.9 has h5py 3.3 and scikit-image 0.18, which the reference env needs.)

What it does
  1. builds small grid scenes, writes them with the reference's own h5 writer
     graph/util.py:save_graph_as_h5 (np.int/np.float/np.bool aliases restored and the
     remote resnet50 feature extractor replaced by zeros — it only fills
     'resnet_feature', which the env never reads);
  2. drives environments/gym_ai2thor/envs/cached.py:THORDiscreteCachedEnv on those h5
     files with seeded ``random`` / ``rand_seed`` and seeded actions, recording every
     reset (start, goal) and every step (state, reward bits, done, emitted frame index);
  3. drives environments/gym_thor_cached.py:THORCachedEnv.reset (multi-scene tasks);
  4. records graph/util.py compute_shortest_path_data, sample_initial_position /
     sample_initial_state and graph/env.py SimpleGraphEnv trajectories (maze, config C1).
Outputs go to tests/golden/*.npz (small fixtures: inputs + expected outputs only).
"""
import importlib.util
import json
import os
import random
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path[:0] = [os.path.join(HERE, "stubs"), REF, REPO]

# numpy aliases removed in 1.24 that the reference still uses (util.py:148,223-224)
np.int = int
np.float = float
np.bool = bool

from oracle.frames import synth_frames  # noqa: E402  (our own hash, numpy only)

import graph.util as gutil  # noqa: E402

gutil.create_resnet = lambda: (lambda observation: np.zeros(2048, dtype=np.float32))


def load_by_path(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


cached_mod = load_by_path("ref_cached", os.path.join(REF, "environments/gym_ai2thor/envs/cached.py"))
multi_mod = load_by_path("ref_gym_thor_cached", os.path.join(REF, "environments/gym_thor_cached.py"))

FRAME_SHAPE = (84, 84, 3)


class FakeThorGrid:
    """Scene object for save_graph_as_h5: maze + render(location, rotation)."""

    def __init__(self, maze, scene_id):
        self.maze = maze
        self.graph = None
        self.scene_id = scene_id
        self.lookup = {p: i for i, p in enumerate(gutil.enumerate_positions(maze))}

    @property
    def observation_shape(self):
        return FRAME_SHAPE

    def render(self, location, rotation):
        idx = self.lookup[tuple(location)] * 4 + rotation
        return synth_frames(self.scene_id, [idx], FRAME_SHAPE)[0]


def make_mazes():
    rng = np.random.RandomState(7)
    m0 = rng.rand(6, 6) > 0.25
    m0[0, 0] = True
    m0[5, 5], m0[4, 5], m0[5, 4] = True, False, False  # isolated cell: spd = -1 + rotation quirk
    m1 = np.ones((4, 4), dtype=bool)
    m2 = rng.rand(5, 7) > 0.2
    m2[2, 3] = True
    return [m0, m1, m2]


def write_h5_scenes(tmp):
    out = {}
    paths = []
    for k, maze in enumerate(make_mazes()):
        g = FakeThorGrid(maze, scene_id=100 + k)
        name = "scene%d" % k
        path = os.path.join(tmp, name + ".h5")
        gutil.save_graph_as_h5(g, path)
        import h5py
        with h5py.File(path, "r") as f:
            out["maze%d" % k] = maze
            out["graph%d" % k] = f["graph"][()]
            out["spd%d" % k] = f["shortest_path_distance"][()]
            out["location%d" % k] = f["location"][()]
            obs = f["observation"][()]
        expect = synth_frames(100 + k, np.arange(len(obs)), FRAME_SHAPE)
        assert np.array_equal(obs, expect), "h5 observation dataset differs from the hash frames"
        paths.append(path)
    return out, paths


def frame_index(img, frames01):
    """Index of the frame the (resized) float image came from, and the residual."""
    d = np.abs(frames01 - img[None]).reshape(len(frames01), -1).max(axis=1)
    i = int(np.argmin(d))
    return i, float(d[i])


def cached_trajectories(paths):
    rec = {}
    cases = [  # (scene, rand_seed, global_seed, n_steps, reset_on_done)
        (0, 11, 5, 700, True),
        (1, 3, 9, 700, True),
        (2, 21, 13, 700, True),
        (1, 4, 2, 60, False),   # keeps stepping after terminal: last_state quirk, collided at goal
    ]
    max_resize_residual = 0.0
    for ci, (scene, rand_seed, global_seed, n_steps, reset_on_done) in enumerate(cases):
        random.seed(global_seed)
        env = cached_mod.THORDiscreteCachedEnv(h5_file_path=paths[scene], rand_seed=rand_seed,
                                               image_size=(84, 84))
        frames01 = env._observations.astype(np.float64) / 255.0
        resets = [(int(env._current_state_idx), int(env._current_goal_idx))]
        # the VecEnv calls reset() once more before the first step
        first = env.reset()
        resets.append((int(env._current_state_idx), int(env._current_goal_idx)))
        arng = np.random.RandomState(1000 + ci)
        actions = arng.randint(0, 4, size=n_steps)
        states, rewards, dones, img_idx, goal_idx, reset_at = [], [], [], [], [], []
        i0, r0 = frame_index(first[0], frames01)
        max_resize_residual = max(max_resize_residual, r0)
        for t, a in enumerate(actions):
            obs, reward, done, info = env.step(int(a))
            assert info == {}
            ii, ri = frame_index(obs[0], frames01)
            gi, rg = frame_index(obs[1], frames01)
            max_resize_residual = max(max_resize_residual, ri, rg)
            states.append(int(env._current_state_idx))
            rewards.append(np.float32(reward).view(np.uint32))
            dones.append(bool(done))
            img_idx.append(ii)
            goal_idx.append(gi)
            if done and reset_on_done:
                env.reset()
                resets.append((int(env._current_state_idx), int(env._current_goal_idx)))
                reset_at.append(t)
        p = "c%d_" % ci
        rec[p + "meta"] = np.array([scene, rand_seed, global_seed, n_steps, int(reset_on_done)])
        rec[p + "actions"] = actions.astype(np.int32)
        rec[p + "resets"] = np.array(resets, dtype=np.int32)
        rec[p + "reset_at"] = np.array(reset_at, dtype=np.int32)
        rec[p + "states"] = np.array(states, dtype=np.int32)
        rec[p + "reward_bits"] = np.array(rewards, dtype=np.uint32)
        rec[p + "dones"] = np.array(dones, dtype=bool)
        rec[p + "img_idx"] = np.array(img_idx, dtype=np.int32)
        rec[p + "goal_idx"] = np.array(goal_idx, dtype=np.int32)
        rec[p + "first_img_idx"] = np.array([i0], dtype=np.int32)
    rec["n_cases"] = np.array([len(cases)])
    rec["max_resize_residual"] = np.array([max_resize_residual])
    return rec


def multiscene(tmpdir):
    os.environ["THOR_DATASET_PATH"] = tmpdir
    tasks = [("scene0", 3), ("scene2", 10), ("scene1", 7), ("scene2", 0)]
    env = multi_mod.THORCachedEnv(tasks)
    env._random = random.Random(1234)
    names = {"scene0": 0, "scene1": 1, "scene2": 2}
    rows = []
    for _ in range(40):
        obs, goal = env.reset()
        sc = env.current_scene
        idx = int(np.nonzero((sc["observations"] == obs).reshape(len(sc["observations"]), -1).all(1))[0][0])
        gidx = int(np.nonzero((sc["observations"] == goal).reshape(len(sc["observations"]), -1).all(1))[0][0])
        scene_name = [k for k, v in env.scenes.items() if v is sc][0]
        rows.append((names[scene_name], env.goal, env.state, idx, gidx))
    step_error = ""
    try:
        env.process(0)
    except Exception as ex:  # documented: broken twin of cached.py step
        step_error = type(ex).__name__
    return {"ms_tasks": np.array([(names[s], g) for s, g in tasks], dtype=np.int32),
            "ms_rows": np.array(rows, dtype=np.int32),
            "ms_seed": np.array([1234]),
            "ms_process_error": np.array([step_error])}


def maze_goldens():
    import graph.env as genv
    from graph.maze_graph import MazeGraph

    rng = np.random.RandomState(3)
    maze = rng.rand(8, 8) > 0.3
    maze[1, 1] = maze[6, 5] = True
    goal = (6, 5)
    dist, acts = gutil.compute_shortest_path_data(maze)
    out = {"maze": maze, "goal": np.array(goal), "distances": dist, "actions": acts}

    mg = MazeGraph(maze, goal)
    env = genv.SimpleGraphEnv(mg)
    np.random.seed(17)
    random.seed(17)
    arng = np.random.RandomState(99)
    starts, states, rewards, dones, obs_list, resets_at = [], [], [], [], [], []
    obs = env.reset()
    starts.append(env.state)
    obs0 = obs
    actions = arng.randint(0, 4, size=1500)
    for t, a in enumerate(actions):
        obs, reward, done, info = env.step(int(a))
        states.append(env.state)
        rewards.append(np.float32(reward).view(np.uint32))
        dones.append(done)
        obs_list.append(obs)
        if done:
            env.reset()
            starts.append(env.state)
            resets_at.append(t)
    out.update(m_actions=actions.astype(np.int32), m_starts=np.array(starts, dtype=np.int32),
               m_states=np.array(states, dtype=np.int32), m_reward_bits=np.array(rewards, dtype=np.uint32),
               m_dones=np.array(dones), m_obs=np.array(obs_list, dtype=np.float32), m_obs0=obs0.astype(np.float32),
               m_resets_at=np.array(resets_at, dtype=np.int32))

    # curriculum samplers (graph/util.py:88-143): positions for several optimal distances
    samples = []
    for opt in (None, 1.0, 3.0, 6.5):
        np.random.seed(5)
        draws = [gutil.sample_initial_position(mg, goal, optimal_distance=opt) for _ in range(60)]
        samples.append(draws)
    out["pos_samples"] = np.array(samples, dtype=np.int32)
    out["pos_opts"] = np.array([-1.0, 1.0, 3.0, 6.5])

    class Oriented:
        pass

    og = Oriented()
    og.maze = maze
    og.graph, og.optimal_actions = dist, acts
    state_samples = []
    for opt in (None, 2.0, 5.0):
        np.random.seed(8)
        state_samples.append([gutil.sample_initial_state(og, (6, 5, 1), optimal_distance=opt) for _ in range(60)])
    out["state_samples"] = np.array(state_samples, dtype=np.int32)
    out["state_opts"] = np.array([-1.0, 2.0, 5.0])
    return out


def main():
    with tempfile.TemporaryDirectory() as tmp:
        scenes, paths = write_h5_scenes(tmp)
        traj = cached_trajectories(paths)
        ms = multiscene(tmp)
    mz = maze_goldens()
    np.savez_compressed(os.path.join(HERE, "h5_scenes.npz"), **scenes)
    np.savez_compressed(os.path.join(HERE, "cached_env.npz"), **traj, **ms)
    np.savez_compressed(os.path.join(HERE, "maze.npz"), **mz)
    manifest = {
        "generator": "tests/golden/gen_env_goldens.py",
        "python": sys.version.split()[0],
        "numpy": np.__version__,
        "frame_shape": FRAME_SHAPE,
        "scene_ids": [100, 101, 102],
        "max_resize_residual": float(traj["max_resize_residual"][0]),
        "thor_cached_process_error": str(ms["ms_process_error"][0]),
    }
    with open(os.path.join(HERE, "env_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest, indent=1))


if __name__ == "__main__":
    main()
