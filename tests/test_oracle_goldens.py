"""Pin the CPU oracle against golden vectors recorded from the reference itself
(tests/golden/gen_env_goldens.py). CPU only."""
import random

import numpy as np

from oracle import envs as oe
from oracle import graph as og
from oracle.frames import synth_frames


def test_h5_tables_match_reference_writer(golden):
    h = golden("h5_scenes.npz")
    for k in range(3):
        graph, spd, loc = og.h5_tables(h["maze%d" % k])
        assert np.array_equal(graph, h["graph%d" % k])
        assert np.array_equal(spd, h["spd%d" % k])
        assert np.array_equal(loc, h["location%d" % k])


def test_isolated_cell_spd_quirk(golden):
    # graph/util.py:240-247: unreachable pairs store -1 + rotation difference
    spd = golden("h5_scenes.npz")["spd0"]
    assert spd.min() == -1 and (spd == 1).any()


def test_cached_env_trajectories(golden):
    h = golden("h5_scenes.npz")
    d = golden("cached_env.npz")
    for ci in range(int(d["n_cases"][0])):
        p = "c%d_" % ci
        scene, rand_seed, global_seed, n_steps, reset_on_done = (int(v) for v in d[p + "meta"])
        graph, spd = h["graph%d" % scene], h["spd%d" % scene]
        sampler = oe.python_random_sampler(len(graph), spd, rand_seed, global_seed)
        env = oe.CachedEnvOracle(graph, spd, sampler)
        resets = [(env.state, env.goal)]
        first = env.reset()
        resets.append((env.state, env.goal))
        assert first[0] == d[p + "first_img_idx"][0]
        for t, a in enumerate(d[p + "actions"]):
            obs, reward, done, info = env.step(int(a))
            assert env.state == d[p + "states"][t], (ci, t)
            assert np.float32(reward).view(np.uint32) == d[p + "reward_bits"][t], (ci, t)
            assert done == bool(d[p + "dones"][t])
            assert obs == (d[p + "img_idx"][t], d[p + "goal_idx"][t]), (ci, t)
            if done and reset_on_done:
                env.reset()
                resets.append((env.state, env.goal))
        assert np.array_equal(np.array(resets), d[p + "resets"])


def test_reward_sign_of_zero(golden):
    d = golden("cached_env.npz")
    bits = set(np.concatenate([d["c%d_reward_bits" % c] for c in range(4)]).tolist())
    # -0.0 plain move, +0.0 collision, 1.0 goal (cached.py:84-88)
    assert bits == {0x80000000, 0x00000000, 0x3F800000}


def test_resize_is_identity_at_equal_size():
    import json
    import os
    from conftest import GOLDEN
    m = json.load(open(os.path.join(GOLDEN, "env_manifest.json")))
    assert m["max_resize_residual"] < 1e-12


def test_multiscene_reset(golden):
    h = golden("h5_scenes.npz")
    d = golden("cached_env.npz")
    tasks = [tuple(t) for t in d["ms_tasks"].tolist()]
    scenes = {k: dict(spd=h["spd%d" % k]) for k in range(3)}
    o = oe.MultiSceneResetOracle(tasks, scenes, random.Random(int(d["ms_seed"][0])))
    for row in d["ms_rows"]:
        scene, goal, s = o.reset()
        assert (scene, goal, s) == (row[0], row[1], row[2])
        assert row[3] == s and row[4] == goal  # raw uint8 frame views of (state, goal)
    assert str(d["ms_process_error"][0]) == "AttributeError"


def test_maze_shortest_paths(golden):
    m = golden("maze.npz")
    dist, acts = og.shortest_path_data(m["maze"])
    assert np.array_equal(dist, m["distances"])
    assert np.array_equal(acts, m["actions"])


def test_maze_env_trajectory(golden):
    m = golden("maze.npz")
    maze, goal = m["maze"], tuple(m["goal"].tolist())
    dist = m["distances"]
    env = oe.SimpleGraphEnvOracle(maze, goal)
    np.random.seed(17)
    starts = [oe.sample_initial_position(maze, dist, goal)]
    obs0 = env.reset(starts[0])
    assert np.array_equal(obs0, m["m_obs0"])
    for t, a in enumerate(m["m_actions"]):
        obs, reward, done, info = env.step(int(a))
        assert tuple(env.state) == tuple(m["m_states"][t])
        assert np.float32(reward).view(np.uint32) == m["m_reward_bits"][t]
        assert done == bool(m["m_dones"][t])
        assert np.array_equal(obs, m["m_obs"][t])
        if done:
            starts.append(oe.sample_initial_position(maze, dist, goal))
            env.reset(starts[-1])
    assert np.array_equal(np.array(starts), m["m_starts"])


def test_curriculum_samplers(golden):
    m = golden("maze.npz")
    maze, goal = m["maze"], tuple(m["goal"].tolist())
    for i, opt in enumerate(m["pos_opts"]):
        np.random.seed(5)
        o = None if opt < 0 else float(opt)
        draws = [oe.sample_initial_position(maze, m["distances"], goal, o) for _ in range(60)]
        assert np.array_equal(np.array(draws), m["pos_samples"][i])
    for i, opt in enumerate(m["state_opts"]):
        np.random.seed(8)
        o = None if opt < 0 else float(opt)
        draws = [oe.sample_initial_state(maze, m["distances"], m["actions"], (6, 5, 1), o) for _ in range(60)]
        assert np.array_equal(np.array(draws), m["state_samples"][i])


def test_synth_frames_deterministic():
    a = synth_frames(3, [0, 5, 7], (8, 8, 3))
    b = synth_frames(3, [0, 5, 7], (8, 8, 3))
    c = synth_frames(4, [0, 5, 7], (8, 8, 3))
    assert a.dtype == np.uint8 and a.shape == (3, 8, 8, 3)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
