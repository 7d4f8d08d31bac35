"""Scene ingestion, CPU only: OrientedGraphEnv tables and pickled
ThorGridWorld loading vs the reference run recorded by tests/golden/gen_ingest_goldens.py,
and the offline h5 conversion/resize tool vs the reference's own preprocessed frames."""
import io
import os
import pickle
import shutil
import subprocess
import sys
import types

import numpy as np
import pytest

from conftest import REPO
from oracle import graph as og
from oracle.envs import compute_rotation_steps
from vnav import scenes

CONDA_PY = "/opt/conda/bin/python3.9"


def _state_index(locs, xyr):
    return {p: i for i, p in enumerate(locs)}[(int(xyr[0]), int(xyr[1]))] * 4 + int(xyr[2])


def _oriented_from_golden(d):
    maze = d["o_maze"]
    X, Y = maze.shape
    # the generator's frames: channel 0 = state id (tp: 255 - id); only ids matter here
    obs = np.zeros((X, Y, 4, 4, 4, 3), dtype=np.uint8)
    for i, (x, y) in enumerate(og.enumerate_positions(maze)):
        for r in range(4):
            obs[x, y, r, :, :, 0] = i * 4 + r
    tp = obs.copy()
    tp[..., 0] = 255 - tp[..., 0]
    return scenes.oriented_scene(maze, obs, [tuple(g) for g in d["o_goals"]], tp_observations=tp)


def test_oriented_tables_match_oracle_rotation_steps(golden):
    """spd = d + compute_rotation_steps (graph/util.py:82-86,119-143) on the reference's
    own distances / optimal actions (maze.npz, recorded from compute_shortest_path_data)."""
    m = golden("maze.npz")
    maze, dist, acts = m["maze"], m["distances"], m["actions"]
    graph, spd, locs, base = scenes.oriented_tables(maze)
    for i, (x, y) in enumerate(locs):
        for j, (gx, gy) in enumerate(locs):
            d = int(dist[x, y, gx, gy])
            assert base[i, j] == d
            for r in range(4):
                for gr in range(4):
                    exp = d + compute_rotation_steps(acts, (gx, gy, gr), (x, y, r)) if d > 0 else (0 if d == 0 else -1)
                    assert spd[i * 4 + r, j * 4 + gr] == exp
    # transitions: graph/util.py:15-25 step + is_valid_state (collision -> -1)
    for i, (x, y) in enumerate(locs):
        for r in range(4):
            for a in range(4):
                nxt = og.oriented_step((x, y, r), a)
                exp = _state_index(locs, nxt) if og.is_valid_state(maze, nxt) else -1
                assert graph[i * 4 + r, a] == exp


def test_oriented_trajectory_matches_reference(golden):
    """Replay the reference OrientedGraphEnv run (starts, goals, actions) through the scene
    tables: states, reward bits, done flags and emitted (rgb, third-person) frame ids."""
    d = golden("ingest.npz")
    sc = _oriented_from_golden(d)
    locs = sc.locations
    starts = [_state_index(locs, s) for s in d["o_starts"]]
    goals = [_state_index(locs, g) for g in d["o_goal_seq"]]
    assert set(goals) <= set(sc.goals)
    r_goal, r_step, r_coll = sc.rewards
    s, g, k = starts[0], goals[0], 0
    assert tuple(d["o_first_frame"]) == (s, 255 - s)
    for t, a in enumerate(d["o_actions"]):
        nxt = sc.graph[s, a]
        coll = nxt < 0
        s = s if coll else int(nxt)
        done = s == g
        rew = r_goal if done else (r_coll if coll else r_step)
        assert s == _state_index(locs, d["o_states"][t]), t
        assert np.float32(rew).view(np.uint32) == d["o_reward_bits"][t], t
        assert done == bool(d["o_dones"][t]), t
        # terminal_obs = 1: the emitted frames are those of the current state
        assert tuple(d["o_frame_ids"][t]) == (sc.observations[s, 0, 0, 0], sc.companion[s, 0, 0, 0]), t
        if done:
            k += 1
            s, g = starts[k], goals[k]
    assert k == len(starts) - 1


def test_oriented_curriculum_support_matches_reference(golden):
    """set_complexity(c): the engine's candidate set 0 < spd <= floor(c*(maxd+offset)+1)
    equals the support of the reference sampler (environments/gym_graph/graph.py:47-52)."""
    d = golden("ingest.npz")
    sc = _oriented_from_golden(d)
    mode, offset = sc.curriculum
    assert mode == 1
    maxd = int(sc.spd.max())
    assert maxd + offset == float(d["o_largest"][0]) + 3
    Y = d["o_maze"].shape[1]
    to_xyr = {}
    for i, (x, y) in enumerate(sc.locations):
        for r in range(4):
            to_xyr[i * 4 + r] = (x * Y + y) * 4 + r
    for ci, c in enumerate(d["o_complexities"]):
        oi = min(max(int(np.floor(float(c) * (maxd + offset) + 1.0)), 0), maxd)
        for gi, goal in enumerate(d["o_goals"]):
            gs = _state_index(sc.locations, goal)
            col = sc.spd[:, gs]
            mine = {to_xyr[s] for s in np.nonzero((col > 0) & (col <= oi))[0]}
            ref = set(np.nonzero(d["o_support_xyr"][ci, gi])[0].tolist())
            assert mine == ref, (c, tuple(goal))


class _FakeGrid:
    pass


def _fake_grid_pickle(maze, obs, tp, goals):
    """A pickle whose class path is graph.thor_graph.ThorGridWorld, as dump_graph writes."""
    mod = types.ModuleType("graph.thor_graph")
    _FakeGrid.__module__ = "graph.thor_graph"
    _FakeGrid.__qualname__ = _FakeGrid.__name__ = "ThorGridWorld"
    mod.ThorGridWorld = _FakeGrid
    saved = {k: sys.modules.get(k) for k in ("graph", "graph.thor_graph")}
    sys.modules.setdefault("graph", types.ModuleType("graph"))
    sys.modules["graph.thor_graph"] = mod
    try:
        g = _FakeGrid()
        g._maze, g._observations, g._tp_observations = maze, obs, tp
        g._depths = g._segmentations = np.zeros(1)
        g.graph, g.optimal_actions = og.shortest_path_data(maze)
        g.goals = goals
        return pickle.dumps(g)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v


def test_load_graph_pickle(tmp_path):
    rng = np.random.RandomState(3)
    maze = rng.rand(4, 5) > 0.3
    maze[0, 0] = True
    obs = rng.randint(0, 256, size=maze.shape + (4, 6, 6, 3)).astype(np.uint8)
    tp = rng.randint(0, 256, size=obs.shape).astype(np.uint8)
    goals = [(0, 0, 2)]
    path = tmp_path / "grid.pkl"
    path.write_bytes(_fake_grid_pickle(maze, obs, tp, goals))
    sc = scenes.load_graph_pickle(str(path))
    ref = scenes.oriented_scene(maze, obs, goals, tp_observations=tp)
    assert np.array_equal(sc.graph, ref.graph) and np.array_equal(sc.spd, ref.spd)
    assert np.array_equal(sc.observations, ref.observations) and np.array_equal(sc.companion, ref.companion)
    assert sc.goals == ref.goals and sc.curriculum == ref.curriculum


def test_load_graph_pickle_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    path = tmp_path / "evil.pkl"
    path.write_bytes(pickle.dumps(Evil()))
    with pytest.raises(pickle.UnpicklingError):
        scenes.load_graph_pickle(str(path))


def _conda_h5_available():
    if not os.path.exists(CONDA_PY):
        return False
    r = subprocess.run([CONDA_PY, "-c", "import h5py, skimage"], capture_output=True)
    return r.returncode == 0


@pytest.mark.skipif(not _conda_h5_available(), reason="needs /opt/conda python with h5py + scikit-image")
def test_h5_to_npz_resize_matches_reference_preprocess(golden, tmp_path):
    """tools/h5_to_npz.py --size 84 84 on a 100x100 h5 scene: tables copied exactly; the
    uint8 frames / 255 are within 0.5/255 of the reference's float frames
    (THORDiscreteCachedEnv._preprocess_frame, cached.py:62-64, recorded by the generator)."""
    d = golden("ingest.npz")
    src = tmp_path / "scene.h5"
    np.savez(tmp_path / "raw.npz", graph=d["r_graph"], spd=d["r_spd"], obs=d["r_frames"])
    writer = ("import h5py, numpy as np; d = np.load(%r); f = h5py.File(%r, 'w'); "
              "f['graph'] = d['graph']; f['shortest_path_distance'] = d['spd']; f['observation'] = d['obs']; "
              "f['location'] = np.zeros((len(d['graph']), 2)); f.close()") % (str(tmp_path / "raw.npz"), str(src))
    subprocess.run([CONDA_PY, "-c", writer], check=True, capture_output=True)
    dst = tmp_path / "scene.npz"
    subprocess.run([CONDA_PY, os.path.join(REPO, "tools", "h5_to_npz.py"), str(src), str(dst), "--size", "84", "84"],
                   check=True, capture_output=True)
    sc = scenes.load_npz(str(dst))
    assert np.array_equal(sc.graph, d["r_graph"]) and np.array_equal(sc.spd, d["r_spd"])
    assert sc.frame_shape == (84, 84, 3)
    got = sc.observations[d["r_pick"]].astype(np.float64) / 255.0
    err = np.abs(got - d["r_expected"].astype(np.float64)).max()
    assert err <= 0.5 / 255 + 1e-6, err
    # same-size conversion is a plain copy
    dst2 = tmp_path / "same.npz"
    subprocess.run([CONDA_PY, os.path.join(REPO, "tools", "h5_to_npz.py"), str(src), str(dst2)], check=True,
                   capture_output=True)
    assert np.array_equal(scenes.load_npz(str(dst2)).observations, d["r_frames"])
