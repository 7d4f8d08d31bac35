"""OrientedGraphEnv scenes (environments/gym_graph/graph.py:9-93, built by
vnav.oriented_scene / load_graph_pickle) through the engine on the GPU, replaying the
reference run recorded by tests/golden/gen_ingest_goldens.py. Bit-exact: states, reward
bits, done flags and the emitted (rgb, third-person) frames; set_complexity draws cover
exactly the reference sampler's support."""
import numpy as np
import pytest
import torch

from test_ingest import _oriented_from_golden, _state_index

pytestmark = pytest.mark.gpu


def test_oriented_env_replays_reference(golden):
    import vnav
    d = golden("ingest.npz")
    sc = _oriented_from_golden(d)
    locs = sc.locations
    starts = [_state_index(locs, s) for s in d["o_starts"]]
    goals = [_state_index(locs, g) for g in d["o_goal_seq"]]
    env = vnav.make("OrientedGraph-v0", [sc], 1, seed=0, max_episode_steps=0)
    env.set_schedule(np.array([list(zip(starts, goals))], dtype=np.int32))
    img, comp = env.reset()
    assert (int(img[0, 0, 0, 0]), int(comp[0, 0, 0, 0])) == tuple(d["o_first_frame"])
    k = 0
    for t, a in enumerate(d["o_actions"]):
        (img, comp), reward, done, info = env.step(torch.tensor([int(a)], device="cuda"))
        assert reward.cpu().numpy().view(np.uint32)[0] == d["o_reward_bits"][t], t
        assert bool(done.item()) == bool(d["o_dones"][t]), t
        ts = int(info["terminal_state"].item())
        assert ts == _state_index(locs, d["o_states"][t]), t
        assert (int(sc.observations[ts, 0, 0, 0]), int(sc.companion[ts, 0, 0, 0])) == tuple(d["o_frame_ids"][t])
        if done.item():
            k += 1
            assert int(info["state"].item()) == starts[k]
        s = int(info["state"].item())
        # emitted frames: the current (post-reset) state's rgb and third-person views
        assert np.array_equal(img[0].cpu().numpy(), sc.observations[s])
        assert np.array_equal(comp[0].cpu().numpy(), sc.companion[s])
    assert k == len(starts) - 1


def test_oriented_curriculum_draws_cover_reference_support(golden):
    import vnav
    d = golden("ingest.npz")
    sc = _oriented_from_golden(d)
    Y = d["o_maze"].shape[1]
    to_xyr = np.zeros(sc.n_states, dtype=np.int64)
    for i, (x, y) in enumerate(sc.locations):
        for r in range(4):
            to_xyr[i * 4 + r] = (x * Y + y) * 4 + r
    gidx = [_state_index(sc.locations, g) for g in d["o_goals"]]
    E = 4096
    env = vnav.VectorEnv([sc], E, seed=11, max_episode_steps=0)  # tasks = the scene's goals
    for ci, c in enumerate(d["o_complexities"]):
        env.set_complexity(float(c))
        seen = np.zeros((len(gidx), sc.n_states), dtype=bool)
        for _ in range(6):
            env.reset()
            st = env.get_state().cpu().numpy()
            for j, g in enumerate(gidx):
                seen[j, st[1][st[2] == g]] = True
        for j in range(len(gidx)):
            mine = set(to_xyr[np.nonzero(seen[j])[0]].tolist())
            ref = set(np.nonzero(d["o_support_xyr"][ci, j])[0].tolist())
            assert mine == ref, (float(c), j)
    assert env.error_flags() == 0
