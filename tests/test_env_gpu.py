"""VectorEnv (libvnav.so vn_step) on the GPU vs the reference goldens and the oracle.

Bit-exact: states, done, reward bits, emitted frame indices and the gathered bytes.
"""
import numpy as np
import pytest
import torch

from oracle import envs as oe
from oracle import graph as og
from oracle.frames import synth_frames

pytestmark = pytest.mark.gpu

FRAME = (84, 84, 3)


def _vnav():
    import vnav
    return vnav


def golden_scenes(golden):
    vnav = _vnav()
    h = golden("h5_scenes.npz")
    out = []
    for k in range(3):
        frames = synth_frames(100 + k, np.arange(len(h["graph%d" % k])), FRAME)
        out.append(vnav.scene_from_arrays(h["graph%d" % k], h["spd%d" % k], frames))
    return out


def test_golden_replay_autoreset(golden):
    vnav = _vnav()
    d = golden("cached_env.npz")
    sc = golden_scenes(golden)
    cases = [0, 1, 2]
    metas = [d["c%d_meta" % c] for c in cases]
    n_steps = int(metas[0][3])
    L = max(len(d["c%d_resets" % c]) for c in cases) - 1
    sched = np.zeros((len(cases), L, 2), dtype=np.int32)
    for i, c in enumerate(cases):
        r = d["c%d_resets" % c][1:]
        sched[i, : len(r)] = r
        sched[i, len(r):] = r[-1]
    env = vnav.VectorEnv(sc, len(cases), seed=1, env_scenes=[int(m[0]) for m in metas], max_episode_steps=0)
    env.set_schedule(sched)
    img, goal = env.reset()
    for i, c in enumerate(cases):
        frames = sc[int(metas[i][0])].observations
        assert np.array_equal(img[i].cpu().numpy(), frames[d["c%d_first_img_idx" % c][0]])
    k = [1] * len(cases)
    acts = np.stack([d["c%d_actions" % c] for c in cases], 1)
    for t in range(n_steps):
        (img, goal), reward, done, info = env.step(torch.as_tensor(acts[t], device="cuda"))
        img, goal = img.cpu().numpy(), goal.cpu().numpy()
        rb = reward.cpu().numpy().view(np.uint32)
        dn = done.cpu().numpy()
        st = info["state"].cpu().numpy()
        ts = info["terminal_state"].cpu().numpy()
        for i, c in enumerate(cases):
            p = "c%d_" % c
            frames = sc[int(metas[i][0])].observations
            assert rb[i] == d[p + "reward_bits"][t], (c, t)
            assert bool(dn[i]) == bool(d[p + "dones"][t]), (c, t)
            assert ts[i] == d[p + "img_idx"][t], (c, t)
            if dn[i]:
                s0, g0 = d[p + "resets"][k[i] + 1]
                k[i] += 1
                assert st[i] == s0
                assert np.array_equal(img[i], frames[s0]) and np.array_equal(goal[i], frames[g0])
            else:
                assert st[i] == d[p + "states"][t], (c, t)
                assert np.array_equal(img[i], frames[d[p + "img_idx"][t]]), (c, t)
                assert np.array_equal(goal[i], frames[d[p + "goal_idx"][t]]), (c, t)
    assert env.error_flags() == 0


def test_golden_no_reset_last_state_quirk(golden):
    vnav = _vnav()
    d = golden("cached_env.npz")
    sc = golden_scenes(golden)
    p = "c3_"
    scene = int(d[p + "meta"][0])
    env = vnav.VectorEnv(sc, 1, seed=2, env_scenes=[scene], max_episode_steps=0, autoreset=False)
    env.set_schedule(d[p + "resets"][1:][None].astype(np.int32))
    env.reset()
    frames = sc[scene].observations
    for t, a in enumerate(d[p + "actions"]):
        (img, goal), reward, done, info = env.step(torch.tensor([int(a)], device="cuda"))
        assert info["state"].item() == d[p + "states"][t]
        assert reward.cpu().numpy().view(np.uint32)[0] == d[p + "reward_bits"][t]
        assert bool(done.item()) == bool(d[p + "dones"][t])
        assert np.array_equal(img[0].cpu().numpy(), frames[d[p + "img_idx"][t]])
        assert np.array_equal(goal[0].cpu().numpy(), frames[d[p + "goal_idx"][t]])


def test_single_env_gym_surface_replays_golden(golden):
    """CachedThorEnv (the single THORDiscreteCachedEnv surface, no auto-reset) replays the
    reference's no-reset trajectory: states, reward bits, dones, and the float64 frames
    _preprocess_frame returns at equal size (u8 / 255), previous obs on terminal steps."""
    vnav = _vnav()
    d = golden("cached_env.npz")
    sc = golden_scenes(golden)
    p = "c3_"
    scene = int(d[p + "meta"][0])
    env = vnav.CachedThorEnv(sc[scene], seed=2, max_episode_steps=0)
    env.set_schedule(d[p + "resets"][1:])
    img, goal = env.reset()
    assert img.dtype == np.float64 and img.shape == FRAME
    frames = sc[scene].observations
    s0, g0 = d[p + "resets"][1]
    assert env.state == (s0, g0)
    assert np.array_equal(img, frames[s0] / 255.0) and np.array_equal(goal, frames[g0] / 255.0)
    for t, a in enumerate(d[p + "actions"]):
        (img, goal), reward, done, info = env.step(int(a))
        assert env.state[0] == d[p + "states"][t], t
        assert np.float32(reward).view(np.uint32) == d[p + "reward_bits"][t], t
        assert done == bool(d[p + "dones"][t]), t
        assert info == {}
        assert np.array_equal(img, frames[d[p + "img_idx"][t]] / 255.0), t
        assert np.array_equal(goal, frames[d[p + "goal_idx"][t]] / 255.0), t
    env.close()


def test_single_env_time_limit_truncates():
    """gym's TimeLimit under the single-env surface: done with TimeLimit.truncated at the
    step limit, then reset() starts a new episode."""
    vnav = _vnav()
    sc = small_scenes()
    env = vnav.CachedThorEnv(sc[1], seed=5, max_episode_steps=3)
    env.reset()
    g = env.state[1]
    seen = None
    for t in range(3):
        _, _, done, info = env.step(0)
        if done:
            seen = (t, info)
            break
    assert seen is not None
    if env.state[0] != g:  # not at the goal: the limit ended it
        assert seen == (2, {"TimeLimit.truncated": True})
    env.close()


def small_scenes(shape=(6, 10, 3)):
    vnav = _vnav()
    out = []
    for k, (X, Y, p) in enumerate([(6, 8, 0.3), (5, 5, 0.0), (7, 4, 0.25)]):
        maze = np.random.RandomState(40 + k).rand(X, Y) >= p
        graph, spd, _ = og.h5_tables(maze)
        if np.prod(shape) % 4 == 0:
            frames = synth_frames(7 + k, np.arange(len(graph)), shape)
        else:  # the hash frames are whole words; odd frame sizes get seeded random bytes
            frames = np.random.RandomState(7 + k).randint(0, 256, size=(len(graph),) + tuple(shape)).astype(np.uint8)
        out.append(vnav.scene_from_arrays(graph, spd, frames))
    return out


def oracle_of(scenes, n, seed, **kw):
    sd = [dict(graph=s.graph, spd=s.spd, rewards=s.rewards, terminal_obs=s.terminal_obs) for s in scenes]
    return oe.VectorEnvOracle(sd, n, seed, **kw)


def compare_step(env_out, o, arena, tag):
    (img, goal), reward, done, info = env_out
    assert np.array_equal(reward.cpu().numpy().view(np.uint32), o["reward"].view(np.uint32)), tag
    assert np.array_equal(done.cpu().numpy(), o["done"]), tag
    assert np.array_equal(info["state"].cpu().numpy(), o["state"]), tag
    assert np.array_equal(info["img_row"].cpu().numpy(), o["img_row"]), tag
    assert np.array_equal(info["goal_row"].cpu().numpy(), o["goal_row"]), tag
    assert np.array_equal(info["ep_length"].cpu().numpy(), o["ep_length"]), tag
    assert np.array_equal(info["terminal_state"].cpu().numpy(), o["terminal_state"]), tag
    assert np.array_equal(info["truncated"].cpu().numpy().astype(bool), o["truncated"]), tag
    assert np.array_equal(info["ep_return"].cpu().numpy().view(np.uint32), o["ep_return"].view(np.uint32)), tag
    if img is not None:
        assert np.array_equal(img.cpu().numpy(), arena[o["img_row"]]), tag
        assert np.array_equal(goal.cpu().numpy(), arena[o["goal_row"]]), tag


@pytest.mark.parametrize("mode", ["env_scene", "tasks"])
def test_vector_env_matches_oracle(mode):
    vnav = _vnav()
    sc = small_scenes()
    arena = np.concatenate([s.observations for s in sc])
    n = 1000
    kw = dict(max_episode_steps=25)
    tasks = None
    if mode == "tasks":
        tasks = [(0, 3), (2, -1), (1, 9), (0, -1)]
    env = vnav.VectorEnv(sc, n, seed=12345, tasks=tasks, **kw)
    o = oracle_of(sc, n, 12345, max_steps=25, tasks=tasks)
    if tasks:  # the constructor reset ran before the tasks were set: re-draw both sides
        env.reset()
        o.reset()
    obs = env.observe()
    ob = o.observe()
    assert np.array_equal(obs[0].cpu().numpy(), arena[ob["img_row"]])
    rng = np.random.RandomState(0)
    for t in range(120):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        if t % 37 == 5:
            a[::97] = -1
            a[1::101] = 4
        out = env.step(torch.as_tensor(a, device="cuda"))
        compare_step(out, o.step(a), arena, (mode, t))
    assert env.error_flags() == o.flags == oe.FLAG_BAD_ACTION


@pytest.mark.parametrize("shape,offset", [((5, 7, 3), 0), ((6, 10, 3), 0), ((4, 8, 3), 0), ((4, 8, 3), 1),
                                          ((4, 8, 3), 4)])
def test_frame_copy_paths_ragged(shape, offset):
    """The 16-B, 4-B and 1-B frame copy paths of vn_step (frame bytes 96 / 180 / 105, and 96
    into output buffers offset by 1 and 4 bytes) at a ragged env count (37 = 9 full
    workgroups + 1 env), bit-exact vs the oracle, with caller-owned outputs."""
    vnav = _vnav()
    sc = small_scenes(shape)
    arena = np.concatenate([s.observations for s in sc])
    n, F = 37, int(np.prod(shape))
    env = vnav.VectorEnv(sc, n, seed=4242, max_episode_steps=11)
    o = oracle_of(sc, n, 4242, max_steps=11)
    buf = torch.zeros(2 * (n * F + 16), dtype=torch.uint8, device="cuda")
    img = buf[offset:offset + n * F].view((n,) + shape)
    g0 = n * F + 16 + offset
    goal = buf[g0:g0 + n * F].view((n,) + shape)
    out = dict(image=img, goal=goal, reward=torch.empty(n, dtype=torch.float32, device="cuda"),
               done=torch.empty(n, dtype=torch.bool, device="cuda"), state=torch.empty(n, dtype=torch.int32, device="cuda"))
    rng = np.random.RandomState(5)
    for t in range(50):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        compare_step(env.step(torch.as_tensor(a, device="cuda"), out=out), o.step(a), arena, (shape, offset, t))
    # nothing outside the two output rows was touched
    b = buf.cpu().numpy()
    assert not b[:offset].any() and not b[offset + n * F:g0].any() and not b[g0 + n * F:].any()


def test_bad_buffers_are_refused():
    """Caller-owned buffers the kernels would write past (or misread) raise before launch."""
    vnav = _vnav()
    sc = small_scenes()
    n = 8
    env = vnav.VectorEnv(sc, n, seed=1)
    F = int(np.prod(env.frame_shape))
    ok = dict(image=torch.empty((n,) + env.frame_shape, dtype=torch.uint8, device="cuda"),
              goal=torch.empty((n,) + env.frame_shape, dtype=torch.uint8, device="cuda"),
              reward=torch.empty(n, dtype=torch.float32, device="cuda"),
              done=torch.empty(n, dtype=torch.bool, device="cuda"),
              state=torch.empty(n, dtype=torch.int32, device="cuda"))
    a = torch.zeros(n, dtype=torch.int32, device="cuda")
    env.step(a, out=ok)
    bad = [("image", torch.empty(n * F - 1, dtype=torch.uint8, device="cuda")),
           ("goal", torch.empty((n,) + env.frame_shape, dtype=torch.float32, device="cuda")),
           ("image", torch.empty((n, 2 * F), dtype=torch.uint8, device="cuda")[:, ::2]),
           ("reward", torch.empty(n + 1, dtype=torch.float32, device="cuda")),
           ("done", torch.empty(n, dtype=torch.uint8, device="cuda")),
           ("state", torch.empty(n, dtype=torch.int64, device="cuda")),
           ("image", torch.empty((n,) + env.frame_shape, dtype=torch.uint8))]
    for k, t in bad:
        with pytest.raises(ValueError):
            env.step(a, out=dict(ok, **{k: t}))
    with pytest.raises(ValueError):
        env.step(torch.zeros(n + 1, dtype=torch.int32, device="cuda"))
    with pytest.raises(ValueError):
        env.reset(torch.ones(n - 1, dtype=torch.bool, device="cuda"))
    with pytest.raises(ValueError):
        env.observe(out=(ok["image"], ok["goal"][:1]))
    with pytest.raises(vnav.VnavError):
        vnav.VectorEnv(sc, 0)
    assert env.error_flags() == 0


def test_c4_env_count_on_one_gpu():
    """Config C4's whole env count (32768 envs, 20 synthetic scenes, 84x84 frames) on one
    GPU: states, rewards, dones and frame rows bit-exact vs the oracle over 12 steps,
    gathered bytes checked on a sample, no error flags."""
    vnav = _vnav()
    sc = [vnav.synthetic_scene(k) for k in range(20)]
    n = 32768
    env = vnav.VectorEnv(sc, n, seed=2024)
    o = oracle_of(sc, n, 2024, max_steps=900)
    bases = np.concatenate([[0], np.cumsum([s.n_states for s in sc])[:-1]])
    rng = np.random.RandomState(11)
    sample = np.sort(rng.choice(n, 48, replace=False))
    idx = torch.as_tensor(sample, device="cuda")
    for t in range(12):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        (img, goal), reward, done, info = env.step(torch.as_tensor(a, device="cuda"))
        ob = o.step(a)
        assert np.array_equal(info["state"].cpu().numpy(), ob["state"]), t
        assert np.array_equal(done.cpu().numpy(), ob["done"]), t
        assert np.array_equal(reward.cpu().numpy().view(np.uint32), ob["reward"].view(np.uint32)), t
        assert np.array_equal(info["img_row"].cpu().numpy(), ob["img_row"]), t
        assert np.array_equal(info["goal_row"].cpu().numpy(), ob["goal_row"]), t
        if t % 4 == 3:
            im, gl = img[idx].cpu().numpy(), goal[idx].cpu().numpy()
            for j, e in enumerate(sample):
                k = int(o.scene[e])
                assert np.array_equal(im[j], synth_frames(k, [ob["img_row"][e] - bases[k]], FRAME)[0])
                assert np.array_equal(gl[j], synth_frames(k, [ob["goal_row"][e] - bases[k]], FRAME)[0])
    assert env.error_flags() == 0


def test_index_only_step_and_masked_reset():
    vnav = _vnav()
    sc = small_scenes()
    n = 300
    env = vnav.VectorEnv(sc, n, seed=9, max_episode_steps=40)
    o = oracle_of(sc, n, 9, max_steps=40)
    arena = np.concatenate([s.observations for s in sc])
    rng = np.random.RandomState(1)
    for t in range(60):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        out = env.step(torch.as_tensor(a, device="cuda"), gather=(t % 2 == 0))
        compare_step(out, o.step(a), arena, t)
        if t == 30:
            mask = np.zeros(n, dtype=bool)
            mask[::3] = True
            env.reset(torch.as_tensor(mask, device="cuda"))
            o.reset(mask)


def test_c2_single_scene_1024_envs():
    """Config C2's shape (cached THOR, 1 scene, 1024 envs, 84x84 frames; BASELINE.json): a
    synthetic 24x24 scene at full frame size, states / rewards / dones / frame rows bit-exact
    vs the oracle over 40 steps (auto-resets included), gathered bytes on a sample."""
    vnav = _vnav()
    sc = [vnav.synthetic_scene(3)]
    n = 1024
    env = vnav.VectorEnv(sc, n, seed=4242)
    o = oracle_of(sc, n, 4242, max_steps=900)
    rng = np.random.RandomState(5)
    sample = np.sort(rng.choice(n, 32, replace=False))
    idx = torch.as_tensor(sample, device="cuda")
    done_seen = 0
    for t in range(40):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        (img, goal), reward, done, info = env.step(torch.as_tensor(a, device="cuda"))
        ob = o.step(a)
        assert np.array_equal(info["state"].cpu().numpy(), ob["state"]), t
        assert np.array_equal(done.cpu().numpy(), ob["done"]), t
        assert np.array_equal(reward.cpu().numpy().view(np.uint32), ob["reward"].view(np.uint32)), t
        assert np.array_equal(info["img_row"].cpu().numpy(), ob["img_row"]), t
        assert np.array_equal(info["goal_row"].cpu().numpy(), ob["goal_row"]), t
        done_seen += int(ob["done"].sum())
        if t % 8 == 7:
            im, gl = img[idx].cpu().numpy(), goal[idx].cpu().numpy()
            for j, e in enumerate(sample):
                assert np.array_equal(im[j], synth_frames(3, [ob["img_row"][e]], FRAME)[0])
                assert np.array_equal(gl[j], synth_frames(3, [ob["goal_row"][e]], FRAME)[0])
    assert done_seen > 0  # episodes ended and were reset inside the window
    assert env.error_flags() == 0


def test_full_size_synthetic_scenes():
    """Config C3's shape: 4096 envs, 4 synthetic 24x24 scenes, 84x84 frames synthesised on
    the device."""
    vnav = _vnav()
    sc = [vnav.synthetic_scene(k) for k in range(4)]
    n = 4096
    env = vnav.VectorEnv(sc, n, seed=77)
    o = oracle_of(sc, n, 77, max_steps=900)
    bases = np.concatenate([[0], np.cumsum([s.n_states for s in sc])[:-1]])
    rng = np.random.RandomState(3)
    sample = rng.choice(n, 64, replace=False)
    for t in range(40):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        (img, goal), reward, done, info = env.step(torch.as_tensor(a, device="cuda"))
        ob = o.step(a)
        assert np.array_equal(info["state"].cpu().numpy(), ob["state"])
        assert np.array_equal(done.cpu().numpy(), ob["done"])
        assert np.array_equal(reward.cpu().numpy().view(np.uint32), ob["reward"].view(np.uint32))
        assert np.array_equal(info["img_row"].cpu().numpy(), ob["img_row"])
        if t % 10 == 0:
            im = img[torch.as_tensor(sample, device="cuda")].cpu().numpy()
            gl = goal[torch.as_tensor(sample, device="cuda")].cpu().numpy()
            for j, e in enumerate(sample):
                k = int(o.scene[e])
                row_i, row_g = ob["img_row"][e] - bases[k], ob["goal_row"][e] - bases[k]
                assert np.array_equal(im[j], synth_frames(k, [row_i], FRAME)[0])
                assert np.array_equal(gl[j], synth_frames(k, [row_g], FRAME)[0])


def test_maze_config_c1(golden):
    """SimpleGraphEnv maze (graph/env.py) through the engine, replaying the golden starts."""
    vnav = _vnav()
    m = golden("maze.npz")
    maze, goal = m["maze"], tuple(m["goal"].tolist())
    scene = vnav.maze_scene(maze, goal)
    lookup = {p: i for i, p in enumerate(scene.locations)}
    g = scene.goals[0]
    starts = [lookup[tuple(s)] for s in m["m_starts"].tolist()]
    env = vnav.VectorEnv([scene], 1, seed=0, tasks=[(0, g)], max_episode_steps=0)
    env.set_schedule(np.array([[(s, g) for s in starts]], dtype=np.int32))
    img, _ = env.reset()
    assert np.array_equal(img[0].cpu().numpy().astype(np.float32) / 255.0, m["m_obs0"])
    k = 0
    for t, a in enumerate(m["m_actions"]):
        (img, _), reward, done, info = env.step(torch.tensor([int(a)], device="cuda"))
        assert reward.cpu().numpy().view(np.uint32)[0] == m["m_reward_bits"][t]
        assert bool(done.item()) == bool(m["m_dones"][t])
        ts = int(info["terminal_state"].item())
        assert scene.locations[ts] == tuple(m["m_states"][t])
        frame = scene.observations[ts].astype(np.float32) / 255.0
        assert np.array_equal(frame, m["m_obs"][t])
        if done.item():
            k += 1
            assert info["state"].item() == starts[k]


def test_reset_exhausted_flag():
    vnav = _vnav()
    # state 2 is unreachable from everything: spd[:, 2] <= 0
    graph = np.array([[1, -1, -1, -1], [0, -1, -1, -1], [-1, -1, -1, -1]], dtype=np.int64)
    spd = np.array([[0, 1, -1], [1, 0, -1], [-1, -1, 0]], dtype=np.int64)
    frames = synth_frames(1, np.arange(3), (4, 4, 4))
    scene = vnav.scene_from_arrays(graph, spd, frames)
    env = vnav.VectorEnv([scene], 64, seed=5, tasks=[(0, 2)])
    env.reset()
    torch.cuda.synchronize()
    assert env.error_flags() & oe.FLAG_RESET_EXHAUSTED


def test_state_checkpoint_roundtrip():
    vnav = _vnav()
    sc = small_scenes()
    env = vnav.VectorEnv(sc, 257, seed=31, max_episode_steps=15)
    acts = [env.random_actions(t).clone() for t in range(40)]
    for t in range(10):
        env.step(acts[t])
    saved = env.get_state().clone()
    ret = env._info["ep_return"].clone()
    first = [env.step(acts[t], gather=False) for t in range(10, 40)]
    first = [(r.clone(), d.clone(), i["state"].clone()) for (_, r, d, i) in first]
    env.set_state(saved)
    for t in range(10, 40):
        _, r, d, i = env.step(acts[t], gather=False)
        r0, d0, s0 = first[t - 10]
        assert torch.equal(r, r0) and torch.equal(d, d0) and torch.equal(i["state"], s0)
    assert ret.shape[0] == 257


@pytest.mark.parametrize("mode,c", [(1, 0.05), (1, 0.3), (2, 0.1), (2, 0.6)])
def test_curriculum_matches_oracle(mode, c):
    vnav = _vnav()
    sc = small_scenes()
    arena = np.concatenate([s.observations for s in sc])
    n = 700
    env = vnav.VectorEnv(sc, n, seed=99, max_episode_steps=7)
    o = oracle_of(sc, n, 99, max_steps=7)
    env.set_complexity(c, mode=mode, offset=1.0)
    o.set_curriculum(c, mode, 1.0)
    env.reset()
    o.reset()
    rng = np.random.RandomState(7)
    for t in range(40):
        a = rng.randint(0, 4, size=n).astype(np.int32)
        compare_step(env.step(torch.as_tensor(a, device="cuda")), o.step(a), arena, (mode, c, t))


def test_curriculum_maze_distribution_matches_reference(golden):
    """SimpleGraphEnv's set_complexity (graph/env.py:101-106): starts ~ sample_initial_position
    (graph/util.py:88-117) with the 0.9/0.1 split; GPU frequencies vs the reference weights."""
    vnav = _vnav()
    m = golden("maze.npz")
    maze, goal = m["maze"], tuple(m["goal"].tolist())
    dist = m["distances"]
    scene = vnav.maze_scene(maze, goal)
    g = scene.goals[0]
    E = 4096
    env = vnav.VectorEnv([scene], E, seed=3, tasks=[(0, g)], max_episode_steps=0)
    c = 0.3
    env.set_complexity(c)
    counts = np.zeros(scene.n_states)
    for _ in range(12):
        env.reset()
        st = env.get_state()[1].cpu().numpy()
        counts += np.bincount(st, minlength=scene.n_states)
    # reference weights (graph/util.py:103-112) with opt = c*(largest-1)+1 (graph/env.py:105)
    opt = c * (dist.max() - 1) + 1
    d = np.array([dist[p + goal] for p in scene.locations])
    pos, neg = (d > 0) & (d <= opt), d > opt
    w = np.where(pos, 0.9 / pos.sum(), 0.0) + np.where(neg, 0.1 / neg.sum(), 0.0)
    expect = w * counts.sum()
    assert counts[w == 0].sum() == 0
    nz = w > 0
    chi2 = (((counts[nz] - expect[nz]) ** 2) / expect[nz]).sum()
    dof = nz.sum() - 1
    assert chi2 < dof + 6 * np.sqrt(2 * dof), (chi2, dof)
    # the reference's own sampler (oracle restatement pinned by goldens) agrees with w
    rng = np.random.RandomState(0)
    ref = np.zeros(scene.n_states)
    lookup = {p: i for i, p in enumerate(scene.locations)}
    for _ in range(4000):
        ref[lookup[oe.sample_initial_position(maze, dist, goal, opt, rng=rng)]] += 1
    chi2r = (((ref[nz] - w[nz] * 4000) ** 2) / (w[nz] * 4000)).sum()
    assert chi2r < dof + 6 * np.sqrt(2 * dof)


def test_maze_config_c1_16_envs(golden):
    """Config C1's shape (graph/maze_graph.py 8x8 maze, 16 parallel envs): 16 SimpleGraphEnv
    instances (graph/env.py:73-143) — each with its own start sequence drawn by the reference
    sampler sample_initial_position (graph/util.py:88-117, restated in oracle/envs.py and
    pinned to the reference's draws by test_oracle_goldens) and its own random actions —
    against one 16-env VectorEnv replaying those starts: reward bits, done, the emitted state
    and observation (render / 255) at every step of every env."""
    vnav = _vnav()
    m = golden("maze.npz")
    maze, goal = m["maze"], tuple(m["goal"].tolist())
    dist = m["distances"]
    scene = vnav.maze_scene(maze, goal)
    lookup = {p: i for i, p in enumerate(scene.locations)}
    g = scene.goals[0]
    E, T, L = 16, 400, 400
    starts = []
    for e in range(E):
        rs = np.random.RandomState(100 + e)
        starts.append([tuple(oe.sample_initial_position(maze, dist, goal, rng=rs)) for _ in range(L)])
    sched = np.array([[(lookup[s], g) for s in st] for st in starts], dtype=np.int32)
    env = vnav.VectorEnv([scene], E, seed=0, tasks=[(0, g)], max_episode_steps=0)
    env.set_schedule(sched)
    img, _ = env.reset()
    oracles = [oe.SimpleGraphEnvOracle(maze, goal) for _ in range(E)]
    nres = [0] * E
    obs = [o.reset(starts[e][0]) for e, o in enumerate(oracles)]
    assert np.array_equal(img.cpu().numpy().astype(np.float32) / 255.0, np.stack(obs))
    rng = np.random.RandomState(7)
    for t in range(T):
        a = rng.randint(0, 4, size=E)
        (img, _), reward, done, info = env.step(torch.as_tensor(a, dtype=torch.int32, device="cuda"))
        rb, dn = reward.cpu().numpy().view(np.uint32), done.cpu().numpy()
        ts, st = info["terminal_state"].cpu().numpy(), info["state"].cpu().numpy()
        frames = img.cpu().numpy().astype(np.float32) / 255.0
        for e in range(E):
            ob, r, d, inf = oracles[e].step(int(a[e]))
            assert rb[e] == np.float32(r).view(np.uint32), (t, e)
            assert bool(dn[e]) == d, (t, e)
            assert scene.locations[ts[e]] == tuple(inf["state"]), (t, e)
            assert np.array_equal(scene.observations[ts[e]].astype(np.float32) / 255.0, ob), (t, e)
            if d:  # baselines auto-reset: the next start of this env's sequence
                nres[e] += 1
                ob = oracles[e].reset(starts[e][nres[e]])
                assert st[e] == lookup[starts[e][nres[e]]], (t, e)
            assert np.array_equal(frames[e], ob), (t, e)
    assert sum(nres) >= E  # episodes finished and restarted on every env on average
