"""A2CTrainer: a full update on the GPU vs the same update restated on the CPU oracle
(torch fp32 model + oracle A2C) from the rollout the GPU produced, and checkpoint/resume."""
import numpy as np
import pytest
import torch

from oracle import a2c as oa2c
from oracle.frames import synth_frames
from oracle.policy import GoalNetOracle, frames_to_float

pytestmark = pytest.mark.gpu


def test_update_matches_cpu_oracle():
    import vnav
    sc = [vnav.synthetic_scene(k) for k in range(2)]
    for s in sc:  # host copies of the frames so the oracle can gather them
        s.observations = synth_frames(s.synth_id, np.arange(s.n_states), s.frame_shape)
    env = vnav.VectorEnv(sc, 12, seed=21, max_episode_steps=6)
    tr = vnav.A2CTrainer(env, num_steps=5, seed=3, max_time_steps=1e6)
    # compare the SECOND update: its RMSprop step divides by the square_avg carried from the
    # first, so the step size depends on the gradient's magnitude (the first step from
    # square_avg = 0 is ~10*lr*sign(g) and would only check signs)
    tr.step(sync=True)
    p0 = tr.params.detach().clone()
    sq0 = tr.square_avg.detach().clone()
    assert sq0.abs().max().item() > 0
    tr.rollout()
    rows_img = tr.rows_img.cpu().numpy()
    rows_goal = tr.rows_goal.cpu().numpy()
    actions = tr.actions.cpu().long()
    rewards = tr.rewards.cpu()
    dones = tr.dones.cpu()
    boot_rows = (env._info["img_row"].cpu().numpy(), env._info["goal_row"].cpu().numpy())
    out_gpu = tr.out.cpu()
    lr = tr.current_lr()
    tr.update()
    torch.cuda.synchronize()

    arena = np.concatenate([s.observations for s in sc])
    ref = GoalNetOracle((84, 84)).load_reference(tr.net.to_reference(p0))
    img = frames_to_float(arena[rows_img])
    gl = frames_to_float(arena[rows_goal])
    logits, value = ref(img, gl)
    np.testing.assert_allclose(logits.detach().numpy(), out_gpu[:, :4].numpy(), rtol=1e-4, atol=1e-5)
    with torch.no_grad():
        _, bv = ref(frames_to_float(arena[boot_rows[0]]), frames_to_float(arena[boot_rows[1]]))
    T, E = 5, 12
    vext = torch.cat([value.detach().view(T, E), bv.view(1, E)])
    R = oa2c.returns(rewards, dones, vext, 0.99)
    loss, _ = oa2c.loss(logits, value.view(-1), actions, R.view(-1))
    loss.backward()
    params = [m.weight for m in (ref.conv1, ref.conv2, ref.conv3, ref.conv4, ref.fc, ref.policy_logits, ref.critic)]
    params += [m.bias for m in (ref.conv1, ref.conv2, ref.conv3, ref.conv4, ref.fc, ref.policy_logits, ref.critic)]
    grads = [p.grad.clone() for p in params]
    names = ["shared_base.0.0", "shared_base.0.2", "conv_base.0.0", "conv_base.0.2", "conv_merge.0.1",
             "policy_logits.0", "critic.0"]
    keys = [n + ".weight" for n in names] + [n + ".bias" for n in names]
    sq_old = tr.net.to_reference(sq0)
    sq = [sq_old[k].clone().view_as(p) for k, p in zip(keys, params)]
    with torch.no_grad():
        oa2c.clip_and_rmsprop([p.data for p in params], grads, sq, lr)
    new = tr.net.to_reference(tr.params)
    old = tr.net.to_reference(p0)
    for k, p, p_old in zip(keys, params, [old[k].view_as(q) for k, q in zip(keys, params)]):
        step_ref = (p.data - p_old)
        step_gpu = (new[k].view_as(p) - p_old)
        scale = step_ref.abs().max().item()
        assert (step_gpu - step_ref).abs().max().item() <= 2e-3 * scale + 1e-9, k


def test_trainer_learns_on_small_scene():
    """Learning check on one tiny scene with a fixed goal (the reference experiment trains a
    fixed (scene, goal) task, experiments/thor_cached_auxiliary.py:73-84): the mean episode
    length after 250 updates is well below the random-policy level of the first updates
    (the very first rollout is skipped: only short episodes can finish inside it)."""
    import vnav
    maze = np.ones((3, 3), dtype=bool)
    from oracle.graph import h5_tables
    graph, spd, _ = h5_tables(maze)
    frames = synth_frames(3, np.arange(len(graph)), (84, 84, 3))
    scene = vnav.scene_from_arrays(graph, spd, frames)
    env = vnav.VectorEnv([scene], 256, seed=1, max_episode_steps=60, tasks=[(0, 5)])
    tr = vnav.A2CTrainer(env, num_steps=20, seed=0, max_time_steps=1e9)
    lengths = []
    for u in range(250):
        m = tr.step(sync=(u < 20 or u >= 240))
        if "raw" not in m:
            lengths.append(m["episode_length"])
    early = np.nanmean(lengths[5:20])
    late = np.nanmean(lengths[-10:])
    assert np.isfinite(late) and late < 0.8 * early, (early, late)


@pytest.mark.parametrize("recurrent", [False, True])
def test_checkpoint_resume_is_exact(recurrent):
    """state_dict after K updates, restored into a fresh env + trainer, continues exactly as
    the uninterrupted run: parameters, optimiser state and the logged metrics (episode
    count / return / length, which need the running per-env returns) match bit for bit."""
    import dataclasses
    import vnav
    # a step penalty and a collision penalty, so the running returns of in-flight episodes
    # are non-zero (with the cached reward table (1, -0, 0) they are 0 until the goal)
    sc = [dataclasses.replace(vnav.synthetic_scene(k), rewards=(1.0, -0.01, -0.1)) for k in range(2)]

    def make():
        env = vnav.VectorEnv(sc, 64, seed=5, max_episode_steps=12)
        return vnav.A2CTrainer(env, num_steps=5, seed=9, max_time_steps=1e6, recurrent=recurrent)

    keys = ("value_loss", "action_loss", "entropy", "episodes", "reward", "episode_length", "grad_norm")
    a = make()
    for _ in range(3):
        a.step(sync=True)
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in a.state_dict().items()}
    assert sd["env_ep_return"].abs().sum().item() > 0  # some episodes are in flight with reward
    ma = [a.step(sync=True) for _ in range(3)]
    pa, sqa = a.params.detach().cpu(), a.square_avg.cpu()
    del a
    b = make()
    b.load_state_dict(sd)
    mb = [b.step(sync=True) for _ in range(3)]
    assert torch.equal(pa, b.params.detach().cpu())
    assert torch.equal(sqa, b.square_avg.cpu())
    for x, y in zip(ma, mb):
        for k in keys:
            assert (x[k] == y[k]) or (np.isnan(x[k]) and np.isnan(y[k])), (k, x[k], y[k])


@pytest.mark.parametrize("recurrent", [False, True])
def test_cuda_graph_updates_are_bit_identical(recurrent):
    """A2CTrainer(cuda_graph=True) — the update captured once in a hipGraph and replayed —
    gives bit-identical parameters, optimiser state, env state and metrics to the eager
    updates, with a learning rate that changes every update (device-side schedule)."""
    import vnav
    sc = [vnav.synthetic_scene(k) for k in range(2)]

    def run(graph):
        env = vnav.VectorEnv(sc, 8, seed=5, max_episode_steps=12)
        tr = vnav.A2CTrainer(env, num_steps=5, seed=9, max_time_steps=400, recurrent=recurrent, cuda_graph=graph)
        ms = [tr.step(sync=True) for _ in range(6)]
        return (tr.params.detach().cpu(), tr.square_avg.cpu(), env.get_state().cpu(), ms, tr.lr_dev.cpu(),
                tr.current_lr())

    pe, se, ee, me, lre, lr_host = run(False)
    pg, sg, eg, mg, lrg, _ = run(True)
    assert torch.equal(pe, pg) and torch.equal(se, sg) and torch.equal(ee, eg)
    assert torch.equal(lre, lrg)
    # the device schedule's lr of the last update is the host LinearSchedule's value before it
    assert float(lre[0]) == float(np.float32(7e-4 * (1.0 - min(5 * 8 * 5 / 400.0, 1.0))))
    keys = ("value_loss", "action_loss", "entropy", "episodes", "reward", "episode_length", "grad_norm")
    for x, y in zip(me, mg):
        for k in keys:
            assert (x[k] == y[k]) or (np.isnan(x[k]) and np.isnan(y[k])), (k, x[k], y[k])
