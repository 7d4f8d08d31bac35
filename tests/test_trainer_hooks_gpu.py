"""deep_rl trainer hooks on A2CTrainer: ``sample_training_batch()`` and
``compute_auxiliary_loss(model, batch, device)`` (experiments/ai2_auxiliary/trainer.py:27-43),
and the replay-sequence source of the aux batch (trainer.py:29, ``self.replay.sample_sequence()``)."""
import numpy as np
import pytest
import torch

from test_aux_gpu import _aux_scene

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / max(float(b.abs().max()), 1e-30))


def _make(cls, recurrent=False, **kw):
    import vnav
    sc = [vnav.synthetic_scene(k) for k in range(2)]
    env = vnav.VectorEnv(sc, 16, seed=4, max_episode_steps=10)
    return cls(env, num_steps=5, seed=2, max_time_steps=1e6, recurrent=recurrent, **kw)


def test_sample_training_batch_then_update_equals_step():
    """step() == sample_training_batch() + update(batch), bit for bit (the default hooks)."""
    import vnav
    a = _make(vnav.A2CTrainer)
    b = _make(vnav.A2CTrainer)
    for _ in range(3):
        a.step(sync=True)
        batch, report = b.sample_training_batch()
        assert set(report) == {"episode_stats"} and batch["actions"].shape == (5, 16)
        b.update(batch)
    assert torch.equal(a.params, b.params) and torch.equal(a.square_avg, b.square_avg)


@pytest.mark.parametrize("recurrent", [False, True])
def test_compute_auxiliary_loss_override_adds_its_gradient(recurrent):
    """A subclass's extra loss <v, params> adds exactly v to the update's gradient; the model
    it receives aliases the trainer's parameters (its forward on the batch's gathered frames
    reproduces the rollout's logits and values for the feed-forward net)."""
    import vnav
    seen = {}

    class Extra(vnav.A2CTrainer):
        def compute_auxiliary_loss(self, model, batch, device):
            assert model.params.data_ptr() == self.params.data_ptr()
            img, goal = batch.observations()
            assert img.shape == (16, 5, 84, 84, 3)
            if not self.recurrent:
                with torch.no_grad():
                    logits, value, _ = model(((img, goal), None))
                seen["logits"] = logits.transpose(0, 1).reshape(-1, 4)
                seen["value"] = value.transpose(0, 1).reshape(-1)
            g = torch.Generator(device="cpu").manual_seed(11)
            self.v = (torch.randn(self.params.numel(), generator=g) * 1e-3).to(device)
            return (model.params * self.v).sum(), {"extra": 1.0}

    base = _make(vnav.A2CTrainer, recurrent)
    ext = _make(Extra, recurrent)
    base.step(sync=True)
    ext.step(sync=True)
    assert ext.aux_losses == {"extra": 1.0}
    diff = ext.grads - base.grads
    scale = float(base.grads.abs().max())
    assert float((diff - ext.v).abs().max()) <= 1e-6 * scale + 1e-9
    assert not torch.equal(ext.params, base.params)
    if not recurrent:  # the rollout's own outputs of the same parameters (before the update)
        assert _rel(seen["logits"], base.out[:, :4]) <= 1e-6
        assert _rel(seen["value"], base.out[:, 4]) <= 1e-6


def test_replay_aux_source():
    """aux_source='replay': the aux loss runs on a sequence drawn from the last rollouts with
    its own trunk forward/backward. With a one-rollout replay the sequence IS the on-policy
    batch, so the gradient equals the fused on-policy path's up to summation order; with a
    longer replay the aux loss still falls as the heads fit."""
    import vnav

    def make(src, size=8, n=64):
        env = vnav.VectorEnv([_aux_scene(0)], n, seed=2, max_episode_steps=50)
        return vnav.A2CTrainer(env, num_steps=5, seed=1, max_time_steps=1e9, aux_weight=0.1, recurrent=True,
                               learning_rate=2e-3, aux_source=src, replay_size=size)

    a, b = make("rollout"), make("replay", size=1)
    a.step(sync=True)
    b.step(sync=True)
    assert _rel(b.grads, a.grads) <= 1e-4
    tr = make("replay", n=256)
    first = tr.step(sync=True)
    for _ in range(30):
        tr.step(sync=False)
    last = tr.step(sync=True)
    assert tr.replay_filled == 8
    assert np.isfinite(last["aux_loss"]) and last["aux_loss"] < 0.8 * first["aux_loss"]
    assert tr.env.error_flags() == 0


def test_graph_recaptured_after_env_reconfiguration():
    """cuda_graph=True: reconfiguring the env after capture (here the episode limit) makes
    the next update capture again, so the replayed graph uses the new configuration — the
    run stays bit-identical to eager updates with the same reconfiguration."""
    import vnav

    def run(graph):
        tr = _make(vnav.A2CTrainer, cuda_graph=graph)
        ms = []
        for u in range(6):
            if u == 3:
                tr.env.set_max_episode_steps(3)
            ms.append(tr.step(sync=False)["raw"])
        return tr.params.detach().clone(), tr.env.get_state().cpu(), torch.stack(ms).cpu()

    pe, ee, me = run(False)
    pg, eg, mg = run(True)
    assert torch.equal(pe, pg) and torch.equal(ee, eg)
    assert torch.equal(me.nan_to_num(-1), mg.nan_to_num(-1))  # raw metrics are copies per update


def test_checkpoint_refuses_other_env_count():
    import vnav
    a = _make(vnav.A2CTrainer)
    a.step(sync=True)
    sd = a.state_dict()
    env = vnav.VectorEnv([vnav.synthetic_scene(0)], 8, seed=4)
    b = vnav.A2CTrainer(env, num_steps=5, seed=2, max_time_steps=1e6)
    with pytest.raises(ValueError):
        b.load_state_dict(sd)
    with pytest.raises(ValueError):
        env.set_state(sd["env_state"])
    with pytest.raises(ValueError):
        env.set_episode_returns(sd["env_ep_return"])


def test_evaluate_leaves_the_schedule():
    """evaluate() restores the device schedule (sampling counter and step count), so the
    training run after it continues as if it had not been evaluated."""
    import vnav
    a, b = _make(vnav.A2CTrainer), _make(vnav.A2CTrainer)
    a.step(sync=True)
    b.step(sync=True)
    s0 = b.sched.clone()
    b.evaluate(episodes=1, max_rollouts=2)
    assert torch.equal(b.sched, s0)
