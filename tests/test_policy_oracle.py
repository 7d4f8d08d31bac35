"""The torch-CPU policy/A2C oracle vs the reference modules' goldens. CPU only."""
import numpy as np
import torch

from oracle import a2c
from oracle.policy import GoalNetOracle, frames_to_float, seeded_reference_state


def _ref_state(d):
    return {k[2:]: d[k] for k in d.files if k.startswith("w:")}


def test_policy84_forward_and_grads(golden):
    d = golden("policy84.npz")
    net = GoalNetOracle((84, 84)).load_reference(_ref_state(d))
    img = frames_to_float(d["image"].reshape(-1, 84, 84, 3))
    goal = frames_to_float(d["goal"].reshape(-1, 84, 84, 3))
    feats = net.features(img, goal)
    logits, value = net(img, goal)
    np.testing.assert_allclose(feats.detach().numpy(), d["features"].reshape(-1, 512), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(logits.detach().numpy(), d["logits"].reshape(-1, 4), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(value.detach().numpy(), d["value"].reshape(-1, 1), rtol=1e-6, atol=1e-6)
    loss, _ = a2c.loss(logits, value.view(-1), torch.as_tensor(d["actions"]).long(), torch.as_tensor(d["returns"]))
    np.testing.assert_allclose(loss.item(), d["loss"][0], rtol=1e-6)
    loss.backward()
    names = {"shared_base.0.0": net.conv1, "shared_base.0.2": net.conv2, "conv_base.0.0": net.conv3,
             "conv_base.0.2": net.conv4, "conv_merge.0.1": net.fc, "policy_logits.0": net.policy_logits,
             "critic.0": net.critic}
    for k, mod in names.items():
        np.testing.assert_allclose(mod.weight.grad.numpy(), d["g:" + k + ".weight"], rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(mod.bias.grad.numpy(), d["g:" + k + ".bias"], rtol=1e-5, atol=1e-7)


def test_policy174_reference_topology(golden):
    d = golden("policy174.npz")
    net = GoalNetOracle((174, 174)).load_reference(seeded_reference_state((174, 174), int(d["seed"][0])))
    img = frames_to_float(d["image"].reshape(-1, 174, 174, 3))
    goal = frames_to_float(d["goal"].reshape(-1, 174, 174, 3))
    logits, value = net(img, goal)
    np.testing.assert_allclose(logits.detach().numpy(), d["logits"].reshape(-1, 4), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(value.detach().numpy(), d["value"].reshape(-1, 1), rtol=1e-5, atol=1e-6)


def test_returns_recursion():
    r = torch.tensor([[1.0, 0.0], [0.0, 1.0], [0.5, 0.0]])
    d = torch.tensor([[0, 0], [1, 0], [0, 0]])
    v = torch.tensor([[0.0, 0.0], [0.0, 0.0], [0.0, 0.0], [2.0, 3.0]])
    R = a2c.returns(r, d, v, 0.9)
    # env 0: t2 = .5 + .9*2 = 2.3; t1 = 0 (done); t0 = 1 + .9*0 = 1
    np.testing.assert_allclose(R[:, 0].numpy(), [1.0, 0.0, 2.3], rtol=1e-6)
    np.testing.assert_allclose(R[:, 1].numpy(), [0.9 * (1 + 0.9 * 2.7), 1 + 0.9 * 2.7, 2.7], rtol=1e-6)
