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


def test_recurrent_oracle_mask_semantics():
    """RecurrentGoalNetOracle: masks of ones = nn.LSTM over the whole sequence; a zero mask
    at step t = restarting the LSTM from zero state at t."""
    from oracle.policy import RecurrentGoalNetOracle
    torch.manual_seed(0)
    net = RecurrentGoalNetOracle((84, 84))
    B, T, A = 2, 5, 4
    img = torch.rand(B, T, 3, 84, 84)
    gl = torch.rand(B, T, 3, 84, 84)
    lra = torch.randn(B, T, A + 1)
    h0, c0 = torch.randn(B, 1, 512), torch.randn(B, 1, 512)
    with torch.no_grad():
        x = torch.cat((net.features(img.flatten(0, 1), gl.flatten(0, 1)).view(B, T, 512), lra), 2)
        y, (h, c) = net.lstm(x, (h0.transpose(0, 1), c0.transpose(0, 1)))
        l1, v1, (h1, c1) = net.forward_seq(img, gl, lra, torch.ones(B, T), (h0, c0))
        np.testing.assert_allclose(l1.numpy(), net.policy_logits(y).numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(h1.numpy(), h.transpose(0, 1).numpy(), rtol=1e-5, atol=1e-6)
        m = torch.ones(B, T)
        m[:, 2] = 0
        l2, _, _ = net.forward_seq(img, gl, lra, m, (h0, c0))
        y2, _ = net.lstm(x[:, 2:])
        np.testing.assert_allclose(l2[:, 2:].numpy(), net.policy_logits(y2).numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(l2[:, :2].numpy(), l1[:, :2].numpy(), rtol=1e-6, atol=1e-7)
