"""The UNREAL heads' restatement (oracle/policy.py pixel_control / reward_prediction) pinned
to the reference modules' goldens (tests/golden/unreal174.npz, models/goal.py:94-137 run by
tests/golden/gen_model_goldens.py): the weights regenerate from the seed, the outputs and
the gradients of the contracted losses match in fp32 (rtol 1e-5 of scale)."""
import numpy as np
import torch

from oracle.policy import (bighouse_pixel_control, bighouse_reward_prediction, pixel_control, reward_prediction,
                           seeded_bighouse_unreal_state, seeded_unreal_state)


def _close(a, b, rtol, what):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err <= rtol, "%s: max err %.3g of scale %.3g" % (what, err, scale)


def test_unreal_oracle_matches_reference_golden(golden):
    d = golden("unreal174.npz")
    sd = {k: torch.as_tensor(v).requires_grad_() for k, v in seeded_unreal_state((174, 174), int(d["seed"][0])).items()}
    B, T = d["h"].shape[:2]
    h = torch.as_tensor(d["h"]).reshape(B * T, 512).requires_grad_()
    q = pixel_control(sd, h)
    _close(q.detach().numpy(), d["q"].reshape(B * T, 4, 42, 42), 1e-5, "q")
    logits = reward_prediction(sd, torch.as_tensor(d["rp_features"]).requires_grad_())
    _close(logits.detach().numpy(), d["rp_logits"], 1e-5, "rp logits")
    feats = torch.as_tensor(d["rp_features"]).requires_grad_()
    logits = reward_prediction(sd, feats)
    ((q * torch.as_tensor(d["dq"]).reshape(q.shape)).sum() + (logits * torch.as_tensor(d["drp"])).sum()).backward()
    _close(h.grad.numpy(), d["dh"].reshape(B * T, 512), 1e-5, "dh")
    _close(feats.grad.numpy(), d["d_rp_features"], 1e-5, "d rp features")
    for name, p in sd.items():
        g = p.grad.numpy()
        if name == "pc_base.0.0.weight":
            g = g[::16]
        _close(g, d["g:" + name], 1e-5, name) if np.abs(d["g:" + name]).max() > 0 else \
            np.testing.assert_array_equal(g, 0.0, err_msg=name)
    # the action branch's gradient is exactly zero: (v + a) - mean_c(a) with one channel
    assert not np.any(d["g:pc_action.0.0.weight"]) and not np.any(d["g:pc_action.0.2.bias"])


def test_bighouse_unreal_oracle_matches_reference_golden(golden):
    """BigHouseModel's UNREAL heads (models/bignet.py:77-111; rp's in_features derived for 84x84)
    restated in oracle/policy.py vs the reference modules' golden (bighouse_unreal84.npz)."""
    d = golden("bighouse_unreal84.npz")
    sd = {k: torch.as_tensor(v).requires_grad_() for k, v in seeded_bighouse_unreal_state(int(d["seed"][0])).items()}
    B, T = d["h"].shape[:2]
    h = torch.as_tensor(d["h"]).reshape(B * T, 512).requires_grad_()
    q = bighouse_pixel_control(sd, h)
    _close(q.detach().numpy(), d["q"].reshape(B * T, 4, 20, 20), 1e-5, "q")
    feats = torch.as_tensor(d["rp_features"]).requires_grad_()
    logits = bighouse_reward_prediction(sd, feats)
    _close(logits.detach().numpy(), d["rp_logits"], 1e-5, "rp logits")
    ((q * torch.as_tensor(d["dq"]).reshape(q.shape)).sum() + (logits * torch.as_tensor(d["drp"])).sum()).backward()
    _close(h.grad.numpy(), d["dh"].reshape(B * T, 512), 1e-5, "dh")
    _close(feats.grad.numpy(), d["d_rp_features"], 1e-5, "d rp features")
    for name, p in sd.items():
        g = p.grad.numpy()
        if name == "pc_base.0.0.weight":
            g = g[::16]
        _close(g, d["g:" + name], 1e-5, name) if np.abs(d["g:" + name]).max() > 0 else \
            np.testing.assert_array_equal(g, 0.0, err_msg=name)
    assert not np.any(d["g:pc_action.0.0.weight"]) and not np.any(d["g:pc_action.0.0.bias"])
