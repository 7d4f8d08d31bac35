"""Generate policy golden vectors by running the REFERENCE model modules (models/goal.py).

Run ONLY in the build container:  python tests/golden/gen_model_goldens.py
(python3.10 + torch; deep_rl.model is replaced by the stand-ins under
tests/golden/stubs/deep_rl because deep-rl==0.2.9 is absent from the image).

Cases
  84x84  BigGoalHouseModel(3, 4) with conv_merge's Linear(9*9*32, 512) rebuilt as
         Linear(288, 512) (the 84x84 trunk ends at 3x3x32) and re-initialised with the
         reference's own init_weights; biases then perturbed so bias paths are exercised.
  174x174 the unmodified reference topology (Linear(2592, 512)).
  unreal174 the pixel-control and reward-prediction heads (goal.py:94-137) at 174x174.
  bighouse_unreal84 BigHouseModel's pixel-control and reward-prediction heads (bignet.py:77-111).
For each: weights (reference state-dict names), uint8 frame inputs, trunk features,
logits and value from the reference modules, and the gradients of the engine's A2C
loss (oracle/a2c.py, parity unpinned at the trainer level) through the reference
modules by torch autograd.
"""
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(HERE, "stubs"), "/root/reference", REPO]

from models.goal import AuxiliaryBigGoalHouseModel, BigGoalHouseModel  # noqa: E402  (the reference modules)
from models.bignet import BigHouseModel  # noqa: E402

from oracle import a2c  # noqa: E402


def build(frame, seed):
    torch.manual_seed(seed)
    model = BigGoalHouseModel(3, 4)
    if frame != 174:
        o = (frame - 7) // 4 + 1
        o = (o - 4) // 2 + 1
        o = (o - 4) // 2 + 1
        lin = nn.Linear(32 * o * o, 512)
        model.init_weights(lin)
        model.conv_merge[0][1] = lin
    g = torch.Generator().manual_seed(seed + 1)
    for name, p in model.named_parameters():
        if name.endswith("bias"):
            p.data.uniform_(-0.05, 0.05, generator=g)
    return model


def reference_forward(model, image_u8, goal_u8):
    """models/goal.py:83-90 up to conv_merge, then the two heads (goal.py:79-80) on the
    pre-LSTM features. Inputs uint8 [B,T,H,W,3] -> float [B,T,3,H,W] / 255."""
    img = image_u8.permute(0, 1, 4, 2, 3).float() / 255.0
    gl = goal_u8.permute(0, 1, 4, 2, 3).float() / 255.0
    a, b = model.shared_base(img), model.shared_base(gl)
    feats = model.conv_merge(model.conv_base(torch.cat((a, b), 2)))
    return feats, model.policy_logits(feats), model.critic(feats)


USED = ("shared_base", "conv_base", "conv_merge", "policy_logits", "critic")


def seeded_weights(model, seed, used=USED):
    """Deterministic weights from numpy's PCG64 (stable across versions) in the reference's
    init distribution U(-1/sqrt(fan_in), 1/sqrt(fan_in)); lets a large case be regenerated
    from its seed instead of being stored."""
    rng = np.random.default_rng(seed)
    for name, p in model.named_parameters():
        if name.split(".")[0] not in used:
            continue
        if name.endswith("bias"):
            v = rng.uniform(-0.05, 0.05, size=p.shape)
        else:
            fan_in = int(np.prod(p.shape[1:]))
            d = 1.0 / np.sqrt(fan_in)
            v = rng.uniform(-d, d, size=p.shape)
        p.data.copy_(torch.as_tensor(v.astype(np.float32)))


def case(frame, B, T, seed, store_weights=True):
    model = build(frame, seed)
    if not store_weights:
        seeded_weights(model, seed)
    rng = np.random.RandomState(seed)
    image = torch.as_tensor(rng.randint(0, 256, size=(B, T, frame, frame, 3)).astype(np.uint8))
    goal = torch.as_tensor(rng.randint(0, 256, size=(B, T, frame, frame, 3)).astype(np.uint8))
    feats, logits, value = reference_forward(model, image, goal)
    N = B * T
    actions = torch.as_tensor(rng.randint(0, 4, size=N))
    rets = torch.as_tensor(rng.randn(N).astype(np.float32))
    loss, _ = a2c.loss(logits.reshape(N, 4), value.reshape(N), actions, rets)
    model.zero_grad()
    loss.backward()
    out = {"image": image.numpy(), "goal": goal.numpy(), "features": feats.detach().numpy(),
           "logits": logits.detach().numpy(), "value": value.detach().numpy(),
           "actions": actions.numpy().astype(np.int32), "returns": rets.numpy(),
           "loss": np.array([loss.item()], dtype=np.float32)}
    out["seed"] = np.array([seed])
    if store_weights:
        for name, p in model.named_parameters():
            if name.split(".")[0] in USED:
                out["w:" + name] = p.detach().numpy()
                out["g:" + name] = p.grad.numpy()
    return out


AUX = ("deconv_depth", "deconv_mask", "deconv_mask_goal")


def aux_case(frame, B, T, seed):
    """AuxiliaryBigGoalHouseModel.forward_deconv (models/goal.py:177-189) at 174x174 (the
    reference topology: Unflatten(32, 9, 9)), weights from the seed (PCG64, trunk + deconv
    heads). Stores the inputs, the three head outputs and, for the summed per-head MSE
    against stored random targets (the _deconv_loss form, ai2_auxiliary/trainer.py:45-55),
    the gradients of the deconv parameters and of the conv_base features."""
    torch.manual_seed(seed)
    model = AuxiliaryBigGoalHouseModel(3, 4)
    seeded_weights(model, seed, USED + AUX)
    rng = np.random.RandomState(seed)
    image = torch.as_tensor(rng.randint(0, 256, size=(B, T, frame, frame, 3)).astype(np.uint8))
    goal = torch.as_tensor(rng.randint(0, 256, size=(B, T, frame, frame, 3)).astype(np.uint8))
    img = image.permute(0, 1, 4, 2, 3).float() / 255.0
    gl = goal.permute(0, 1, 4, 2, 3).float() / 255.0
    a, b = model.shared_base(img), model.shared_base(gl)
    feats = model.conv_base(torch.cat((a, b), 2))
    feats.retain_grad()
    preds = (model.deconv_depth(feats), model.deconv_mask(feats), model.deconv_mask_goal(feats))
    # forward_deconv itself must agree with the staged computation above
    with torch.no_grad():
        ref_preds, _ = model.forward_deconv(((img, gl), None), None, None)
    for p, q in zip(preds, ref_preds):
        assert torch.equal(p, q)
    targets = [torch.as_tensor(rng.rand(*p.shape).astype(np.float32)) for p in preds]
    loss = sum(nn.functional.mse_loss(p, t) for p, t in zip(preds, targets))
    model.zero_grad()
    loss.backward()
    out = {"image": image.numpy(), "goal": goal.numpy(), "seed": np.array([seed]),
           "features": feats.detach().numpy(), "d_features": feats.grad.numpy(),
           "loss": np.array([loss.item()], dtype=np.float32)}
    for k, (p, t) in enumerate(zip(preds, targets)):
        out["pred%d" % k] = p.detach().numpy()
        out["target%d" % k] = t.numpy()
    for name, p in model.named_parameters():
        if name.split(".")[0] in AUX:
            out["g:" + name] = p.grad.numpy()
    return out


BIG_USED = ("conv_base", "conv_merge", "policy_logits", "critic")


def bighouse_case(B, T, seed):
    """BigHouseModel (models/bignet.py:26-75, unmodified: its Linear(7*7*32) fits 84x84):
    conv_base + conv_merge features and the heads on them (the LSTM's MaskedRNN semantics are
    unpinned), weights from the seed (PCG64). Stores the inputs, features, logits, value and
    the engine's A2C loss gradients of the conv and head parameters."""
    torch.manual_seed(seed)
    model = BigHouseModel(3, 4)
    seeded_weights(model, seed, BIG_USED)
    rng = np.random.RandomState(seed)
    image = torch.as_tensor(rng.randint(0, 256, size=(B, T, 84, 84, 3)).astype(np.uint8))
    img = (image.permute(0, 1, 4, 2, 3).float() / 255.0).contiguous()
    feats = model.conv_merge(model.conv_base(img))
    logits, value = model.policy_logits(feats), model.critic(feats)
    N = B * T
    actions = torch.as_tensor(rng.randint(0, 4, size=N))
    rets = torch.as_tensor(rng.randn(N).astype(np.float32))
    loss, _ = a2c.loss(logits.reshape(N, 4), value.reshape(N), actions, rets)
    model.zero_grad()
    loss.backward()
    out = {"image": image.numpy(), "features": feats.detach().numpy(), "logits": logits.detach().numpy(),
           "value": value.detach().numpy(), "actions": actions.numpy().astype(np.int32), "returns": rets.numpy(),
           "loss": np.array([loss.item()], dtype=np.float32), "seed": np.array([seed])}
    for name, p in model.named_parameters():
        if name.split(".")[0] in ("conv_base", "policy_logits", "critic"):
            out["g:" + name] = p.grad.numpy()
    return out


UNREAL = ("pc_base", "pc_action", "pc_value", "rp")


def unreal_case(B, T, R, seed):
    """BigGoalHouseModel's UNREAL heads (models/goal.py:94-137) at 174x174, the reference
    topology (pc_base 512 -> 32x9x9, rp Linear(9*9*32*3, 3)). Weights from the seed (PCG64,
    the four modules only, named_parameters order; the trunk from seed + 1, used only to make
    the rp inputs). pixel_control runs on stored LSTM features h [B,T,512] (its _forward_base is
    replaced by one returning h: MaskedRNN's semantics are absent) and reward_prediction on R
    samples of 3 frames; both losses are sums against stored random weights (dq, drp), so the
    stored gradients are those of the heads' outputs contracted with them."""
    torch.manual_seed(seed)
    model = BigGoalHouseModel(3, 4)
    seeded_weights(model, seed, UNREAL)
    seeded_weights(model, seed + 1, ("shared_base", "conv_base"))
    rng = np.random.RandomState(seed)
    h = torch.as_tensor((rng.rand(B, T, 512) * 2.0 - 0.5).astype(np.float32)).requires_grad_()
    f = model.pc_base(h).view(B, T, 32, 9, 9)
    a = model.pc_action(f)
    q = model.pc_value(f) + a - a.mean(2, keepdim=True)
    model._forward_base = lambda inputs, masks, states: (h, None)
    with torch.no_grad():
        q_ref, _ = model.pixel_control(None, None, None)
    assert torch.equal(q, q_ref)
    dq = torch.as_tensor(rng.randn(*q.shape).astype(np.float32))
    image = torch.as_tensor(rng.randint(0, 256, size=(R, 3, 174, 174, 3)).astype(np.uint8))
    goal = torch.as_tensor(rng.randint(0, 256, size=(R, 3, 174, 174, 3)).astype(np.uint8))
    img = image.permute(0, 1, 4, 2, 3).float() / 255.0
    gl = goal.permute(0, 1, 4, 2, 3).float() / 255.0
    feats = model.conv_base(torch.cat((model.shared_base(img), model.shared_base(gl)), 2)).detach().requires_grad_()
    logits = model.rp(feats)
    with torch.no_grad():
        assert torch.equal(logits, model.reward_prediction(((img, gl), None)))
    drp = torch.as_tensor(rng.randn(R, 3).astype(np.float32))
    model.zero_grad()
    ((q * dq).sum() + (logits * drp).sum()).backward()
    out = {"seed": np.array([seed]), "h": h.detach().numpy(), "q": q.detach().numpy(), "dq": dq.numpy(),
           "dh": h.grad.numpy(), "rp_features": feats.detach().numpy(), "rp_logits": logits.detach().numpy(),
           "drp": drp.numpy(), "d_rp_features": feats.grad.numpy()}
    for name, p in model.named_parameters():
        if name.split(".")[0] in UNREAL:
            out["g:" + name] = p.grad.numpy()
    out["g:pc_base.0.0.weight"] = out["g:pc_base.0.0.weight"][::16].copy()  # every 16th row (size)
    return out


BIG_UNREAL = ("pc_base", "pc_action", "pc_value", "rp")


def bighouse_unreal_case(B, T, R, seed):
    """BigHouseModel's UNREAL heads (models/bignet.py:77-111) at 84x84: pixel control (pc_base
    Linear(512, 32*9*9) + ReLU, pc_action / pc_value one ConvTranspose2d(32, 1 / A, 4, 2) + ReLU
    each, value + action - mean(action)) on stored LSTM features h [B,T,512] (_forward_base
    replaced, as in unreal_case), and reward prediction on R samples of 3 frames. bignet.py's rp is
    Linear(9*9*32*3, 3), which fits only 100x100 inputs (conv_base ends at 9x9 there, at 7x7 for
    84x84 frames: view(R, -1) gives 3*7*7*32 = 4704): rebuilt as Linear(4704, 3) and re-initialised
    with the reference's own init_weights (the derived-in_features deviation of the 84x84 goal
    net's conv_merge). Weights from the seed (PCG64) over the four modules, conv_base from seed + 1."""
    torch.manual_seed(seed)
    model = BigHouseModel(3, 4)
    model.rp = nn.Linear(3 * 7 * 7 * 32, 3)
    model.init_weights(model.rp)
    seeded_weights(model, seed, BIG_UNREAL)
    seeded_weights(model, seed + 1, ("conv_base",))
    rng = np.random.RandomState(seed)
    h = torch.as_tensor((rng.rand(B, T, 512) * 2.0 - 0.5).astype(np.float32)).requires_grad_()
    f = model.pc_base(h).view(B, T, 32, 9, 9)
    a = model.pc_action(f)
    q = model.pc_value(f) + a - a.mean(2, keepdim=True)
    model._forward_base = lambda inputs, masks, states: (h, None)
    with torch.no_grad():
        q_ref, _ = model.pixel_control(None, None, None)
    assert torch.equal(q, q_ref)
    dq = torch.as_tensor(rng.randn(*q.shape).astype(np.float32))
    image = torch.as_tensor(rng.randint(0, 256, size=(R, 3, 84, 84, 3)).astype(np.uint8))
    img = (image.permute(0, 1, 4, 2, 3).float() / 255.0).contiguous()  # TransposeImage's arrays
    feats = model.conv_base(img).detach().requires_grad_()
    logits = model.rp(feats.view(R, -1))
    with torch.no_grad():
        assert torch.equal(logits, model.reward_prediction((img, None)))
    drp = torch.as_tensor(rng.randn(R, 3).astype(np.float32))
    model.zero_grad()
    ((q * dq).sum() + (logits * drp).sum()).backward()
    out = {"seed": np.array([seed]), "h": h.detach().numpy(), "q": q.detach().numpy(), "dq": dq.numpy(),
           "dh": h.grad.numpy(), "image": image.numpy(), "rp_features": feats.detach().numpy(),
           "rp_logits": logits.detach().numpy(), "drp": drp.numpy(), "d_rp_features": feats.grad.numpy()}
    for name, p in model.named_parameters():
        if name.split(".")[0] in BIG_UNREAL:
            out["g:" + name] = p.grad.numpy()
    out["g:pc_base.0.0.weight"] = out["g:pc_base.0.0.weight"][::16].copy()  # every 16th row (size)
    return out


def main():
    np.savez_compressed(os.path.join(HERE, "policy84.npz"), **case(84, 3, 2, 11))
    np.savez_compressed(os.path.join(HERE, "policy174.npz"), **case(174, 2, 1, 12, store_weights=False))
    np.savez_compressed(os.path.join(HERE, "aux174.npz"), **aux_case(174, 2, 1, 13))
    np.savez_compressed(os.path.join(HERE, "bighouse84.npz"), **bighouse_case(2, 2, 14))
    np.savez_compressed(os.path.join(HERE, "unreal174.npz"), **unreal_case(2, 3, 3, 15))
    np.savez_compressed(os.path.join(HERE, "bighouse_unreal84.npz"), **bighouse_unreal_case(2, 3, 3, 16))
    n_params = sum(p.numel() for n, p in build(84, 0).named_parameters() if n.split(".")[0] in USED)
    print("84x84 trunk+heads parameters:", n_params)


if __name__ == "__main__":
    main()
