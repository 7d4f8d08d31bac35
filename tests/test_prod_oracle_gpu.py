"""Production-size kernel paths against the fp64 oracle, directly.

The training update runs its batches through kernels that small test batches never reach:
persistent conv kernels that wrap their grids (conv1 banded forward / weight gradient,
the x6 conv2 / conv3 weight gradients with the two-stage slab reduce, the parity-class
input gradients, the conv2 input gradient), products with enough tiles to skip split-K
(>= 128 tiles: the conv_merge / head / LSTM products at >= 4096 rows) and the LSTM at
thousands of envs. These tests run those paths at batch sizes that take them — 84x84 with
4096 samples, 174x174 with 512 samples through the scene-cache row gather plus the aux
heads' fused loss, the LSTM core at 1024 envs — and compare every output and parameter
gradient with oracle/policy.py evaluated in float64 on the CPU.

ReLU ties: a pre-activation within fp32 rounding of zero can take the other side of its
ReLU on the GPU, and its channel's weight gradient then moves by ~1e-3 of the scale (a
tie, not an error). Instead of shrinking the batch until no tie occurs, the oracle is run
with the GPU forward's own ReLU masks (GoalNetOracle.forward_masked), read from the
activation store the kernels wrote; every mask bit that disagrees with the sign of the
oracle's own pre-activation is asserted to be a tie (|z| <= 1e-5 of the layer's scale).

Tolerances (north star): outputs 1e-5, parameter gradients 1e-4 of each tensor's scale.
Logits and values are also checked element by element: |gpu - fp64| <= 1e-5 |fp64| + a floor
of 1e-6 of the tensor's scale (a logit near zero is a sum of cancelling terms whose fp32
rounding is set by the terms, not by the sum: the floor states that absolute bound).
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import a2c as oa2c
from oracle.policy import (AuxHeadsOracle, GoalNetOracle, aux_targets, frames_to_float, trunk_sizes)

pytestmark = pytest.mark.gpu

NAMES = {"shared_base.0.0": "conv1", "shared_base.0.2": "conv2", "conv_base.0.0": "conv3",
         "conv_base.0.2": "conv4", "conv_merge.0.1": "fc", "policy_logits.0": "policy_logits",
         "critic.0": "critic"}
AUX_NAMES = ("deconv_depth", "deconv_mask", "deconv_mask_goal")


def _err(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-30)


ELEM_RTOL, ELEM_FLOOR = 1e-5, 1e-6


def _elementwise(a, b, rtol=ELEM_RTOL, floor=ELEM_FLOOR):
    """max over elements of |a - b| / (rtol |b| + floor max|b|): <= 1 passes."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float((np.abs(a - b) / (rtol * np.abs(b) + floor * max(np.abs(b).max(), 1e-30))).max())


def _check_outputs(o_logits, o_value, logits, value):
    """Logits / values: normwise 1e-5 of scale and the elementwise bound above."""
    assert _err(o_logits, logits) <= 1e-5
    assert _err(o_value, value) <= 1e-5
    e = (_elementwise(o_logits, logits), _elementwise(o_value, value))
    assert max(e) <= 1.0, "elementwise logits / values: %.3g / %.3g of the bound" % e
    return e


def _acts_views(net, acts, n):
    """The activation store the forward wrote (csrc/vn_policy.hip acts_at): [conv1 ReLU
    bitmask | X1 | X2 | X3 | X4 | X5], each sample-contiguous NHWC, frames 2i (image) and
    2i + 1 (goal)."""
    o1, o2, o3 = trunk_sizes(*net.frame_hw)
    msz = 2 * o1[0] * o1[1]
    sz = [2 * o1[0] * o1[1] * 32, 2 * o2[0] * o2[1] * 32, o3[0] * o3[1] * 64, o3[0] * o3[1] * 32, 512]
    assert net.act_floats == msz + sum(sz)
    out = {"M1": acts[:n * msz].view(torch.int32).view(n, 2, o1[0], o1[1])}
    p = n * msz
    shapes = [(n, 2, o1[0], o1[1], 32), (n, 2, o2[0], o2[1], 32), (n, o3[0], o3[1], 64), (n, o3[0], o3[1], 32),
              (n, 512)]
    for i, sh in enumerate(shapes):
        out["X%d" % (i + 1)] = acts[p:p + n * sz[i]].view(sh)
        p += n * sz[i]
    return out


def _gpu_masks(net, acts, n):
    """0/1 float64 masks (NCHW) of every trunk ReLU from the GPU's activations; checks that
    conv1's channel bitmask (what conv2's input gradient reads) equals X1 > 0."""
    v = _acts_views(net, acts, n)
    x1 = v["X1"] > 0
    bits = (v["M1"][..., None] >> torch.arange(32, device=acts.device, dtype=torch.int32)) & 1
    assert torch.equal(bits.bool(), x1), "conv1 ReLU bitmask != X1 > 0"

    def nchw(t):
        return t.permute(0, 3, 1, 2).double().cpu()
    return {"m1i": nchw(x1[:, 0]), "m1g": nchw(x1[:, 1]), "m2i": nchw(v["X2"][:, 0] > 0),
            "m2g": nchw(v["X2"][:, 1] > 0), "m3": nchw(v["X3"] > 0), "m4": nchw(v["X4"] > 0),
            "m5": (v["X5"] > 0).double().cpu()}


def _check_masks_are_signs(masks, pre):
    """A mask bit may differ from the sign of the oracle's pre-activation only at a tie."""
    pairs = {"m1i": "z1i", "m1g": "z1g", "m2i": "z2i", "m2g": "z2g", "m3": "z3", "m4": "z4", "m5": "z5"}
    flips = {}
    for m, z in pairs.items():
        zz = pre[z].detach()
        bad = (masks[m] > 0) != (zz > 0)
        if bad.any():
            worst = float(zz[bad].abs().max() / zz.abs().max())
            assert worst <= 1e-5, "%s: mask disagrees with the oracle's sign at |z| = %.3g of scale" % (m, worst)
        flips[m] = int(bad.sum())
    return flips


def _grads_vs_oracle(net, grads, ref, heads=None, tol=1e-4):
    mine = net.to_reference(grads)
    errs = {}
    for k, attr in NAMES.items():
        mod = getattr(ref, attr)
        for kind in ("weight", "bias"):
            errs[k + "." + kind] = _err(mine[k + "." + kind].numpy(), getattr(mod, kind).grad.numpy())
    if heads is not None:
        for h, name in zip(heads.heads, AUX_NAMES):
            for i, layer in ((1, h[0]), (3, h[2])):
                for kind in ("weight", "bias"):
                    key = "%s.0.%d.%s" % (name, i, kind)
                    errs[key] = _err(mine[key].numpy(), getattr(layer, kind).grad.numpy())
    bad = {k: "%.3g" % e for k, e in errs.items() if e > tol}
    assert not bad, bad
    return max(errs.values())


def _noisy_policy(hw, seed, aux=False):
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(seed)
    pol = GoalNavPolicy(3, 4, hw, aux=aux)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
        if aux:  # block-diagonal second head layer, zero pad channel (the layout's structure)
            w1, b1, w2, b2 = pol.net.views(pol.params.data)["aux"]
            m = torch.zeros(48, 8, device=w2.device)
            m[0:16, 0] = 1
            m[16:32, 1:4] = 1
            m[32:48, 4:7] = 1
            w2.mul_(m[:, None, None, :])
            b2[7] = 0.0
    return pol


def _loss_grad(out, actions, rets):
    from vnav import _lib
    lib = _lib.load()
    n = out.shape[0]
    dout = torch.zeros_like(out)
    stats = torch.zeros(4, dtype=torch.float32, device=out.device)
    _lib.check(lib.vn_a2c_loss_grad(_lib.ptr(out), _lib.ptr(actions), _lib.ptr(rets), n, 4, ctypes.c_float(0.5),
                                    ctypes.c_float(0.01), _lib.ptr(dout), _lib.ptr(stats),
                                    _lib.stream_ptr(out.device)), "vn_a2c_loss_grad")
    return dout


def test_84_batch4096_forward_backward_vs_fp64_oracle():
    """84x84, 4096 samples (the bench's per-step env count): forward outputs, conv_merge
    features and every parameter gradient of the A2C loss vs the fp64 oracle."""
    from vnav.policy import frames_from_batch
    pol = _noisy_policy((84, 84), 21)
    net, params = pol.net, pol.params.data
    n = 4096
    g = torch.Generator(device="cuda").manual_seed(5)
    img = torch.randint(0, 256, (n, 84, 84, 3), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (n, 84, 84, 3), dtype=torch.uint8, device="cuda", generator=g)
    actions = torch.randint(0, 4, (n,), dtype=torch.int32, device="cuda", generator=g)
    rets = torch.randn(n, device="cuda", generator=g)
    acts = net.new_acts(n)
    out = torch.zeros((n, 8), device="cuda")
    frames = frames_from_batch(img, gl)
    net.forward(params, frames, n, acts, n, 0, out)
    masks = _gpu_masks(net, acts, n)
    x5 = net.x5(acts, n).double().cpu()
    dout = _loss_grad(out, actions, rets)
    grads = torch.zeros_like(params)
    ws = torch.empty(net.workspace_floats(n), device="cuda")
    net.backward(params, frames, n, acts, n, dout, grads, ws)
    torch.cuda.synchronize()

    ref = GoalNetOracle((84, 84)).load_reference(pol.reference_state_dict()).double()
    fi, fg = frames_to_float(img.cpu()).double(), frames_to_float(gl.cpu()).double()
    logits, value, _, pre = ref.forward_masked(fi, fg, masks)
    flips = _check_masks_are_signs(masks, pre)
    o = out.cpu().numpy()
    _check_outputs(o[:, :4], o[:, 4], logits.detach().numpy(), value.detach().numpy().ravel())
    assert _err(x5.numpy(), (pre["z5"] * masks["m5"]).detach().numpy()) <= 1e-5
    loss, _ = oa2c.loss(logits, value.view(-1), actions.cpu().long(), rets.cpu().double())
    loss.backward()
    worst = _grads_vs_oracle(net, grads, ref)
    print("84x84 n=4096: worst gradient error %.3g of scale; tie flips %s" % (worst, flips))


def _aux_scene(hw=(174, 174), X=6):
    import vnav
    rng = np.random.RandomState(3)
    Y = X
    h, w = hw
    maze = np.ones((X, Y), dtype=bool)
    obs = rng.randint(0, 256, size=(X, Y, 4, h, w, 3)).astype(np.uint8)
    dep = rng.randint(0, 256, size=(X, Y, 4, h, w, 1)).astype(np.uint8)
    seg = rng.randint(0, 256, size=(X, Y, 4, h, w, 3)).astype(np.uint8)
    return vnav.oriented_scene(maze, obs, [(0, 0, 1)], depths=dep, segmentations=seg)


def _gather(env, rows):
    from vnav import _lib
    arena, fb, _, _ = env.frame_arena()
    dst = torch.empty((rows.numel(),) + tuple(env.frame_shape), dtype=torch.uint8, device=env.device)
    _lib.check(env.lib.vn_gather_rows(ctypes.c_void_p(arena), int(fb), _lib.ptr(rows), rows.numel(), _lib.ptr(dst),
                                      env._stream()), "vn_gather_rows")
    return dst


@pytest.mark.parametrize("hw,n", [((174, 174), 512), ((300, 400), 512)], ids=["174x174", "c5_300x400"])
def test_batch_rows_aux_vs_fp64_oracle(hw, n):
    """174x174 (the reference topology) and config C5's 300x400 (the size-adaptive trunk:
    74x99 -> 36x48 -> 17x23, conv_merge over 12,512 features, heads to 74x98), 512 samples
    gathered from the scene cache by row, as the trainer's update runs them (the C5 leg's
    rollout forward runs 512 envs per step): trunk + heads forward, the aux heads' fused loss
    (vn_aux_forward_loss_grad), the aux backward into dL/dX4 and the trunk backward of the
    A2C loss + 0.1 x the deconv loss — outputs, predictions and every gradient vs fp64, with
    the GPU's ReLU masks (no tie search)."""
    import vnav
    from vnav.policy import AuxTargets, frames_from_rows
    pol = _noisy_policy(hw, 8, aux=True)
    net, params = pol.net, pol.params.data
    env = vnav.VectorEnv([_aux_scene(hw, 6 if hw == (174, 174) else 4)], 8, seed=1)
    arena, fb, rows_total, _ = env.frame_arena()
    w = 0.1
    g = torch.Generator(device="cuda").manual_seed(9)
    rows_i = torch.randint(0, rows_total, (n,), dtype=torch.int32, device="cuda", generator=g)
    rows_g = torch.randint(0, rows_total, (n,), dtype=torch.int32, device="cuda", generator=g)
    actions = torch.randint(0, 4, (n,), dtype=torch.int32, device="cuda", generator=g)
    rets = torch.randn(n, device="cuda", generator=g)
    frames = frames_from_rows(arena, fb, rows_i, rows_g)
    acts = net.new_acts(n)
    out = torch.zeros((n, 8), device="cuda")
    net.forward(params, frames, n, acts, n, 0, out)
    masks = _gpu_masks(net, acts, n)
    dout = _loss_grad(out, actions, rets)
    depth, seg = env.aux_arena
    table = net.aux_target_table(depth, seg)
    tg = AuxTargets(table.data_ptr(), rows_i.data_ptr(), rows_g.data_ptr())
    a1, pred = net.aux_buffers(n)
    dpred = torch.empty_like(pred)
    stats = torch.zeros(4, device="cuda")
    aws = torch.empty(net.aux_workspace_floats(), device="cuda")
    net.aux_forward_loss_grad(params, acts, n, n, a1, pred, tg, w, dpred, stats, aws)
    amasks = [(a1[..., 16 * h:16 * h + 16] > 0).permute(0, 3, 1, 2).double().cpu() for h in range(3)]
    grads = torch.zeros_like(params)
    dx4 = torch.empty((n, net.fc_in), device="cuda")
    net.aux_backward(params, acts, n, n, a1, dpred, grads, dx4, aws)
    ws = torch.empty(net.workspace_floats(n), device="cuda")
    net.backward_ex(params, frames, n, acts, n, dout, None, dx4, grads, ws)
    img, gl = _gather(env, rows_i).cpu(), _gather(env, rows_g).cpu()
    ri, rg = rows_i.cpu().numpy(), rows_g.cpu().numpy()
    dd, ss = depth.cpu().numpy(), seg.cpu().numpy()
    torch.cuda.synchronize()

    sd = pol.reference_state_dict()
    ref = GoalNetOracle(hw).load_reference(sd).double()
    heads = AuxHeadsOracle().load_reference(sd).double()
    logits, value, x4, pre = ref.forward_masked(frames_to_float(img).double(), frames_to_float(gl).double(), masks)
    flips = _check_masks_are_signs(masks, pre)
    preds, apre = heads.forward_masked(x4, amasks)
    for m, z in zip(amasks, apre):
        bad = (m > 0) != (z.detach() > 0)
        if bad.any():
            assert float(z.detach()[bad].abs().max() / z.detach().abs().max()) <= 1e-5
    o = out.cpu().numpy()
    _check_outputs(o[:, :4], o[:, 4], logits.detach().numpy(), value.detach().numpy().ravel())
    ph, pw = net.aux_layout["p_hw"]
    tgt = [t.double() for t in aux_targets(dd[ri], ss[ri], ss[rg], 4, (ph, pw))]
    mse = [torch.nn.functional.mse_loss(p, t) for p, t in zip(preds, tgt)]
    numel = np.array([1, 3, 3]) * n * ph * pw
    assert _err(stats[:3].cpu().numpy() / numel, np.array([m.item() for m in mse])) <= 1e-5
    loss, _ = oa2c.loss(logits, value.view(-1), actions.cpu().long(), rets.cpu().double())
    (loss + w * sum(mse)).backward()
    worst = _grads_vs_oracle(net, grads, ref, heads)
    print("%dx%d n=%d + aux: worst gradient error %.3g of scale; tie flips %s" % (hw[0], hw[1], n, worst, flips))


@pytest.mark.parametrize("E", [2048, 1024, 16, 5])
def test_lstm_core_vs_fp64_torch_lstm(E):
    """The recurrent core at 2048 envs x 3 steps (6144 rows: the trunk-feature gradient
    dz5 = dgates x W_ih takes the unsplit 128 x 128 EpiMask product the training update runs at
    >= 4096 rows), at 1024 envs x 3 steps (gates / dh products past the split-K
    threshold, the weight gradient over 3072 rows) and at 16 / 5 envs (the fused VALU
    steps of vn_skinny.h: xcat + gates + cell, dh product + next cell backward): per-step
    (h, c), the heads on h, and the gradients of W_ih, W_hh, both biases, the heads and
    dL/dZ5 (masked by the features' ReLU) vs torch's float64 nn.LSTM with the restated
    MaskedRNN convention."""
    from vnav.policy import PolicyNet
    net = PolicyNet((84, 84), 4, recurrent=True)
    params = net.init_params(3)
    with torch.no_grad():
        params.add_(torch.randn(params.shape, generator=torch.Generator().manual_seed(2)).cuda() * 0.01)
    T, A = 3, 4
    N = T * E
    L = net.lstm
    g = torch.Generator(device="cuda").manual_seed(4)
    x5 = torch.relu(torch.randn((N, 512), device="cuda", generator=g))
    lra = torch.zeros((T, E, A + 1), device="cuda")
    lra[..., :A].scatter_(2, torch.randint(0, A, (T, E, 1), device="cuda", generator=g), 1.0)
    lra[..., A] = (torch.rand((T, E), device="cuda", generator=g) < 0.1).float()
    masks = (torch.rand((T, E), device="cuda", generator=g) > 0.05).float()
    lra *= masks[..., None]
    h0 = torch.randn((E, 512), device="cuda", generator=g) * 0.5
    c0 = torch.randn((E, 512), device="cuda", generator=g) * 0.5
    xcat = torch.zeros((N, L["xcat"]), device="cuda")
    la = torch.zeros((N, 2048), device="cuda")
    c_all = torch.zeros((N, 512), device="cuda")
    h_all = torch.zeros((N, 512), device="cuda")
    gates = torch.zeros((E, 2048), device="cuda")
    out = torch.zeros((N, 8), device="cuda")
    for t in range(T):
        sl = slice(t * E, (t + 1) * E)
        hp = h0 if t == 0 else h_all[(t - 1) * E:t * E]
        cp = c0 if t == 0 else c_all[(t - 1) * E:t * E]
        net.lstm_step(params, E, x5[sl], lra[t], masks[t], hp, cp, xcat[sl], gates, la[sl], c_all[sl], h_all[sl])
    net.heads(params, h_all, N, out)
    actions = torch.randint(0, A, (N,), dtype=torch.int32, device="cuda", generator=g)
    rets = torch.randn(N, device="cuda", generator=g)
    dout = _loss_grad(out, actions, rets)
    grads = torch.zeros_like(params)
    dz5 = torch.zeros((N, 512), device="cuda")
    ws = torch.empty(net.lstm_workspace_floats(T, E), device="cuda")
    net.lstm_backward(params, T, E, dout, h_all, xcat, la, c_all, c0, masks, x5, dz5, grads, ws)
    torch.cuda.synchronize()

    sd = net.to_reference(params)
    lstm = torch.nn.LSTM(512 + A + 1, 512, batch_first=True).double()
    for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
        getattr(lstm, name).data.copy_(sd["rnn.inner." + name].double())
    pl = torch.nn.Linear(512, A).double()
    cr = torch.nn.Linear(512, 1).double()
    for mod, k in ((pl, "policy_logits.0"), (cr, "critic.0")):
        mod.weight.data.copy_(sd[k + ".weight"].double())
        mod.bias.data.copy_(sd[k + ".bias"].double())
    xf = x5.cpu().double().view(T, E, 512).requires_grad_()
    x = torch.cat((xf, lra.cpu().double()), 2)
    h, c = h0.cpu().double()[None], c0.cpu().double()[None]
    m = masks.cpu().double()
    ys, cs = [], []
    for t in range(T):
        y, (h, c) = lstm(x[t][:, None], (h * m[t][None, :, None], c * m[t][None, :, None]))
        ys.append(y[:, 0])
        cs.append(c[0])
    y = torch.cat(ys)
    assert _err(h_all.cpu().numpy(), y.detach().numpy()) <= 1e-5
    assert _err(c_all.cpu().numpy(), torch.cat(cs).detach().numpy()) <= 1e-5
    logits, value = pl(y), cr(y)
    o = out.cpu().numpy()
    _check_outputs(o[:, :4], o[:, 4], logits.detach().numpy(), value.detach().numpy().ravel())
    loss, _ = oa2c.loss(logits, value.view(-1), actions.cpu().long(), rets.cpu().double())
    loss.backward()
    mine = net.to_reference(grads)
    errs = {"dz5": _err(dz5.cpu().numpy(), (xf.grad * (xf > 0)).reshape(N, 512).detach().numpy())}
    for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
        errs[name] = _err(mine["rnn.inner." + name].numpy(), getattr(lstm, name).grad.numpy())
    for mod, k in ((pl, "policy_logits.0"), (cr, "critic.0")):
        errs[k + ".weight"] = _err(mine[k + ".weight"].numpy(), mod.weight.grad.numpy())
        errs[k + ".bias"] = _err(mine[k + ".bias"].numpy(), mod.bias.grad.numpy())
    bad = {k: "%.3g" % e for k, e in errs.items() if e > 1e-4}
    assert not bad, bad
    print("LSTM E=%d T=3: worst gradient error %.3g of scale" % (E, max(errs.values())))


def test_logged_run_shape_trainer_update_vs_fp64_oracle():
    """The reference's own batch (outputs/output.txt: 174x174, LSTM + deconv heads, aux weight
    0.1, 4 envs x 20 steps): the second rollout + update of A2CTrainer — the small-batch
    split-K products and their epilogues, the per-step LSTM / sampling / index-only env
    step / step_post kernels — restated in float64: the env transitions against the env
    oracle driven by the same actions, the sampled actions against the Philox inverse-CDF
    draw on the rollout's logits, the rollout's logits / values against the masked fp64
    network, and the update's total gradient (A2C + 0.1 x deconv loss through BPTT) against
    the fp64 gradient."""
    import dataclasses
    import vnav
    from oracle import envs as oe
    from oracle import graph as og
    from oracle import philox
    from vnav import dist as vdist
    from vnav.policy import frames_from_rows
    maze = np.random.RandomState(2).rand(5, 6) > 0.2
    graph, spd, _ = og.h5_tables(maze)
    ns = len(graph)
    rng = np.random.RandomState(4)
    frames = rng.randint(0, 256, size=(ns, 174, 174, 3)).astype(np.uint8)
    scene = vnav.scene_from_arrays(graph, spd, frames)
    scene = dataclasses.replace(scene, depth=rng.randint(0, 256, size=(ns, 174, 174, 1)).astype(np.uint8),
                                segmentation=rng.randint(0, 256, size=(ns, 174, 174, 3)).astype(np.uint8))
    T, E, A, seed, env_seed, w = 20, 4, 4, 3, 11, 0.1
    env = vnav.VectorEnv([scene], E, seed=env_seed, max_episode_steps=25)
    tr = vnav.A2CTrainer(env, num_steps=T, seed=seed, max_time_steps=1e6, recurrent=True, aux_weight=w)
    o = oe.VectorEnvOracle([dict(graph=graph, spd=spd, rewards=scene.rewards)], E, env_seed, max_steps=25)
    tr.step(sync=True)
    a1 = tr.actions.cpu().numpy().reshape(T, E)
    for t in range(T):
        o.step(a1[t])
    h0, c0 = tr.h0.cpu().double(), tr.c0.cpu().double()
    p0 = tr.params.detach().clone()
    tr.rollout()
    net = tr.net
    N = T * E
    masks = _gpu_masks(net, tr.acts, N)
    bmasks = _gpu_masks(net, tr.boot_acts, E)
    # the aux heads' ReLU masks: the same first layer run on the rollout's X4
    a1buf, predbuf = net.aux_buffers(N)
    net.aux_forward(tr.params, tr.acts, N, N, a1buf, predbuf, torch.empty(net.aux_workspace_floats(), device="cuda"))
    amasks = [(a1buf[..., 16 * h:16 * h + 16] > 0).permute(0, 3, 1, 2).double().cpu() for h in range(3)]
    rows_i, rows_g = tr.rows_img.cpu().numpy(), tr.rows_goal.cpu().numpy()
    brows = (env._info["img_row"].cpu().numpy(), env._info["goal_row"].cpu().numpy())
    actions = tr.actions.cpu().long()
    rewards, dones = tr.rewards.cpu(), tr.dones.cpu()
    out = tr.out.cpu().double()
    boot = tr.boot_out.cpu().double()
    lmask, lra = tr.masks.cpu().double(), tr.lra.cpu().double()
    bmask, blra = tr.boot_mask.cpu().double(), tr.boot_lra.cpu().double()
    tr.update()
    grads = tr.grads.clone()
    torch.cuda.synchronize()

    # env transitions (index-only vn_step) vs the env oracle on the same actions
    a2 = actions.numpy().reshape(T, E)
    for t in range(T):
        r = o.step(a2[t])
        ri = rows_i[(t + 1) * E:(t + 2) * E] if t + 1 < T else brows[0]
        rg = rows_g[(t + 1) * E:(t + 2) * E] if t + 1 < T else brows[1]
        assert np.array_equal(ri, r["img_row"]) and np.array_equal(rg, r["goal_row"]), t
        assert np.array_equal(rewards[t].numpy().view(np.uint32), r["reward"].view(np.uint32)), t
        assert np.array_equal(dones[t].numpy(), r["done"]), t
    # sampled actions: Philox stream 3 inverse-CDF on the rollout's logits (vn_a2c.hip sample_kernel)
    k = vdist.rank_seed(seed, 0)
    lg = out[:, :A].numpy().astype(np.float32).reshape(T, E, A)
    for t in range(T):
        ctr = T * 1 + t  # updates so far x T + step
        rr = philox.philox4x32_10(np.arange(E), ctr & 0xffffffff, ctr >> 32, philox.STREAM_POLICY,
                                  k & 0xffffffff, k >> 32)[0]
        u = (rr >> 8).astype(np.float32) * np.float32(1.0 / 16777216.0)
        p = np.exp(lg[t] - lg[t].max(1, keepdims=True))
        p = p / p.sum(1, keepdims=True)
        cdf = np.cumsum(p, 1)
        want = np.minimum((u[:, None] >= cdf[:, :A - 1]).sum(1), A - 1)
        near = np.abs(u[:, None] - cdf[:, :A - 1]).min(1) < 1e-5
        assert np.array_equal(want[~near], a2[t][~near]), t

    sd = net.to_reference(p0)
    ref = GoalNetOracle((174, 174)).load_reference(sd).double()
    heads = AuxHeadsOracle().load_reference(sd).double()
    lstm = torch.nn.LSTM(512 + A + 1, 512, batch_first=True).double()
    for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
        getattr(lstm, name).data.copy_(sd["rnn.inner." + name].double())
    fl = lambda x: frames_to_float(torch.as_tensor(x)).double()  # noqa: E731
    _, _, x4, pre = ref.forward_masked(fl(frames[rows_i]), fl(frames[rows_g]), masks)
    _check_masks_are_signs(masks, pre)
    x5 = (pre["z5"] * masks["m5"]).view(T, E, 512)
    _, _, _, bpre = ref.forward_masked(fl(frames[brows[0]]), fl(frames[brows[1]]), bmasks)
    xb = bpre["z5"] * bmasks["m5"]
    h, c = h0[None], c0[None]
    ys = []
    for t in range(T):
        m = lmask[t][None, :, None]
        y, (h, c) = lstm(torch.cat((x5[t], lra[t]), 1)[:, None], (h * m, c * m))
        ys.append(y[:, 0])
    m = bmask[None, :, None]
    yb, _ = lstm(torch.cat((xb, blra), 1)[:, None], (h * m, c * m))
    y = torch.cat(ys)
    logits, value = ref.policy_logits(y), ref.critic(y).view(-1)
    vboot = ref.critic(yb[:, 0]).view(-1)
    _check_outputs(out[:, :A].numpy(), out[:, A].numpy(), logits.detach().numpy(), value.detach().numpy())
    assert _err(boot[:, A].numpy(), vboot.detach().numpy()) <= 1e-5
    assert _elementwise(boot[:, A].numpy(), vboot.detach().numpy()) <= 1.0
    vext = torch.cat([value.detach().view(T, E), vboot.detach().view(1, E)])
    R = oa2c.returns(rewards.double(), dones, vext, 0.99)
    loss, _ = oa2c.loss(logits, value, actions, R.view(-1))
    preds, apre = heads.forward_masked(x4, amasks)
    dd, ss = scene.depth, scene.segmentation
    ph, pw = net.aux_layout["p_hw"]
    tgt = [t_.double() for t_ in aux_targets(dd[rows_i], ss[rows_i], ss[rows_g], 4, (ph, pw))]
    (loss + w * sum(torch.nn.functional.mse_loss(p, t_) for p, t_ in zip(preds, tgt))).backward()
    mine = net.to_reference(grads)
    errs = {}
    for k_, attr in NAMES.items():
        mod = getattr(ref, attr)
        for kind in ("weight", "bias"):
            errs[k_ + "." + kind] = _err(mine[k_ + "." + kind].numpy(), getattr(mod, kind).grad.numpy())
    for name in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0"):
        errs[name] = _err(mine["rnn.inner." + name].numpy(), getattr(lstm, name).grad.numpy())
    for hd, name in zip(heads.heads, AUX_NAMES):
        for i, layer in ((1, hd[0]), (3, hd[2])):
            for kind in ("weight", "bias"):
                key = "%s.0.%d.%s" % (name, i, kind)
                errs[key] = _err(mine[key].numpy(), getattr(layer, kind).grad.numpy())
    bad = {k_: "%.3g" % e for k_, e in errs.items() if e > 1e-4}
    assert not bad, bad
    print("logged-run shape (174x174, LSTM + aux, 4 envs x 20): worst gradient error %.3g" % max(errs.values()))
