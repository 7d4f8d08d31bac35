"""UNREAL heads (models/goal.py:94-137) on the HIP path: pixel control (pc_base product,
the stacked 32 -> 64 and block-diagonal 64 -> 8 transposed convs, the value/action
combination) and reward prediction (Linear on three frames' conv_base maps), through the
C ABI (vn_pc_forward / vn_pc_backward / vn_rp_forward / vn_rp_backward).
  * vs the REFERENCE modules' goldens at 174x174 (tests/golden/unreal174.npz);
  * vs the fp64 restatement (oracle/policy.py) at 84x84, 174x174 and 300x400 (rp's
    in_features derived from the frame) on batches that take several tiles.
Tolerances: outputs rtol 1e-5 of scale, gradients 1e-4 of scale (as test_aux_gpu.py);
the pc_action branch's gradients are exactly zero, as torch computes them."""
import numpy as np
import pytest
import torch

from oracle.policy import (pixel_control, reward_prediction, seeded_reference_state, seeded_unreal_state,
                           UNREAL_PARAM_ORDER)

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, what):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err <= rtol, "%s: max err %.3g of scale %.3g" % (what, err, scale)


def _net(hw):
    from vnav.policy import PolicyNet
    return PolicyNet(hw, 4, device="cuda:0", unreal=True)


def _run(net, params, h, dq, feats_nhwc, drp, dh_init=None):
    """Forward and backward of both heads; returns q, dh, rp logits, dx, grads (reference names)."""
    n = h.shape[0]
    ws = torch.empty(net.pc_workspace_floats(), dtype=torch.float32, device="cuda")
    pcb, a1, p2, q = net.pc_buffers(n)
    net.pc_forward(params, h, n, pcb, a1, p2, q, ws)
    q_out = q.clone()
    A = net.num_actions
    masks = {"pc_base": (pcb > 0).permute(0, 3, 1, 2).cpu(), "pc_value.0": (a1[..., :32] > 0).permute(0, 3, 1, 2).cpu(),
             "pc_action.0": (a1[..., 32:] > 0).permute(0, 3, 1, 2).cpu(),
             "pc_value.2": (p2[..., :A] > 0).permute(0, 3, 1, 2).cpu(),
             "pc_action.2": (p2[..., A:A + 1] > 0).permute(0, 3, 1, 2).cpu()}
    grads = torch.zeros_like(params)
    dh = dh_init.clone() if dh_init is not None else torch.empty((n, 512), dtype=torch.float32, device="cuda")
    net.pc_backward(params, h, n, pcb, a1, p2, dq.contiguous(), grads, dh, ws, accumulate=dh_init is not None)
    R = feats_nhwc.shape[0]
    out = torch.empty((R, 4), dtype=torch.float32, device="cuda")
    net.rp_forward(params, feats_nhwc, R, out)
    dout = torch.zeros((R, 4), dtype=torch.float32, device="cuda")
    dout[:, :3] = drp
    dx = torch.empty_like(feats_nhwc)
    net.rp_backward(params, feats_nhwc, R, dout, grads, dx, ws)
    torch.cuda.synchronize()
    return q_out, dh, out[:, :3], dx, net.to_reference(grads), masks


def _nhwc_frames(feats):
    """[R, 3, 32, h3, w3] (the reference's conv_base output of 3 frames) -> [R, 3 * h3 * w3 * 32]."""
    return feats.permute(0, 1, 3, 4, 2).reshape(feats.shape[0], -1).contiguous()


def test_unreal_heads_match_reference_174(golden):
    d = golden("unreal174.npz")
    seed = int(d["seed"][0])
    net = _net((174, 174))
    sd = {**seeded_reference_state((174, 174), 0), **seeded_unreal_state((174, 174), seed)}
    params = net.from_reference(sd)
    B, T = d["h"].shape[:2]
    n = B * T
    h = torch.as_tensor(d["h"]).reshape(n, 512).cuda()
    dq = torch.as_tensor(d["dq"]).reshape(n, 4, 42, 42).permute(0, 2, 3, 1).cuda()
    feats = torch.as_tensor(d["rp_features"])
    q, dh, logits, dx, g, _ = _run(net, params, h, dq, _nhwc_frames(feats).cuda(), torch.as_tensor(d["drp"]).cuda())
    _close(q.permute(0, 3, 1, 2).cpu().numpy(), d["q"].reshape(n, 4, 42, 42), 1e-5, "q")
    _close(logits.cpu().numpy(), d["rp_logits"], 1e-5, "rp logits")
    _close(dh.cpu().numpy(), d["dh"].reshape(n, 512), 1e-4, "dh")
    R = feats.shape[0]
    dx_ref = _nhwc_frames(torch.as_tensor(d["d_rp_features"])).numpy()
    _close(dx.cpu().numpy(), dx_ref.reshape(R, -1), 1e-5, "d rp features")
    for name in UNREAL_PARAM_ORDER:
        got = g[name].numpy()
        if name == "pc_base.0.0.weight":
            got = got[::16]
        want = d["g:" + name]
        if name.startswith("pc_action"):
            np.testing.assert_array_equal(got, 0.0, err_msg=name)
            assert not np.any(want)
        else:
            _close(got, want, 1e-4, name)


@pytest.mark.parametrize("hw,n,R", [((84, 84), 37, 50), ((174, 174), 70, 33), ((300, 400), 19, 9)])
def test_unreal_heads_vs_fp64_oracle(hw, n, R):
    net = _net(hw)
    params = net.init_params(seed=3)
    v = net.views(params)
    with torch.no_grad():  # biases off zero so the bias paths and ReLU masks are exercised
        u = v["unreal"]
        g = torch.Generator(device="cpu").manual_seed(4)
        for k in ("pc_b", "b1", "b2", "rp_b"):
            u[k].copy_((torch.rand(u[k].shape, generator=g) * 0.1 - 0.05).to(u[k].device))
        u["b2"][5:] = 0.0
        u["rp_b"][3] = 0.0
    ref = {k: t.double().requires_grad_() for k, t in net.to_reference(params).items() if k in UNREAL_PARAM_ORDER}
    torch.manual_seed(5)
    h = (torch.rand(n, 512) * 2.0 - 0.5)
    dq = torch.randn(n, 4, 42, 42)
    h3, w3 = net.o3
    feats = torch.randn(R, 3, 32, h3, w3) * 0.1
    drp = torch.randn(R, 3)
    dh0 = torch.randn(n, 512)
    q, dh, logits, dx, g, masks = _run(net, params, h.cuda(), dq.permute(0, 2, 3, 1).cuda(),
                                       _nhwc_frames(feats).cuda(), drp.cuda(), dh_init=dh0.cuda())
    h64 = h.double().requires_grad_()
    f64 = feats.double().requires_grad_()
    q_ref = pixel_control(ref, h64, masks)  # the GPU's ReLU masks: no tie can flip between them
    l_ref = reward_prediction(ref, f64)
    ((q_ref * dq.double()).sum() + (l_ref * drp.double()).sum()).backward()
    _close(q.permute(0, 3, 1, 2).cpu().numpy(), q_ref.detach().numpy(), 1e-5, "q")
    _close(logits.cpu().numpy(), l_ref.detach().numpy(), 1e-5, "rp logits")
    _close((dh.cpu() - dh0).numpy(), h64.grad.numpy(), 1e-4, "dh (accumulated)")
    _close(dx.cpu().numpy(), _nhwc_frames(f64.grad).numpy(), 1e-5, "d rp features")
    for name in UNREAL_PARAM_ORDER:
        if name.startswith("pc_action"):
            np.testing.assert_array_equal(g[name].numpy(), 0.0, err_msg=name)
        else:
            _close(g[name].numpy(), ref[name].grad.numpy(), 1e-4, name)


def test_unreal_flag_taken_for_bighouse():
    """BigHouseModel's own heads (bignet.py:77-111; tests/test_bighouse_unreal_gpu.py); the aux
    deconv heads stay BigGoalHouseModel's."""
    from vnav import _lib
    from vnav.policy import PolicyNet
    net = PolicyNet((84, 84), 4, device="cuda:0", arch="bighouse", unreal=True)
    assert net.pc_side == 20
    with pytest.raises(_lib.VnavError):
        PolicyNet((84, 84), 4, device="cuda:0", arch="bighouse", aux=True)


# ---- the UNREAL losses (csrc/vn_unreal_loss.hip) vs oracle/unreal.py (parity unpinned:
# deep_rl's UnrealTrainer is absent; the oracle restates the published algorithm) ----------

def _loss_case(seed=7, T=5, E=7, S=4, A=4, H=174, W=174, rows=40):
    g = torch.Generator().manual_seed(seed)
    arena = torch.randint(0, 256, (rows, H, W, 3), generator=g, dtype=torch.uint8)
    rows_img = torch.randint(0, rows, (T * E,), generator=g, dtype=torch.int32)
    rows_last = torch.randint(0, rows, (E,), generator=g, dtype=torch.int32)
    actions = torch.randint(0, A, (T * E,), generator=g, dtype=torch.int32)
    dones = torch.rand((T, E), generator=g) < 0.2
    rewards = torch.where(torch.rand((T, E), generator=g) < 0.5, 0.0, torch.where(torch.rand((T, E), generator=g) < 0.5,
                                                                                   1.0, -0.01))
    return dict(T=T, E=E, S=S, A=A, H=H, W=W, arena=arena, rows_img=rows_img, rows_last=rows_last, actions=actions,
                dones=dones, rewards=rewards.float(), g=g)


@pytest.mark.parametrize("hw", [(174, 174), (300, 400)])
def test_pc_loss_kernel_vs_oracle(hw):
    from oracle import unreal
    from vnav import _lib
    lib = _lib.load()
    c = _loss_case(H=hw[0], W=hw[1])
    T, E, S, A = c["T"], c["E"], c["S"], c["A"]
    # the heads' maps after their ReLUs: value channels 0..A-1, action channel A, padding
    p2 = torch.relu(torch.randn(((T + 1) * S, 42, 42, 8), generator=c["g"]) * 0.3)
    p2[..., A + 1:] = 0.0
    q = (p2[..., :A] + p2[..., A:A + 1]) - p2[..., A:A + 1]
    P = _lib.ptr
    d = {k: c[k].cuda() for k in ("arena", "rows_img", "rows_last", "actions", "dones")}
    dp2 = p2.cuda()
    stats = torch.zeros(1, device="cuda")
    w = 0.05
    _lib.check(lib.vn_unreal_pc_loss_grad(P(dp2), P(d["actions"]), P(d["dones"]), P(d["arena"]),
                                          hw[0] * hw[1] * 3, hw[0], hw[1], P(d["rows_img"]), P(d["rows_last"]), T, E, S,
                                          A, ctypes_float(0.9), ctypes_float(w), P(stats), None), "pc loss")
    torch.cuda.synchronize()
    # oracle on the first S envs: frames t = 0..T-1 from the rollout rows, t = T the last obs
    rows = torch.cat((c["rows_img"].view(T, E)[:, :S], c["rows_last"][None, :S])).long()
    frames = c["arena"][rows]
    loss, grad = unreal.pc_loss(q.view(T + 1, S, 42, 42, A), frames, c["actions"].view(T, E)[:, :S],
                                c["dones"][:, :S])
    # dL/dp2: the q gradient under the value channels' ReLU, 0 on the action channel and padding
    want = torch.zeros((T + 1, S, 42, 42, 8), dtype=torch.float64)
    want[..., :A] = grad * (p2.view(T + 1, S, 42, 42, 8)[..., :A] > 0)
    _close(dp2.cpu().view(T + 1, S, 42, 42, 8).numpy() / w, want.numpy(), 1e-5, "dp2")
    np.testing.assert_allclose(stats.item() / (T * S * 42 * 42), loss.item(), rtol=1e-5)


def test_rp_and_vr_kernels_vs_oracle():
    from oracle import unreal
    from vnav import _lib
    lib = _lib.load()
    c = _loss_case(seed=8, T=9, E=6, S=5)
    T, E, S = c["T"], c["E"], c["S"]
    n = (T - 2) * S
    logits = torch.randn((n, 4), generator=c["g"])
    P = _lib.ptr
    rw, dn = c["rewards"].cuda(), c["dones"].cuda()
    lg, dl, st = logits.cuda(), torch.full((n, 4), 5.0, device="cuda"), torch.zeros(2, device="cuda")
    _lib.check(lib.vn_unreal_rp_loss_grad(P(lg), P(rw), P(dn), T, E, S, ctypes_float(1.0), P(dl), P(st), None), "rp")
    loss, grad, count = unreal.rp_loss(logits[:, :3], c["rewards"][:, :S], c["dones"][:, :S])
    torch.cuda.synchronize()
    assert int(st[1].item()) == count > 0
    np.testing.assert_allclose(st[0].item(), loss.item(), rtol=1e-5)
    _close(dl[:, :3].cpu().numpy(), grad.numpy(), 1e-5, "dlogits")
    assert not dl[:, 3].any()
    # scatter of the rp input gradient into dX4 rows t*E + e (fixed order: slots 2, 1, 0)
    F = 64
    dx = torch.randn((n, 3, F), generator=c["g"])
    dx4 = torch.randn((T * E, F), generator=c["g"])
    out, dxd = dx4.clone().cuda(), dx.cuda()  # referenced until the kernel ran
    _lib.check(lib.vn_unreal_rp_scatter(P(dxd), T, E, S, F, P(out), 1, None), "scatter")
    torch.cuda.synchronize()
    want = dx4.clone().view(T, E, F)
    dxv = dx.view(T - 2, S, 3, F)
    for k in range(3):
        want[k:k + T - 2, :S] += dxv[:, :, k]
    _close(out.cpu().numpy(), want.view(T * E, F).numpy(), 1e-6, "scatter")
    # value replay: dout's value column += vr_weight * d mean (V - R)^2 / dV on the first S envs
    A = 4
    outp = torch.randn((T * E, 8), generator=c["g"])
    ret = torch.randn((T * E,), generator=c["g"])
    dout = torch.randn((T * E, 8), generator=c["g"])
    dd, vs = dout.clone().cuda(), torch.zeros(1, device="cuda")
    od, rd = outp.cuda(), ret.cuda()
    _lib.check(lib.vn_unreal_vr_grad(P(od), P(rd), T, E, S, A, ctypes_float(1.0), P(dd), P(vs), None), "vr")
    loss, grad = unreal.vr_loss(outp[:, A].view(T, E)[:, :S], ret.view(T, E)[:, :S])
    torch.cuda.synchronize()
    got = (dd.cpu() - dout)[:, A].view(T, E)
    _close(got[:, :S].numpy(), grad.numpy(), 1e-5, "vr grad")
    assert not got[:, S:].any() and torch.equal(dd.cpu()[:, :A], dout[:, :A])
    np.testing.assert_allclose(vs.item() / (T * S), loss.item(), rtol=1e-5)


def ctypes_float(x):
    import ctypes
    return ctypes.c_float(x)


def _unreal_env(n_envs, seed=2):
    import vnav
    from test_aux_gpu import _aux_scene
    return vnav.VectorEnv([_aux_scene(0, (174, 174, 3))], n_envs, seed=seed, max_episode_steps=30)


def test_trainer_unreal_losses_and_graph():
    """A2CTrainer(unreal=True) with the aux heads (the thor-cached-auxiliary workload): the
    pc / rp / vr losses are reported and finite, the pc_action branch never moves (its
    gradient is exactly zero), pc_value and rp do; the hipGraph replay of the update is
    bit-identical to the eager updates."""
    import vnav

    def run(graph):
        env = _unreal_env(24)
        tr = vnav.A2CTrainer(env, num_steps=6, seed=3, max_time_steps=1e9, recurrent=True, aux_weight=0.1,
                             unreal=True, unreal_envs=8, cuda_graph=graph)
        p0 = tr.params.detach().clone()
        ms = [tr.step(sync=True) for _ in range(4)]
        return tr, p0, ms

    tr, p0, ms = run(False)
    for m in ms:
        for k in ("pc_loss", "rp_loss", "vr_loss", "aux_loss", "value_loss"):
            assert np.isfinite(m[k]), (k, m)
        assert m["pc_loss"] > 0 and m["rp_loss"] >= 0
    # no reward in these few steps: reward prediction learns class 0 (its CE reaches 0 in fp32)
    assert ms[0]["rp_loss"] > ms[-1]["rp_loss"]
    net = tr.net
    v0, v1 = net.views(p0)["unreal"], net.views(tr.params)["unreal"]
    A = net.num_actions
    assert torch.equal(v0["w1"][..., 32:], v1["w1"][..., 32:]) and torch.equal(v0["w2"][32:], v1["w2"][32:])
    assert not torch.equal(v0["w1"][..., :32], v1["w1"][..., :32])
    assert not torch.equal(v0["w2"][:32, ..., :A], v1["w2"][:32, ..., :A])
    assert not torch.equal(v0["pc_w"], v1["pc_w"]) and not torch.equal(v0["rp_w"], v1["rp_w"])
    trg, _, msg = run(True)
    assert torch.equal(tr.params, trg.params) and torch.equal(tr.square_avg, trg.square_avg)
    for x, y in zip(ms, msg):
        for k in ("rp_loss", "value_loss", "grad_norm"):
            assert x[k] == y[k], (k, x[k], y[k])
        # the pc loss statistic sums per-workgroup partials with atomics (metric only)
        np.testing.assert_allclose(x["pc_loss"], y["pc_loss"], rtol=1e-5)


def test_unreal_replayed_sequence_of_this_rollout_equals_on_policy_losses():
    """unreal_source='replay' with a one-slot ring replays the rollout just collected: its own
    trunk, LSTM (from the (h, c) the rollout started from) and heads pass over the first S envs
    must give the on-policy path's pc / rp / vr losses and the same total gradient, up to
    rounding (the replayed batch runs other product paths: (T + 1) S samples against E). Both
    trainers then step on; the replayed path's checkpoint resumes bit-exactly."""
    import vnav
    E, T, S = 16, 5, 16
    trs = []
    for src in ("rollout", "replay"):
        env = _unreal_env(E, seed=5)
        trs.append(vnav.A2CTrainer(env, num_steps=T, seed=3, max_time_steps=1e9, recurrent=True, unreal=True,
                                   unreal_envs=S, unreal_source=src, replay_size=1))
    a, b = trs
    assert b.replay and b.unreal_source == "replay" and a.unreal_source == "rollout"
    stats = []
    for tr in trs:
        batch, _ = tr.sample_training_batch()
        tr.update(batch)
        torch.cuda.synchronize()
        stats.append(tr.unreal_stats.clone())
    assert torch.equal(a.actions, b.actions) and torch.equal(a.rows_img, b.rows_img)
    sa, sb = stats
    np.testing.assert_allclose(sb.cpu().numpy(), sa.cpu().numpy(), rtol=2e-4, atol=1e-7)
    ga, gb = a.net.to_reference(a.grads), b.net.to_reference(b.grads)
    bad = {}
    for k in ga:
        ref = ga[k].numpy().astype(np.float64)
        sc = np.abs(ref).max()
        if sc == 0:
            continue
        e = np.abs(gb[k].numpy() - ref).max() / sc
        if e > 1e-4:
            bad[k] = "%.3g" % e
    assert not bad, bad
    # resume: a checkpoint of the replay trainer reproduces its next updates exactly
    import copy
    sd = copy.deepcopy(b.state_dict())
    m1 = [b.step(sync=True) for _ in range(2)]
    env = _unreal_env(E, seed=5)
    c = vnav.A2CTrainer(env, num_steps=T, seed=3, max_time_steps=1e9, recurrent=True, unreal=True, unreal_envs=S,
                        unreal_source="replay", replay_size=1)
    c.load_state_dict(sd)
    m2 = [c.step(sync=True) for _ in range(2)]
    assert torch.equal(b.params, c.params)
    for x, y in zip(m1, m2):
        assert x["rp_loss"] == y["rp_loss"] and x["vr_loss"] == y["vr_loss"]


def test_goal_nav_policy_reward_prediction_and_pixel_control(golden):
    """GoalNavPolicy(unreal=True).reward_prediction on uint8 frames vs the REFERENCE module's
    golden (the frames regenerate from the golden's seed: gen_model_goldens.unreal_case draws
    them after h and dq), its rp gradients; pixel_control's Q maps and gradients reach the
    LSTM and pc_value, never pc_action."""
    from vnav.policy import GoalNavPolicy
    d = golden("unreal174.npz")
    seed = int(d["seed"][0])
    pol = GoalNavPolicy(3, 4, (174, 174), recurrent=True, unreal=True)
    sd = {**seeded_reference_state((174, 174), seed + 1), **seeded_unreal_state((174, 174), seed)}
    g = torch.Generator().manual_seed(seed)
    for k, shape in (("weight_ih_l0", (2048, 517)), ("weight_hh_l0", (2048, 512)), ("bias_ih_l0", (2048,)),
                     ("bias_hh_l0", (2048,))):
        sd["rnn.inner." + k] = ((torch.rand(shape, generator=g) * 2 - 1) * 0.044).numpy()
    pol.load_reference_state_dict(sd)
    rng = np.random.RandomState(seed)
    B, T = d["h"].shape[:2]
    rng.rand(B, T, 512)
    rng.randn(*d["q"].shape)
    R = d["rp_logits"].shape[0]
    image = torch.as_tensor(rng.randint(0, 256, size=(R, 3, 174, 174, 3)).astype(np.uint8)).cuda()
    goal = torch.as_tensor(rng.randint(0, 256, size=(R, 3, 174, 174, 3)).astype(np.uint8)).cuda()
    logits = pol.reward_prediction(((image, goal), None))
    _close(logits.detach().cpu().numpy(), d["rp_logits"], 1e-5, "rp logits")
    (logits * torch.as_tensor(d["drp"]).cuda()).sum().backward()
    g = pol.net.to_reference(pol.params.grad)
    for k in ("rp.1.weight", "rp.1.bias"):
        _close(g[k].numpy(), d["g:" + k], 1e-4, k)
    assert g["conv_base.0.0.weight"].abs().max() > 0  # through the trunk
    pol.params.grad = None
    Bp, Tp = 3, 4
    img = torch.randint(0, 256, (Bp, Tp, 174, 174, 3), dtype=torch.uint8).cuda()
    q, (h, c) = pol.pixel_control(((img, img.flip(0)), None))
    assert q.shape == (Bp, Tp, 4, 42, 42) and h.shape == (Bp, 1, 512)
    assert torch.isfinite(q).all()
    (q * torch.randn_like(q)).sum().backward()
    g = pol.net.to_reference(pol.params.grad)
    assert g["pc_value.0.0.weight"].abs().max() > 0 and g["rnn.inner.weight_hh_l0"].abs().max() > 0
    assert g["shared_base.0.0.weight"].abs().max() > 0
    assert not g["pc_action.0.0.weight"].any() and not g["pc_action.0.2.bias"].any()
