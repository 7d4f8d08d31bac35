"""BigHouseModel's UNREAL heads (models/bignet.py:77-111) on the HIP path: pixel control
(pc_base product, pc_value / pc_action as one 32 -> 8 transposed conv on the 9x9 map, the
value/action combination on a 20x20 map) and reward prediction (Linear on three frames'
conv_base maps, 3 * 7*7*32 inputs at 84x84), through the C ABI.
  * vs the REFERENCE modules' goldens (tests/golden/bighouse_unreal84.npz);
  * vs the fp64 restatement (oracle/policy.py) on batches that take several tiles;
  * the 20-cell pixel-control loss vs oracle/unreal.py (parity unpinned, as for the 42-cell one);
  * BigHousePolicy(unreal=True) and A2CTrainer(arch="bighouse", unreal=True) end to end.
Tolerances: outputs rtol 1e-5 of scale, gradients 1e-4 of scale (as test_unreal_gpu.py); the
pc_action branch's gradients are exactly zero, as torch computes them."""
import ctypes

import numpy as np
import pytest
import torch

from oracle.policy import (BIGHOUSE_UNREAL_PARAM_ORDER, bighouse_pixel_control, bighouse_reward_prediction,
                           seeded_bighouse_state, seeded_bighouse_unreal_state)

pytestmark = pytest.mark.gpu


def _close(a, b, rtol, what):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err <= rtol, "%s: max err %.3g of scale %.3g" % (what, err, scale)


def _net(recurrent=False):
    from vnav.policy import PolicyNet
    return PolicyNet((84, 84), 4, device="cuda:0", arch="bighouse", recurrent=recurrent, unreal=True)


def _nhwc(feats):
    """[R, 3, 32, 7, 7] (conv_base of 3 frames) -> [R, 3 * 7 * 7 * 32]."""
    return feats.permute(0, 1, 3, 4, 2).reshape(feats.shape[0], -1).contiguous()


def _run(net, params, h, dq, feats_nhwc, drp, dh_init=None):
    n = h.shape[0]
    A = net.num_actions
    ws = torch.empty(net.pc_workspace_floats(), dtype=torch.float32, device="cuda")
    pcb, a1, p2, q = net.pc_buffers(n)
    assert a1 is None and p2.shape == (n, 20, 20, 8) and q.shape == (n, 20, 20, A)
    net.pc_forward(params, h, n, pcb, a1, p2, q, ws)
    q_out = q.clone()
    masks = {"pc_base": (pcb > 0).permute(0, 3, 1, 2).cpu(), "pc_value": (p2[..., :A] > 0).permute(0, 3, 1, 2).cpu(),
             "pc_action": (p2[..., A:A + 1] > 0).permute(0, 3, 1, 2).cpu()}
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


def test_bighouse_unreal_layout():
    net = _net()
    U = net.unreal_layout
    assert U["w2"] == U["b2"] == U["rp_w"]  # no second layer
    assert U["b1"] - U["w1"] == 32 * 16 * 8 and U["w2"] - U["b1"] == 8
    assert net.n_params == U["rp_b"] + 4
    v = net.views(net.init_params(seed=1))["unreal"]
    assert "w2" not in v and v["rp_w"].shape == (3, 3 * 1568)
    assert not v["w1"][..., 5:].any() and v["w1"][..., 4].abs().max() <= 0.25


def test_bighouse_unreal_heads_match_reference(golden):
    d = golden("bighouse_unreal84.npz")
    seed = int(d["seed"][0])
    net = _net()
    sd = {**seeded_bighouse_state(0), **seeded_bighouse_unreal_state(seed)}
    params = net.from_reference(sd)
    back = net.to_reference(params)
    for k in BIGHOUSE_UNREAL_PARAM_ORDER:  # the layout round-trips the reference's tensors
        np.testing.assert_array_equal(back[k].numpy(), sd[k], err_msg=k)
    B, T = d["h"].shape[:2]
    n = B * T
    h = torch.as_tensor(d["h"]).reshape(n, 512).cuda()
    dq = torch.as_tensor(d["dq"]).reshape(n, 4, 20, 20).permute(0, 2, 3, 1).cuda()
    feats = torch.as_tensor(d["rp_features"])
    q, dh, logits, dx, g, _ = _run(net, params, h, dq, _nhwc(feats).cuda(), torch.as_tensor(d["drp"]).cuda())
    _close(q.permute(0, 3, 1, 2).cpu().numpy(), d["q"].reshape(n, 4, 20, 20), 1e-5, "q")
    _close(logits.cpu().numpy(), d["rp_logits"], 1e-5, "rp logits")
    _close(dh.cpu().numpy(), d["dh"].reshape(n, 512), 1e-4, "dh")
    R = feats.shape[0]
    _close(dx.cpu().numpy(), _nhwc(torch.as_tensor(d["d_rp_features"])).numpy().reshape(R, -1), 1e-5,
           "d rp features")
    for name in BIGHOUSE_UNREAL_PARAM_ORDER:
        got = g[name].numpy()
        if name == "pc_base.0.0.weight":
            got = got[::16]
        want = d["g:" + name]
        if name.startswith("pc_action"):
            np.testing.assert_array_equal(got, 0.0, err_msg=name)
            assert not np.any(want)
        else:
            _close(got, want, 1e-4, name)


@pytest.mark.parametrize("n,R", [(37, 50), (130, 7)])
def test_bighouse_unreal_heads_vs_fp64_oracle(n, R):
    net = _net()
    params = net.init_params(seed=3)
    v = net.views(params)
    with torch.no_grad():  # biases off zero so the bias paths and ReLU masks are exercised
        u = v["unreal"]
        g = torch.Generator(device="cpu").manual_seed(4)
        for k in ("pc_b", "b1", "rp_b"):
            u[k].copy_((torch.rand(u[k].shape, generator=g) * 0.1 - 0.05).to(u[k].device))
        u["b1"][5:] = 0.0
        u["rp_b"][3] = 0.0
    ref = {k: t.double().requires_grad_() for k, t in net.to_reference(params).items()
           if k in BIGHOUSE_UNREAL_PARAM_ORDER}
    torch.manual_seed(5)
    h = torch.rand(n, 512) * 2.0 - 0.5
    dq = torch.randn(n, 4, 20, 20)
    feats = torch.randn(R, 3, 32, 7, 7) * 0.1
    drp = torch.randn(R, 3)
    dh0 = torch.randn(n, 512)
    q, dh, logits, dx, g, masks = _run(net, params, h.cuda(), dq.permute(0, 2, 3, 1).cuda(), _nhwc(feats).cuda(),
                                       drp.cuda(), dh_init=dh0.cuda())
    h64 = h.double().requires_grad_()
    f64 = feats.double().requires_grad_()
    q_ref = bighouse_pixel_control(ref, h64, masks)  # the GPU's ReLU masks: no tie can flip between them
    l_ref = bighouse_reward_prediction(ref, f64)
    ((q_ref * dq.double()).sum() + (l_ref * drp.double()).sum()).backward()
    _close(q.permute(0, 3, 1, 2).cpu().numpy(), q_ref.detach().numpy(), 1e-5, "q")
    _close(logits.cpu().numpy(), l_ref.detach().numpy(), 1e-5, "rp logits")
    _close((dh.cpu() - dh0).numpy(), h64.grad.numpy(), 1e-4, "dh (accumulated)")
    _close(dx.cpu().numpy(), _nhwc(f64.grad).numpy(), 1e-5, "d rp features")
    for name in BIGHOUSE_UNREAL_PARAM_ORDER:
        if name.startswith("pc_action"):
            np.testing.assert_array_equal(g[name].numpy(), 0.0, err_msg=name)
        else:
            _close(g[name].numpy(), ref[name].grad.numpy(), 1e-4, name)


def test_pc_loss_kernel_20_cells_vs_oracle():
    """vn_unreal_pc_loss_grad_ex with the 20 x 20 map on 84x84 frames (centre 80x80 crop)."""
    from oracle import unreal
    from test_unreal_gpu import _loss_case
    from vnav import _lib
    lib = _lib.load()
    c = _loss_case(H=84, W=84, seed=9)
    T, E, S, A, C = c["T"], c["E"], c["S"], c["A"], 20
    p2 = torch.relu(torch.randn(((T + 1) * S, C, C, 8), generator=c["g"]) * 0.3)
    p2[..., A + 1:] = 0.0
    q = (p2[..., :A] + p2[..., A:A + 1]) - p2[..., A:A + 1]
    P = _lib.ptr
    d = {k: c[k].cuda() for k in ("arena", "rows_img", "rows_last", "actions", "dones")}
    dp2 = p2.cuda()
    stats = torch.zeros(1, device="cuda")
    w = 0.05
    # the 42-cell entry point refuses 84x84 frames (a 168-px crop)
    assert lib.vn_unreal_pc_loss_grad(P(dp2), P(d["actions"]), P(d["dones"]), P(d["arena"]), 84 * 84 * 3, 84, 84,
                                      P(d["rows_img"]), P(d["rows_last"]), T, E, S, A, ctypes.c_float(0.9),
                                      ctypes.c_float(w), P(stats), None) != 0
    _lib.check(lib.vn_unreal_pc_loss_grad_ex(P(dp2), C, P(d["actions"]), P(d["dones"]), P(d["arena"]), 84 * 84 * 3,
                                             84, 84, P(d["rows_img"]), P(d["rows_last"]), T, E, S, A,
                                             ctypes.c_float(0.9), ctypes.c_float(w), P(stats), None), "pc loss 20")
    torch.cuda.synchronize()
    rows = torch.cat((c["rows_img"].view(T, E)[:, :S], c["rows_last"][None, :S])).long()
    loss, grad = unreal.pc_loss(q.view(T + 1, S, C, C, A), c["arena"][rows], c["actions"].view(T, E)[:, :S],
                                c["dones"][:, :S])
    want = torch.zeros((T + 1, S, C, C, 8), dtype=torch.float64)
    want[..., :A] = grad * (p2.view(T + 1, S, C, C, 8)[..., :A] > 0)
    _close(dp2.cpu().view(T + 1, S, C, C, 8).numpy() / w, want.numpy(), 1e-5, "dp2")
    np.testing.assert_allclose(stats.item() / (T * S * C * C), loss.item(), rtol=1e-5)


def test_bighouse_policy_reward_prediction_and_pixel_control(golden):
    """BigHousePolicy(unreal=True).reward_prediction on the golden's uint8 frames (conv_base from
    the golden's seed + 1) vs the REFERENCE module, its rp gradients and the trunk gradient;
    pixel_control's Q maps [B,T,A,20,20] and gradients reach the LSTM and pc_value, never pc_action."""
    from vnav.policy import BigHousePolicy
    d = golden("bighouse_unreal84.npz")
    seed = int(d["seed"][0])
    pol = BigHousePolicy(3, 4, recurrent=True, unreal=True)
    sd = {**seeded_bighouse_state(seed + 1), **seeded_bighouse_unreal_state(seed)}
    g = torch.Generator().manual_seed(seed)
    for k, shape in (("weight_ih_l0", (2048, 517)), ("weight_hh_l0", (2048, 512)), ("bias_ih_l0", (2048,)),
                     ("bias_hh_l0", (2048,))):
        sd["rnn.inner." + k] = ((torch.rand(shape, generator=g) * 2 - 1) * 0.044).numpy()
    pol.load_reference_state_dict(sd)
    image = torch.as_tensor(d["image"]).cuda()  # [R, 3, 84, 84, 3] uint8
    logits = pol.reward_prediction((image, None))
    _close(logits.detach().cpu().numpy(), d["rp_logits"], 1e-5, "rp logits")
    (logits * torch.as_tensor(d["drp"]).cuda()).sum().backward()
    gr = pol.net.to_reference(pol.params.grad)
    for k in ("rp.weight", "rp.bias"):
        _close(gr[k].numpy(), d["g:" + k], 1e-4, k)
    assert gr["conv_base.0.0.weight"].abs().max() > 0  # through the trunk (dX3 into backward_ex)
    pol.params.grad = None
    Bp, Tp = 3, 4
    img = torch.randint(0, 256, (Bp, Tp, 84, 84, 3), dtype=torch.uint8).cuda()
    q, (h, c) = pol.pixel_control((img, None))
    assert q.shape == (Bp, Tp, 4, 20, 20) and h.shape == (Bp, 1, 512)
    assert torch.isfinite(q).all()
    (q * torch.randn_like(q)).sum().backward()
    gr = pol.net.to_reference(pol.params.grad)
    assert gr["pc_value.0.0.weight"].abs().max() > 0 and gr["rnn.inner.weight_hh_l0"].abs().max() > 0
    assert gr["conv_base.0.0.weight"].abs().max() > 0
    assert not gr["pc_action.0.0.weight"].any() and not gr["pc_action.0.0.bias"].any()


def test_bighouse_trainer_unreal():
    """A2CTrainer(arch='bighouse', unreal=True) on 84x84 frames: pc (20 cells) / rp / vr losses
    finite and reported, pc_action never moves, pc_value / pc_base / rp do; the hipGraph replay
    is bit-identical to the eager updates."""
    import vnav
    from oracle.frames import synth_frames
    from oracle.graph import h5_tables
    graph, spd, _ = h5_tables(np.ones((3, 3), dtype=bool))
    scene = vnav.scene_from_arrays(graph, spd, synth_frames(3, np.arange(len(graph)), (84, 84, 3)))

    def run(graph, source="rollout"):
        env = vnav.VectorEnv([scene], 16, seed=2, max_episode_steps=30, tasks=[(0, 5)])
        tr = vnav.A2CTrainer(env, num_steps=5, seed=3, max_time_steps=1e9, recurrent=True, arch="bighouse",
                             unreal=True, unreal_envs=8, cuda_graph=graph, unreal_source=source)
        p0 = tr.params.detach().clone()
        return tr, p0, [tr.step(sync=True) for _ in range(3)]

    tr, p0, ms = run(False)
    assert tr.pc_cells == 20
    for m in ms:
        for k in ("pc_loss", "rp_loss", "vr_loss", "value_loss"):
            assert np.isfinite(m[k]), (k, m)
        assert m["pc_loss"] > 0
    v0, v1 = tr.net.views(p0)["unreal"], tr.net.views(tr.params)["unreal"]
    A = tr.net.num_actions
    assert torch.equal(v0["w1"][..., A:], v1["w1"][..., A:]) and torch.equal(v0["b1"][A:], v1["b1"][A:])
    assert not torch.equal(v0["w1"][..., :A], v1["w1"][..., :A])
    assert not torch.equal(v0["pc_w"], v1["pc_w"]) and not torch.equal(v0["rp_w"], v1["rp_w"])
    trg, _, msg = run(True)
    assert torch.equal(tr.params, trg.params)
    for x, y in zip(ms, msg):
        for k in ("rp_loss", "value_loss", "grad_norm"):
            assert x[k] == y[k], (k, x[k], y[k])
    trr, _, msr = run(False, "replay")
    for m in msr:
        assert np.isfinite(m["pc_loss"]) and np.isfinite(m["rp_loss"])


def test_bighouse_unreal_trainer_learns_on_small_scene():
    """A2CTrainer(arch='bighouse', unreal=True) on the BigHouseModel learning test's task
    (tests/test_bighouse_gpu.py): with the pixel-control / reward-prediction / value-replay losses
    added (20-cell pixel control on 84x84 frames) the policy still learns the fixed-goal task."""
    import vnav
    from oracle.frames import synth_frames
    from oracle.graph import h5_tables
    graph, spd, _ = h5_tables(np.ones((3, 3), dtype=bool))
    scene = vnav.scene_from_arrays(graph, spd, synth_frames(3, np.arange(len(graph)), (84, 84, 3)))
    env = vnav.VectorEnv([scene], 256, seed=1, max_episode_steps=60, tasks=[(0, 5)])
    tr = vnav.A2CTrainer(env, num_steps=20, seed=0, max_time_steps=1e9, recurrent=True, learning_rate=2e-3,
                         arch="bighouse", unreal=True)
    lengths, pc = [], []
    for u in range(800):
        m = tr.step(sync=(u < 20 or u >= 790))
        if "raw" not in m:
            lengths.append(m["episode_length"])
            pc.append(m["pc_loss"])
    early = np.nanmean(lengths[5:20])
    late = np.nanmean(lengths[-10:])
    assert np.isfinite(late) and late < 0.8 * early, (early, late)
    assert all(np.isfinite(pc))
