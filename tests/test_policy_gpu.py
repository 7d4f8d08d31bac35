"""Policy forward/backward HIP kernels vs the reference modules' goldens and the torch
fp32 CPU oracle. Tolerances: logits/values/features rtol 1e-5 (north-star bar);
parameter gradients rtol 1e-4 of each tensor's scale (long fp32 reductions summed in a
different order)."""
import ctypes

import numpy as np
import pytest
import torch

from oracle import a2c as oa2c
from oracle.policy import GoalNetOracle, frames_to_float, seeded_reference_state

pytestmark = pytest.mark.gpu


def _ref_state(d):
    return {k[2:]: d[k] for k in d.files if k.startswith("w:")}


def _close(a, b, rtol, what):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    err = np.abs(a - b).max() / scale
    assert err <= rtol, "%s: max err %.3g of scale %.3g" % (what, err, scale)


def run_forward(net, params, image, goal):
    from vnav.policy import frames_from_batch
    n = image.shape[0]
    acts = net.new_acts(n)
    out = torch.zeros((n, 8), dtype=torch.float32, device="cuda")
    net.forward(params, frames_from_batch(image, goal), n, acts, n, 0, out)
    return out, acts


def x5_of(net, acts, n):
    return net.x5(acts, n)


def _act_sizes(net):
    h, w = net.frame_hw
    o1 = ((h - 7) // 4 + 1, (w - 7) // 4 + 1)
    o2 = ((o1[0] - 4) // 2 + 1, (o1[1] - 4) // 2 + 1)
    o3 = ((o2[0] - 4) // 2 + 1, (o2[1] - 4) // 2 + 1)
    return [2 * o1[0] * o1[1] * 32, 2 * o2[0] * o2[1] * 32, o3[0] * o3[1] * 64, o3[0] * o3[1] * 32, 512]


def test_forward_matches_reference_84(golden):
    from vnav.policy import PolicyNet
    d = golden("policy84.npz")
    net = PolicyNet((84, 84), 4)
    params = net.from_reference(_ref_state(d))
    img = torch.as_tensor(d["image"].reshape(-1, 84, 84, 3)).cuda()
    gl = torch.as_tensor(d["goal"].reshape(-1, 84, 84, 3)).cuda()
    out, acts = run_forward(net, params, img, gl)
    out = out.cpu().numpy()
    _close(out[:, :4], d["logits"].reshape(-1, 4), 1e-5, "logits")
    _close(out[:, 4:5], d["value"].reshape(-1, 1), 1e-5, "value")
    _close(x5_of(net, acts, img.shape[0]).cpu().numpy(), d["features"].reshape(-1, 512), 1e-5, "features")


def test_forward_matches_reference_174(golden):
    from vnav.policy import PolicyNet
    d = golden("policy174.npz")
    net = PolicyNet((174, 174), 4)
    params = net.from_reference(seeded_reference_state((174, 174), int(d["seed"][0])))
    img = torch.as_tensor(d["image"].reshape(-1, 174, 174, 3)).cuda()
    gl = torch.as_tensor(d["goal"].reshape(-1, 174, 174, 3)).cuda()
    out, acts = run_forward(net, params, img, gl)
    out = out.cpu().numpy()
    _close(out[:, :4], d["logits"].reshape(-1, 4), 1e-5, "logits")
    _close(out[:, 4:5], d["value"].reshape(-1, 1), 1e-5, "value")


def loss_grad_dev(out, actions, rets, vc=0.5, ec=0.01):
    from vnav import _lib
    lib = _lib.load()
    n = out.shape[0]
    dout = torch.zeros_like(out)
    stats = torch.zeros(4, dtype=torch.float32, device="cuda")
    _lib.check(lib.vn_a2c_loss_grad(_lib.ptr(out), _lib.ptr(actions), _lib.ptr(rets), n, 4, ctypes.c_float(vc),
                                    ctypes.c_float(ec), _lib.ptr(dout), _lib.ptr(stats),
                                    _lib.stream_ptr(out.device)), "loss_grad")
    return dout, stats


def test_backward_matches_reference_84(golden):
    from vnav.policy import PolicyNet, frames_from_batch
    d = golden("policy84.npz")
    net = PolicyNet((84, 84), 4)
    params = net.from_reference(_ref_state(d))
    img = torch.as_tensor(d["image"].reshape(-1, 84, 84, 3)).cuda()
    gl = torch.as_tensor(d["goal"].reshape(-1, 84, 84, 3)).cuda()
    n = img.shape[0]
    out, acts = run_forward(net, params, img, gl)
    actions = torch.as_tensor(d["actions"]).cuda()
    rets = torch.as_tensor(d["returns"]).cuda()
    dout, stats = loss_grad_dev(out, actions, rets)
    grads = torch.empty_like(params)
    ws = torch.empty(net.workspace_floats(n), dtype=torch.float32, device="cuda")
    net.backward(params, frames_from_batch(img, gl), n, acts, n, dout, grads, ws)
    g = net.to_reference(grads)
    for k, v in g.items():
        _close(v.numpy(), d["g:" + k], 1e-4, k)
    s = stats.cpu().numpy() / n
    loss = 0.5 * s[0] + s[1] - 0.01 * s[2]
    np.testing.assert_allclose(loss, d["loss"][0], rtol=1e-5)


def test_autograd_policy_vs_torch_oracle():
    """GoalNavPolicy through torch.autograd (custom Function over the HIP kernels) vs the
    CPU oracle at a larger batch, random weights/biases, both input formats."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(0)
    pol = GoalNavPolicy(3, 4, (84, 84))
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    ref = GoalNetOracle((84, 84)).load_reference(pol.reference_state_dict())
    B, T = 4, 5
    rng = np.random.RandomState(1)
    img = torch.as_tensor(rng.randint(0, 256, size=(B, T, 84, 84, 3)).astype(np.uint8))
    gl = torch.as_tensor(rng.randint(0, 256, size=(B, T, 84, 84, 3)).astype(np.uint8))
    logits, value, _ = pol(((img.cuda(), gl.cuda()), None), None, None)
    actions = torch.as_tensor(rng.randint(0, 4, size=B * T))
    rets = torch.as_tensor(rng.randn(B * T).astype(np.float32))
    loss, _ = oa2c.loss(logits.reshape(-1, 4), value.reshape(-1), actions.cuda(), rets.cuda())
    loss.backward()
    rl, rv = ref(frames_to_float(img.reshape(-1, 84, 84, 3)), frames_to_float(gl.reshape(-1, 84, 84, 3)))
    _close(logits.detach().cpu().reshape(-1, 4), rl.detach(), 1e-5, "logits")
    _close(value.detach().cpu().reshape(-1, 1), rv.detach(), 1e-5, "value")
    rloss, _ = oa2c.loss(rl, rv.view(-1), actions, rets)
    rloss.backward()
    mine = pol.net.to_reference(pol.params.grad)
    names = {"shared_base.0.0": ref.conv1, "shared_base.0.2": ref.conv2, "conv_base.0.0": ref.conv3,
             "conv_base.0.2": ref.conv4, "conv_merge.0.1": ref.fc, "policy_logits.0": ref.policy_logits,
             "critic.0": ref.critic}
    for k, mod in names.items():
        _close(mine[k + ".weight"].numpy(), mod.weight.grad.numpy(), 1e-4, k + ".weight")
        _close(mine[k + ".bias"].numpy(), mod.bias.grad.numpy(), 1e-4, k + ".bias")
    # float CHW input (the reference wrapper format) gives the same outputs
    lf, vf, _ = pol(((frames_to_float(img).cuda(), frames_to_float(gl).cuda()), None), None, None)
    _close(lf.detach().cpu(), logits.detach().cpu(), 1e-5, "f32 input logits")


def _policy_174(seed):
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(seed)
    pol = GoalNavPolicy(3, 4, (174, 174))
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    return pol


def _grads_174(pol, img, gl, actions, rets):
    pol.params.grad = None
    logits, value, _ = pol(((img.cuda(), gl.cuda()), None), None, None)
    loss, _ = oa2c.loss(logits.reshape(-1, 4), value.reshape(-1), actions.cuda(), rets.cuda())
    loss.backward()
    return logits.detach().cpu().reshape(-1, 4), value.detach().cpu().reshape(-1), pol.params.grad.clone()


def test_autograd_policy_174_vs_torch_oracle():
    """The reference's unmodified 174x174 topology (42x42 -> 20x20 -> 9x9, Linear(2592)):
    forward and every parameter gradient vs the float64 CPU oracle. Inputs are chosen with
    no conv1/conv2 pre-activation within 5e-7 of zero: a ReLU tie flipped by fp32 rounding
    moves its conv gradient by ~1e-3 of the scale (the gradients are sums with heavy
    cancellation), a tie rather than an error (test_policy_174_large_batch_consistency
    covers large batches against the GPU's own small-batch gradients)."""
    import torch.nn.functional as F
    pol = _policy_174(3)
    ref = GoalNetOracle((174, 174)).load_reference(pol.reference_state_dict()).double()
    n = 4
    for seed in range(4, 400):
        rng = np.random.RandomState(seed)
        img = torch.as_tensor(rng.randint(0, 256, size=(n, 1, 174, 174, 3)).astype(np.uint8))
        gl = torch.as_tensor(rng.randint(0, 256, size=(n, 1, 174, 174, 3)).astype(np.uint8))
        fi = frames_to_float(img.reshape(-1, 174, 174, 3)).double()
        fg = frames_to_float(gl.reshape(-1, 174, 174, 3)).double()
        with torch.no_grad():
            z1 = [ref.conv1(v) for v in (fi, fg)]
            z2 = [ref.conv2(F.relu(z)) for z in z1]
            margin = min(float(z.abs().min()) for z in z1 + z2)
        if margin > 5e-7:
            break
    assert margin > 5e-7
    actions = torch.as_tensor(rng.randint(0, 4, size=n))
    rets = torch.as_tensor(rng.randn(n).astype(np.float32))
    logits, value, grad = _grads_174(pol, img, gl, actions, rets)
    rl, rv = ref(fi, fg)
    _close(logits, rl.detach(), 1e-5, "logits")
    _close(value, rv.detach().view(-1), 1e-5, "value")
    rloss, _ = oa2c.loss(rl, rv.view(-1), actions, rets.double())
    rloss.backward()
    mine = pol.net.to_reference(grad)
    names = {"shared_base.0.0": ref.conv1, "shared_base.0.2": ref.conv2, "conv_base.0.0": ref.conv3,
             "conv_base.0.2": ref.conv4, "conv_merge.0.1": ref.fc, "policy_logits.0": ref.policy_logits,
             "critic.0": ref.critic}
    errs = {}
    for k, mod in names.items():
        for kind in ("weight", "bias"):
            b = getattr(mod, kind).grad.numpy()
            errs[k + "." + kind] = np.abs(mine[k + "." + kind].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
    bad = {k: "%.3g" % e for k, e in errs.items() if e > 1e-4}
    assert not bad, bad


def test_policy_174_large_batch_consistency():
    """128 samples at 174x174 in one batch — the banded conv1 kernels (5 bands per frame)
    and the 8-wave conv2 input gradient wrap their persistent grids — against the same
    samples in 4 batches of 32 (no grid wraps): per-sample outputs agree, and the batch
    gradient equals the mean of the small-batch gradients (identical ReLU masks: every
    forward kernel computes a sample independently of the batch; batches of <= 16 samples
    take the few-env kernels of vn_skinny.h, which sum in another order, so the parts stay
    above that size)."""
    pol = _policy_174(5)
    B = 128
    rng = np.random.RandomState(7)
    img = torch.as_tensor(rng.randint(0, 256, size=(B, 1, 174, 174, 3)).astype(np.uint8))
    gl = torch.as_tensor(rng.randint(0, 256, size=(B, 1, 174, 174, 3)).astype(np.uint8))
    actions = torch.as_tensor(rng.randint(0, 4, size=B))
    rets = torch.as_tensor(rng.randn(B).astype(np.float32))
    logits, value, grad = _grads_174(pol, img, gl, actions, rets)
    parts = [_grads_174(pol, img[k:k + 32], gl[k:k + 32], actions[k:k + 32], rets[k:k + 32]) for k in range(0, B, 32)]
    _close(logits, torch.cat([p[0] for p in parts]), 1e-6, "logits")
    _close(value, torch.cat([p[1] for p in parts]), 1e-6, "value")
    gmean = sum(p[2].double() for p in parts) / len(parts)
    mine, ref = pol.net.to_reference(grad), pol.net.to_reference(gmean.float())
    bad = {}
    for k in ref:
        b = ref[k].numpy().astype(np.float64)
        e = np.abs(mine[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad


@pytest.mark.parametrize("hw,N", [((174, 174), 20480), ((300, 400), 4608)])
def test_policy_offsets_past_2g_elements(hw, N):
    """20480 samples at 174x174 (4608 at 300x400, config C5) in one batch: conv1's output
    alone is 2.31e9 (2.16e9) floats, so every
    kernel addresses activations past int32 element offsets. The first and last 64 samples
    give the outputs they give alone, and the gradient of a loss on the last 64 samples,
    taken inside the full batch (zero output gradient elsewhere), equals that loss's
    gradient run alone — both to 1e-5 of scale (the north-star bar; small batches split K,
    so the long sums run in another order). An addressing error would be O(1)."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(9)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    k = 64
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((k, 1, 4), device="cuda", generator=g)
    cv = torch.randn((k, 1, 1), device="cuda", generator=g)

    def run(a, b, sl):
        pol.params.grad = None
        logits, value, _ = pol(((a, b), None), None, None)
        ((logits[sl] * cl).sum() + (value[sl] * cv).sum()).backward()
        return logits.detach(), value.detach(), pol.params.grad.clone()

    logits, value, grad = run(img, gl, slice(N - k, N))
    l_last, v_last, g_last = run(img[-k:], gl[-k:], slice(0, k))
    _close(logits[-k:].cpu(), l_last.cpu(), 1e-5, "logits of the last samples")
    _close(value[-k:].cpu(), v_last.cpu(), 1e-5, "values of the last samples")
    l_first, v_first, _ = run(img[:k], gl[:k], slice(0, k))
    _close(logits[:k].cpu(), l_first.cpu(), 1e-5, "logits of the first samples")
    _close(value[:k].cpu(), v_first.cpu(), 1e-5, "values of the first samples")
    mine, ref = pol.net.to_reference(grad), pol.net.to_reference(g_last)
    bad = {}
    for key in ref:
        b = ref[key].numpy().astype(np.float64)
        e = np.abs(mine[key].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[key] = "%.3g" % e
    assert not bad, bad


def test_row_gather_equals_dense_batch():
    import vnav
    from vnav.policy import PolicyNet, frames_from_batch, frames_from_rows
    sc = [vnav.synthetic_scene(k) for k in range(2)]
    env = vnav.VectorEnv(sc, 50, seed=4)
    (img, gl) = env.observe()
    net = PolicyNet((84, 84), 4)
    params = net.init_params(3)
    out1, _ = run_forward(net, params, img, gl)
    arena, fb, _, _ = env.frame_arena()
    acts = net.new_acts(50)
    out2 = torch.zeros_like(out1)
    net.forward(params, frames_from_rows(arena, fb, env._info["img_row"], env._info["goal_row"]), 50, acts, 50, 0, out2)
    assert torch.equal(out1, out2)


def test_a2c_kernels_vs_oracle():
    from vnav import _lib
    lib = _lib.load()
    st = _lib.stream_ptr(torch.device("cuda", 0))
    T, E = 7, 33
    g = torch.Generator().manual_seed(0)
    rewards = (torch.rand(T, E, generator=g) < 0.2).float()
    dones = torch.rand(T, E, generator=g) < 0.1
    boot = torch.randn(E, 8, generator=g)
    R = torch.zeros(T * E, device="cuda")
    rw_d, dn_d, bt_d = rewards.cuda(), dones.cuda(), boot.cuda()  # keep device tensors alive
    _lib.check(lib.vn_a2c_returns(_lib.ptr(rw_d), _lib.ptr(dn_d), _lib.ptr(bt_d), T, E, 4,
                                  ctypes.c_float(0.99), _lib.ptr(R), st), "returns")
    vext = torch.zeros(T + 1, E)
    vext[T] = boot[:, 4]
    Rref = oa2c.returns(rewards, dones, vext, 0.99)
    _close(R.cpu().view(T, E), Rref, 1e-6, "returns")
    # loss gradient vs autograd on the oracle loss
    N = T * E
    out = torch.randn(N, 8, generator=g)
    acts = torch.randint(0, 4, (N,), generator=g)
    out_d, acts_d, R_d = out.cuda(), acts.int().cuda(), Rref.view(-1).cuda()
    dout, stats = loss_grad_dev(out_d, acts_d, R_d)
    lg = out[:, :4].clone().requires_grad_(True)
    v = out[:, 4].clone().requires_grad_(True)
    loss, parts = oa2c.loss(lg, v, acts, Rref.view(-1))
    loss.backward()
    _close(dout.cpu()[:, :4], lg.grad, 1e-5, "dlogits")
    _close(dout.cpu()[:, 4], v.grad, 1e-5, "dvalue")
    s = stats.cpu() / N
    np.testing.assert_allclose(s[0].item(), parts["value_loss"].item(), rtol=1e-5)
    np.testing.assert_allclose(s[1].item(), parts["action_loss"].item(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(s[2].item(), parts["entropy"].item(), rtol=1e-5)
    # clip + RMSprop vs the torch restatement, two steps
    P = 10001
    p0 = torch.randn(P, generator=g)
    gr = torch.randn(P, generator=g) * 0.01
    pd, sq = p0.clone().cuda(), torch.zeros(P, device="cuda")
    gr_d = gr.cuda()
    part = torch.zeros(512, dtype=torch.float64, device="cuda")
    sc = torch.zeros(2, device="cuda")
    pr, sr = [p0.clone()], [torch.zeros(P)]
    for it in range(2):
        _lib.check(lib.vn_grad_norm(_lib.ptr(gr_d), P, ctypes.c_float(0.5), ctypes.c_float(0.5), _lib.ptr(part),
                                    _lib.ptr(sc), st), "norm")
        _lib.check(lib.vn_rmsprop_step(_lib.ptr(pd), _lib.ptr(gr_d), _lib.ptr(sq), P, ctypes.c_float(0.5),
                                       _lib.ptr(sc), ctypes.c_float(7e-4), ctypes.c_float(0.99),
                                       ctypes.c_float(1e-5), st), "rmsprop")
        norm = oa2c.clip_and_rmsprop(pr, [gr * 0.5], sr, 7e-4)
        np.testing.assert_allclose(sc[0].item(), norm.item(), rtol=1e-5)
    _close(pd.cpu(), pr[0], 1e-6, "params after RMSprop")


def test_sampling_distribution():
    from vnav import _lib
    from oracle import philox
    lib = _lib.load()
    n = 200000
    logits = torch.tensor([[0.5, -1.0, 2.0, 0.0]]).repeat(n, 1)
    out = torch.zeros(n, 8)
    out[:, :4] = logits
    a = torch.zeros(n, dtype=torch.int32, device="cuda")
    out_d = out.cuda()
    _lib.check(lib.vn_policy_sample(_lib.ptr(out_d), n, 4, ctypes.c_uint64(5), ctypes.c_uint64(9), _lib.ptr(a),
                                    None, None, None, _lib.stream_ptr(a.device)), "sample")
    a = a.cpu().numpy()
    p = torch.softmax(logits[0], 0).numpy()
    freq = np.bincount(a, minlength=4) / n
    assert np.abs(freq - p).max() < 5e-3
    # the inverse-CDF draw restated on the host (Philox stream 3) picks the same actions
    r = philox.philox4x32_10(np.arange(n), 9, 0, philox.STREAM_POLICY, 5, 0)[0]
    u = (r >> 8).astype(np.float64) * (1.0 / 16777216.0)
    cdf = np.cumsum(p)
    ref = np.minimum(np.searchsorted(cdf[:-1], u, side="right"), 3)
    assert (ref == a).mean() > 0.999


def test_policy_refuses_mismatched_frames_and_moves_host_frames():
    """Frames the kernels would misread (another geometry, dtype, layout, batch) raise
    before launch; host-resident frames are moved to the policy's device (same outputs)."""
    import vnav
    pol = vnav.GoalNavPolicy(frame_hw=(84, 84), seed=3)
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (2, 3, 84, 84, 3), generator=g, dtype=torch.uint8)
    goal = torch.randint(0, 256, (2, 3, 84, 84, 3), generator=g, dtype=torch.uint8)
    on_dev = pol(((img.cuda(), goal.cuda()), None))[0]
    on_host = pol(((img, goal), None))[0]
    assert torch.equal(on_dev, on_host)
    bad = [(torch.zeros((2, 3, 174, 174, 3), dtype=torch.uint8), torch.zeros((2, 3, 174, 174, 3), dtype=torch.uint8)),
           (img.cuda(), goal.cuda()[:1]),
           (img.cuda().to(torch.int32), goal.cuda().to(torch.int32)),
           (img.cuda()[..., :2], goal.cuda()[..., :2])]
    for a, b in bad:
        with pytest.raises(ValueError):
            pol(((a, b), None))
    net = pol.net
    with pytest.raises(ValueError):  # non-contiguous batch straight into the autograd function
        from vnav.policy import _GoalNavFunction
        x = torch.zeros((4, 84, 84, 3), dtype=torch.uint8, device="cuda")[::2]
        _GoalNavFunction.apply(pol.params, x, x, net)


def test_feedforward_gradient_of_heads_without_output_is_zero():
    """The feed-forward policy's backward writes the trunk and head blocks; an aux policy's deconv
    heads take no gradient from the policy output and their block must come back exactly zero
    (it was uninitialised memory until round 6: non-finite in ~1/256 of the entries,
    tools/nan_stress.py), and repeated backward passes are bitwise equal."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(43)
    hw = (174, 174)
    pol = GoalNavPolicy(3, 4, hw, recurrent=False, aux=True)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    N = 77
    g = torch.Generator(device="cuda").manual_seed(19)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    outs = []
    for _ in range(2):
        junk = torch.full((pol.params.numel() * 4,), float("nan"), device="cuda")  # poison the allocator's cache
        del junk
        pol.params.grad = None
        logits, value, _ = pol(((img, gl), None), None, None)
        ((logits * cl).sum() + value.sum()).backward()
        torch.cuda.synchronize()
        outs.append(pol.params.grad.clone())
    gr = outs[0]
    assert torch.isfinite(gr).all()
    X = pol.net.aux_layout
    assert float(gr[X["w1"]:X["b2"] + 8].abs().max()) == 0.0
    assert torch.equal(outs[0], outs[1])
