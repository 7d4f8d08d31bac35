"""Goal-frame deduplication (vn_goal_runs, include/vnav.h): shared_base runs on an env's
goal frame once per goal run (models/goal.py:88 runs it at every step; the goal frame is
constant within an episode), the backward sums a run's goal-map gradients before the conv2 /
conv1 backward.

* the run bookkeeping kernels (vn_goal_runs_step / vn_goal_runs_rollout) vs numpy;
* the policy forward with goal runs equals the forward without them bitwise (the
  frame-level kernels are batch-independent), and its backward's gradients match the fp64
  oracle (tests/test_prod_oracle_gpu.py's masked-oracle method) at 1e-4 of scale and the
  non-deduplicated backward at 1e-5;
* A2CTrainer with and without deduplication: the same rollout bitwise (outputs, actions,
  env transitions) and the same update gradients to 1e-5 of scale (LSTM + aux heads, 174x174;
  LSTM, 84x84);
* configurations without frame-list kernels refuse goal runs instead of ignoring them.
C5's 300x400 geometry takes goal runs through the banded conv2 input gradient, the f32 conv2
weight gradient and the row-limited generic conv2 forward product.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle.policy import GoalNetOracle, frames_to_float
from test_prod_oracle_gpu import _check_outputs, _err, _grads_vs_oracle, _gpu_masks, _loss_grad, _noisy_policy

pytestmark = pytest.mark.gpu


def _np_runs(dones):
    """Reference bookkeeping: run starts, per-sample goal delta, run lengths, start list."""
    T, E = dones.shape
    start = np.ones((T, E), dtype=bool)
    start[1:] = dones[:-1]
    delta = np.zeros((T, E), dtype=np.int32)
    for t in range(1, T):
        delta[t] = np.where(start[t], 0, delta[t - 1] - E)
    runlen = np.zeros((T, E), dtype=np.int32)
    for e in range(E):
        end = T - 1
        for t in range(T - 1, -1, -1):
            if dones[t, e]:
                end = t
            if start[t, e]:
                runlen[t, e] = end - t + 1
    return start, delta, runlen, np.flatnonzero(start.ravel())


def _step_runs(lib, _lib, dones, t, delta, lst, cnt):
    P = _lib.ptr
    E = dones.shape[1]
    _lib.check(lib.vn_goal_runs_step(P(dones[t - 1]) if t else None, P(delta[t - 1]) if t else None, E,
                                     P(delta[t]), P(lst[t]), P(cnt[t:t + 1]), _lib.stream_ptr(dones.device)),
               "vn_goal_runs_step")


@pytest.mark.parametrize("T,E,p", [(20, 4096, 0.02), (3, 17, 0.5), (5, 1000, 1.0), (4, 2500, 0.0)])
def test_goal_run_kernels_match_numpy(T, E, p):
    from vnav import _lib
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(T * E)
    dones = torch.rand((T, E), device="cuda", generator=g) < p
    delta = torch.full((T, E), 7, dtype=torch.int32, device="cuda")
    lst = torch.full((T, E), -1, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(T + 1, dtype=torch.int32, device="cuda")
    for t in range(T):
        _step_runs(lib, _lib, dones, t, delta, lst, cnt)
    all_list = torch.full((T * E,), -1, dtype=torch.int32, device="cuda")
    runlen = torch.zeros(T * E, dtype=torch.int32, device="cuda")
    _lib.check(lib.vn_goal_runs_rollout(_lib.ptr(dones), T, E, _lib.ptr(all_list), _lib.ptr(runlen),
                                        _lib.ptr(cnt[T:]), _lib.stream_ptr(dones.device)), "vn_goal_runs_rollout")
    torch.cuda.synchronize()
    start, d_ref, rl_ref, list_ref = _np_runs(dones.cpu().numpy())
    assert np.array_equal(delta.cpu().numpy(), d_ref)
    c = cnt.cpu().numpy()
    for t in range(T):
        assert c[t] == start[t].sum()
        assert np.array_equal(lst[t, :c[t]].cpu().numpy(), np.flatnonzero(start[t]))
    assert c[T] == len(list_ref)
    assert np.array_equal(all_list[:c[T]].cpu().numpy(), list_ref)
    assert np.array_equal(runlen.cpu().numpy()[list_ref], rl_ref.ravel()[list_ref])


def _rollout_batch(hw, T, E, seed, p_done=0.3):
    """Dense uint8 frames of a T x E rollout (time-major) whose goal frames change only after
    a done, with the dones."""
    h, w = hw
    g = torch.Generator(device="cuda").manual_seed(seed)
    N = T * E
    img = torch.randint(0, 256, (N, h, w, 3), dtype=torch.uint8, device="cuda", generator=g)
    dones = torch.rand((T, E), device="cuda", generator=g) < p_done
    pool = torch.randint(0, 256, (E * T, h, w, 3), dtype=torch.uint8, device="cuda", generator=g)
    gid = np.zeros((T, E), dtype=np.int64)
    d = dones.cpu().numpy()
    nxt = E
    gid[0] = np.arange(E)
    for t in range(1, T):
        for e in range(E):
            if d[t - 1, e]:
                gid[t, e] = nxt
                nxt += 1
            else:
                gid[t, e] = gid[t - 1, e]
    gl = pool[torch.as_tensor(gid.ravel(), device="cuda")].contiguous()
    return img, gl, dones


# the wide cases step enough envs for conv3's goal-aware product to run whole-K (>= 128 tiles,
# the bench's form; the narrow ones take its split-K form)
@pytest.mark.parametrize("hw,T,E", [((84, 84), 4, 64), ((174, 174), 3, 24), ((300, 400), 3, 20),
                                    ((84, 84), 2, 928), ((174, 174), 2, 208), ((300, 400), 2, 48)],
                         ids=["84x84", "174x174", "c5_300x400", "84x84_wide", "174x174_wide", "c5_wide"])
def test_dedup_forward_bitwise_and_backward_vs_fp64_oracle(hw, T, E):
    from vnav import _lib
    from vnav.policy import frames_from_batch
    lib = _lib.load()
    pol = _noisy_policy(hw, 12)
    net, params = pol.net, pol.params.data
    N = T * E
    assert net.goal_runs_supported(E) and not net.goal_runs_supported(16)
    img, gl, dones = _rollout_batch(hw, T, E, 31)
    delta = torch.zeros((T, E), dtype=torch.int32, device="cuda")
    lst = torch.zeros((T, E), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(T + 1, dtype=torch.int32, device="cuda")
    acts_d, acts_f = net.new_acts(N), net.new_acts(N)
    out_d, out_f = torch.zeros((N, 8), device="cuda"), torch.zeros((N, 8), device="cuda")
    for t in range(T):
        sl = slice(t * E, (t + 1) * E)
        fr = frames_from_batch(img[sl], gl[sl])
        _step_runs(lib, _lib, dones, t, delta, lst, cnt)
        gr = _lib.GoalRuns()
        gr.goal_list, gr.goal_count, gr.goal_delta = lst[t].data_ptr(), cnt[t:t + 1].data_ptr(), delta[t].data_ptr()
        net.forward(params, fr, E, acts_d, N, t * E, out_d[sl], goals=gr)
        net.forward(params, fr, E, acts_f, N, t * E, out_f[sl])
    torch.cuda.synchronize()
    assert torch.equal(out_d, out_f), "the deduplicated forward must equal the full forward bitwise"
    assert torch.equal(net.x5(acts_d, N), net.x5(acts_f, N))
    n_goal = int(cnt[:T].sum())
    assert E <= n_goal < N  # some goal frames were skipped
    # backward: the update's runs over the whole rollout
    g = torch.Generator(device="cuda").manual_seed(3)
    actions = torch.randint(0, 4, (N,), dtype=torch.int32, device="cuda", generator=g)
    rets = torch.randn(N, device="cuda", generator=g)
    dout = _loss_grad(out_f, actions, rets)
    masks = _gpu_masks(net, acts_f, N)  # every sample's own goal maps (full forward)
    rl = torch.zeros(N, dtype=torch.int32, device="cuda")
    _lib.check(lib.vn_goal_runs_rollout(_lib.ptr(dones), T, E, _lib.ptr(lst.view(-1)), _lib.ptr(rl), _lib.ptr(cnt[T:]),
                                        _lib.stream_ptr(dones.device)), "vn_goal_runs_rollout")
    gr = _lib.GoalRuns()
    gr.goal_list, gr.goal_count, gr.goal_delta = lst.data_ptr(), cnt[T:].data_ptr(), delta.data_ptr()
    gr.run_length, gr.num_envs = rl.data_ptr(), E
    fr = frames_from_batch(img, gl)
    gd, gf = torch.zeros_like(params), torch.zeros_like(params)
    ws = torch.empty(net.workspace_floats(N), device="cuda")
    net.backward_ex(params, fr, N, acts_d, N, dout, None, None, gd, ws, goals=gr)
    net.backward_ex(params, fr, N, acts_f, N, dout, None, None, gf, ws)
    torch.cuda.synchronize()
    mine, full = net.to_reference(gd), net.to_reference(gf)
    errs = {k: _err(mine[k].numpy(), full[k].numpy()) for k in full}
    bad = {k: "%.3g" % e for k, e in errs.items() if e > 1e-5}
    assert not bad, bad
    ref = GoalNetOracle(hw).load_reference(pol.reference_state_dict()).double()
    logits, value, _, _ = ref.forward_masked(frames_to_float(img.cpu()).double(), frames_to_float(gl.cpu()).double(),
                                             masks)
    o = out_d.cpu().numpy()
    _check_outputs(o[:, :4], o[:, 4], logits.detach().numpy(), value.detach().numpy().ravel())
    from oracle import a2c as oa2c
    loss, _ = oa2c.loss(logits, value.view(-1), actions.cpu().long(), rets.cpu().double())
    loss.backward()
    worst = _grads_vs_oracle(net, gd, ref)
    print("%dx%d dedup: %d of %d goal frames computed; worst gradient error %.3g of scale vs fp64, %.3g vs full"
          % (hw[0], hw[1], n_goal, N, worst, max(errs.values())))


def _trainer_pair(hw, E, aux, T=5, seed=4):
    import vnav
    from bench import aux_scenes
    scenes = aux_scenes(2, hw + (3,)) if aux else [vnav.synthetic_scene(k, frame_shape=hw + (3,)) for k in range(2)]
    out = []
    for dedup in (True, False):
        env = vnav.VectorEnv(scenes, E, seed=seed, max_episode_steps=3)
        out.append(vnav.A2CTrainer(env, num_steps=T, seed=2, max_time_steps=1e6, recurrent=True,
                                   aux_weight=0.1 if aux else 0.0, dedup_goals=dedup))
    return out


@pytest.mark.parametrize("hw,E,aux", [((174, 174), 32, True), ((84, 84), 96, False), ((300, 400), 24, True)],
                         ids=["174_lstm_aux", "84_lstm", "c5_lstm_aux"])
def test_trainer_dedup_equals_full(hw, E, aux):
    a, b = _trainer_pair(hw, E, aux)
    assert a.dedup_goals and not b.dedup_goals
    for _ in range(2):  # the second rollout starts from carried state and mid-episode goals
        a.rollout()
        b.rollout()
        torch.cuda.synchronize()
        for name in ("out", "actions", "rewards", "dones", "rows_img", "rows_goal", "boot_out"):
            assert torch.equal(getattr(a, name), getattr(b, name)), name
        T = a.num_steps
        assert int(a.goal_count[:T].sum()) < T * a.env.num_envs
        a.grads.zero_()
        b.grads.zero_()
        a.update()
        b.update()
        torch.cuda.synchronize()
        ga, gb = a.net.to_reference(a.grads), b.net.to_reference(b.grads)
        errs = {k: _err(ga[k].numpy(), gb[k].numpy()) for k in gb if gb[k].abs().max() > 0}
        bad = {k: "%.3g" % e for k, e in errs.items() if e > 1e-5}
        assert not bad, bad
        # continue both from the same parameters so the next rollout is identical again
        b.params.copy_(a.params)
        b.square_avg.copy_(a.square_avg)


def test_goal_runs_refused_where_unsupported():
    """A few envs (the skinny paths), BigHouseModel (no goal branch) and the A/B overrides
    that select kernels without frame lists take no goal runs: an error, never a silent
    fallback."""
    import os
    from vnav import _lib
    from vnav.policy import PolicyNet, frames_from_batch
    net = PolicyNet((84, 84), 4)
    assert not net.goal_runs_supported(16) and net.goal_runs_supported(17)
    n = 16
    img = torch.zeros((n, 84, 84, 3), dtype=torch.uint8, device="cuda")
    z = torch.zeros(n, dtype=torch.int32, device="cuda")
    gr = _lib.GoalRuns()
    gr.goal_list, gr.goal_count, gr.goal_delta = z.data_ptr(), z.data_ptr(), z.data_ptr()
    with pytest.raises(_lib.VnavError, match="goal runs"):
        net.forward(net.init_params(0), frames_from_batch(img, img), n, net.new_acts(n), n, 0,
                    torch.zeros((n, 8), device="cuda"), goals=gr)
    assert not PolicyNet((84, 84), 4, recurrent=True, arch="bighouse").goal_runs_supported(512)
    os.environ["VN_WGRAD_GENERIC"] = "1"
    try:
        assert not net.goal_runs_supported(512)
    finally:
        os.environ.pop("VN_WGRAD_GENERIC")
    assert PolicyNet((300, 400), 4).goal_runs_supported(512)


def test_dedup_off_for_companion_frames():
    """An oriented scene with third-person companion frames (OrientedGraphEnv's render tuple,
    environments/gym_graph/graph.py:60-61) emits a second frame that changes every step: the
    trainer must not reuse a run start's goal maps there. Auto mode turns the
    deduplication off, an explicit request is refused, and the rollout outputs equal the
    forward of the frames actually emitted."""
    import numpy as np
    import vnav
    rng = np.random.default_rng(3)
    maze = np.ones((6, 6), dtype=bool)
    obs = rng.integers(0, 256, size=(6, 6, 4, 84, 84, 3), dtype=np.uint8)
    tp = rng.integers(0, 256, size=(6, 6, 4, 84, 84, 3), dtype=np.uint8)
    scene = vnav.oriented_scene(maze, obs, goals=[(5, 5, 0)], tp_observations=tp)
    E = 32
    env = vnav.VectorEnv([scene], E, seed=1, max_episode_steps=50)
    with pytest.raises(ValueError, match="companion"):
        vnav.A2CTrainer(env, num_steps=4, recurrent=False, dedup_goals=True)
    tr = vnav.A2CTrainer(env, num_steps=4, recurrent=False)
    assert not tr.dedup_goals and tr.net.goal_runs_supported(E)
    tr.rollout()
    torch.cuda.synchronize()
    T = tr.num_steps
    # the second frame differs between steps of one episode (so a run start's maps would be stale)
    assert not torch.equal(tr.rows_goal[:E], tr.rows_goal[E:2 * E])
    out = torch.zeros_like(tr.out)
    acts = tr.net.new_acts(T * E)
    for t in range(T):
        sl = slice(t * E, (t + 1) * E)
        tr.net.forward(tr.params, tr._frames(tr.rows_img[sl], tr.rows_goal[sl]), E, acts, T * E, t * E, out[sl])
    torch.cuda.synchronize()
    assert torch.equal(out, tr.out)


@pytest.mark.parametrize("flag", ["VN_CONV3F_GATHER"])
@pytest.mark.parametrize("hw,E", [((174, 174), 208), ((300, 400), 48), ((84, 84), 64)],
                         ids=["174x174", "c5_300x400", "84x84_splitk"])
def test_conv3_forward_forms_bitwise(flag, hw, E):
    """conv3's forward product with goal runs reaching back into the previous step's samples
    (whole K with a ragged last row tile; split K at 84x84): the gather with per-slot offsets
    kept across the K loop (the default) against the generic gather (`VN_CONV3F_GATHER`): the
    same products in the same k order, X5 and the outputs bitwise."""
    import os
    from vnav import _lib
    from vnav.policy import frames_from_batch
    lib = _lib.load()
    pol = _noisy_policy(hw, 12)
    net, params = pol.net, pol.params.data
    T = 2
    N = T * E
    img, gl, dones = _rollout_batch(hw, T, E, 17, p_done=0.5)

    def run(on):
        if on:
            os.environ[flag] = "1"
        try:
            delta = torch.zeros((T, E), dtype=torch.int32, device="cuda")
            lst = torch.zeros((T, E), dtype=torch.int32, device="cuda")
            cnt = torch.zeros(T + 1, dtype=torch.int32, device="cuda")
            acts = net.new_acts(N)
            acts.fill_(float("nan"))
            out = torch.zeros((N, 8), device="cuda")
            for t in range(T):
                sl = slice(t * E, (t + 1) * E)
                _step_runs(lib, _lib, dones, t, delta, lst, cnt)
                gr = _lib.GoalRuns()
                gr.goal_list, gr.goal_count, gr.goal_delta = lst[t].data_ptr(), cnt[t:t + 1].data_ptr(), delta[t].data_ptr()
                net.forward(params, frames_from_batch(img[sl], gl[sl]), E, acts, N, t * E, out[sl], goals=gr)
            torch.cuda.synchronize()
            return net.x5(acts, N).clone(), out[:, :5].clone()
        finally:
            os.environ.pop(flag, None)

    (x_def, o_def), (x_on, o_on) = run(False), run(True)
    assert not torch.isnan(o_def).any() and float(x_def.abs().max()) > 0
    assert torch.equal(x_def, x_on), float((x_def - x_on).abs().max())
    assert torch.equal(o_def, o_on)


@pytest.mark.parametrize("hw,E,back", [((84, 84), 32, 110000), ((174, 174), 24, 22000)],
                         ids=["84x84", "174x174"])
def test_goal_runs_reaching_back_past_2GB(hw, E, back):
    """Goal runs whose starts lie more than 2 GB of conv2 maps behind this call's samples (the
    bench's 20 x 4096 rollouts reach ~8 GB back at 174x174): a call at activation offset `back`
    with every goal half read from the samples a first call wrote at offset 0 (goal_count 0: no
    goal frame of its own) against a plain forward of the same frames — outputs and X5 bitwise.
    conv3's gather keeps those offsets in 16-byte units (NhwcIm2colGoalF); a byte offset, or a
    buffer descriptor based at this call's samples, would miss them."""
    from vnav import _lib
    from vnav.policy import frames_from_batch
    pol = _noisy_policy(hw, 13)
    net, params = pol.net, pol.params.data
    assert net.goal_runs_supported(E)
    g = torch.Generator(device="cuda").manual_seed(23)
    img0 = torch.randint(0, 256, (E,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    img1 = torch.randint(0, 256, (E,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (E,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cap = back + E
    acts = net.new_acts(cap)
    out0 = torch.zeros((E, 8), device="cuda")
    net.forward(params, frames_from_batch(img0, gl), E, acts, cap, 0, out0)  # the goal halves at samples 0..E-1
    delta = torch.full((E,), -back, dtype=torch.int32, device="cuda")
    lst = torch.zeros(E, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    gr = _lib.GoalRuns()
    gr.goal_list, gr.goal_count, gr.goal_delta = lst.data_ptr(), cnt.data_ptr(), delta.data_ptr()
    out_far = torch.zeros((E, 8), device="cuda")
    net.forward(params, frames_from_batch(img1, gl), E, acts, cap, back, out_far, goals=gr)
    ref_acts = net.new_acts(E)
    out_ref = torch.zeros((E, 8), device="cuda")
    net.forward(params, frames_from_batch(img1, gl), E, ref_acts, E, 0, out_ref)
    torch.cuda.synchronize()
    assert torch.isfinite(out_ref).all()
    assert torch.equal(out_far, out_ref), float((out_far - out_ref).abs().max())
    assert torch.equal(net.x5(acts, cap)[back:], net.x5(ref_acts, E))
    del acts
