"""Pre-split weight operands (SplitRows, csrc/vn_policy.hip): at training batches (>= 256
samples) the forward splits conv2's, conv3's and conv_merge's weights into bf16 planes once
per call instead of once per tile. The split is the same truncation chain, so the forward is
bit-identical to the per-tile form (VN_NO_PRESPLIT=1) — activations and outputs, with and
without goal runs."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _noisy(hw, seed):
    from vnav.policy import PolicyNet
    net = PolicyNet(hw, 4, device="cuda:0")
    params = net.init_params(seed)
    g = torch.Generator(device="cpu").manual_seed(seed + 1)
    with torch.no_grad():
        v = net.views(params)
        for name in ("conv1", "conv2", "conv3", "conv4", "fc", "head"):
            b = v[name][1]
            b.copy_((torch.rand(b.shape, generator=g) * 0.1 - 0.05).to(b.device))
    return net, params


def _forward(net, params, fr, n, goals=None, presplit=True, T=1, E=None):
    acts = net.new_acts(n)
    out = torch.zeros((n, 8), device="cuda")
    if presplit:
        os.environ.pop("VN_NO_PRESPLIT", None)
    else:
        os.environ["VN_NO_PRESPLIT"] = "1"
    try:
        if goals is None:
            net.forward(params, fr, n, acts, n, 0, out)
        else:
            for t, (f, g) in enumerate(zip(fr, goals)):
                net.forward(params, f, E, acts, n, t * E, out[t * E:(t + 1) * E], goals=g)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("VN_NO_PRESPLIT", None)
    return acts, out


@pytest.mark.parametrize("hw,n", [((84, 84), 512), ((174, 174), 300), ((300, 400), 260)],
                         ids=["84x84", "174x174", "c5_300x400"])
def test_presplit_forward_is_bit_identical(hw, n):
    from vnav.policy import frames_from_batch
    net, params = _noisy(hw, 5)
    g = torch.Generator(device="cuda").manual_seed(7)
    img = torch.randint(0, 256, (n,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (n,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    fr = frames_from_batch(img, gl)
    a1, o1 = _forward(net, params, fr, n, presplit=True)
    a0, o0 = _forward(net, params, fr, n, presplit=False)
    assert torch.equal(o1, o0) and torch.equal(a1, a0)


def test_presplit_goal_runs_c5_bit_identical():
    """C5's conv2 forward with goal runs is the row-limited generic product over FrameListIm2col:
    the pre-split weight operand there too."""
    from vnav import _lib
    from vnav.policy import frames_from_batch
    from test_goal_runs_gpu import _rollout_batch, _step_runs
    lib = _lib.load()
    hw, T, E = (300, 400), 2, 260
    net, params = _noisy(hw, 9)
    img, gl, dones = _rollout_batch(hw, T, E, 13)
    delta = torch.zeros((T, E), dtype=torch.int32, device="cuda")
    lst = torch.zeros((T, E), dtype=torch.int32, device="cuda")
    cnt = torch.zeros(T + 1, dtype=torch.int32, device="cuda")
    frs, grs = [], []
    for t in range(T):
        sl = slice(t * E, (t + 1) * E)
        frs.append(frames_from_batch(img[sl], gl[sl]))
        _step_runs(lib, _lib, dones, t, delta, lst, cnt)
        gr = _lib.GoalRuns()
        gr.goal_list, gr.goal_count, gr.goal_delta = lst[t].data_ptr(), cnt[t:t + 1].data_ptr(), delta[t].data_ptr()
        grs.append(gr)
    a1, o1 = _forward(net, params, frs, T * E, goals=grs, presplit=True, E=E)
    a0, o0 = _forward(net, params, frs, T * E, goals=grs, presplit=False, E=E)
    assert torch.equal(o1, o0) and torch.equal(net.x5(a1, T * E), net.x5(a0, T * E))


def test_presplit_lstm_gates_bit_identical():
    """The LSTM step's gates product on the pre-split W_cat (E >= 256): h, c, gates and the
    activations bitwise equal to the per-tile split."""
    from vnav.policy import PolicyNet
    E = 300
    net = PolicyNet((84, 84), 4, device="cuda:0", recurrent=True)
    params = net.init_params(3)
    L = net.lstm
    g = torch.Generator(device="cuda").manual_seed(2)
    x5 = torch.rand((E, 512), device="cuda", generator=g)
    lra = torch.rand((E, 5), device="cuda", generator=g)
    mask = (torch.rand(E, device="cuda", generator=g) > 0.2).float()
    h0 = torch.randn((E, 512), device="cuda", generator=g)
    c0 = torch.randn((E, 512), device="cuda", generator=g)

    def run(presplit):
        bufs = [torch.zeros((E, L["xcat"]), device="cuda"), torch.zeros((E, 2048), device="cuda"),
                torch.zeros((E, 2048), device="cuda"), torch.zeros((E, 512), device="cuda"),
                torch.zeros((E, 512), device="cuda")]
        if presplit:
            os.environ.pop("VN_NO_PRESPLIT", None)
        else:
            os.environ["VN_NO_PRESPLIT"] = "1"
        try:
            net.lstm_step(params, E, x5, lra, mask, h0, c0, *bufs)
            torch.cuda.synchronize()
        finally:
            os.environ.pop("VN_NO_PRESPLIT", None)
        return bufs

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


def test_presplit_trainer_updates_bit_identical():
    """Two LSTM + aux updates of 300 envs with and without the pre-split weight operands
    (forward, LSTM step, LSTM backward, conv_merge input gradient): the same parameters,
    optimiser state and actions, bitwise."""
    import vnav
    from test_aux_gpu import _aux_scene

    def make():
        env = vnav.VectorEnv([_aux_scene(0, (84, 84, 3))], 300, seed=4, max_episode_steps=12)
        return vnav.A2CTrainer(env, num_steps=4, seed=2, max_time_steps=1e9, recurrent=True, aux_weight=0.1)

    a, b = make(), make()
    for _ in range(2):
        a.step(sync=True)
        os.environ["VN_NO_PRESPLIT"] = "1"
        try:
            b.step(sync=True)
        finally:
            os.environ.pop("VN_NO_PRESPLIT", None)
        assert torch.equal(a.actions, b.actions)
    assert torch.equal(a.params, b.params) and torch.equal(a.square_avg, b.square_avg)
