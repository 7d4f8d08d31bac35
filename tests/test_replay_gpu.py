"""The device-side replay ring (vn_replay_push_draw) and what it enables: an update with
replay sources captured in a hipGraph, the replay gradients joined inside the norm kernel
(vn_grad_norm_join), the side-stream disjointness guard, checkpoints whose ring does not
match the trainer, the update(None) path, and BigHouseModel reference state dicts with the
reference's 7776-input rp.

The reference's replay buffer is deep_rl's (absent, experiments/ai2_auxiliary/trainer.py:27-31:
``self.replay.sample_sequence()``): capacity, sequence shape and draw are parity unpinned; the
ring here is checked against its own numpy restatement (push into slot pos, uniform draw over
the filled slots with Philox4x32-10 stream 4, oracle/philox.py)."""
import copy
import ctypes
import os
import warnings

import numpy as np
import pytest
import torch

from oracle.philox import philox4x32_10, seed_key, uniform_below

pytestmark = pytest.mark.gpu


def _unreal_env(n_envs, seed=2):
    import vnav
    from test_aux_gpu import _aux_scene
    return vnav.VectorEnv([_aux_scene(0, (174, 174, 3))], n_envs, seed=seed, max_episode_steps=30)


def test_replay_push_draw_kernel_vs_numpy():
    """Segments of 4-byte and 1-byte elements, strided sources, a 3-slot ring over 7 pushes:
    ring slots, the drawn slot's copy (including a draw of the slot just written) and the meta
    [next slot, filled, counter, drawn] equal the numpy restatement."""
    from vnav import _lib
    lib = _lib.load()
    R, seed = 3, 0x1234_5678_9ABC
    k0, k1 = seed_key(seed)
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1)
    src_i = torch.zeros((4, 7), dtype=torch.int32, device=dev)   # rows 4, cols 5 of 7
    src_f = torch.zeros(9, dtype=torch.float32, device=dev)      # rows 1, cols 9
    src_b = torch.zeros((3, 6), dtype=torch.bool, device=dev)    # rows 3, cols 4 of 6 (bytes)
    ring_i = torch.full((R, 20), -1, dtype=torch.int32, device=dev)
    ring_f = torch.full((R, 11), -1.0, dtype=torch.float32, device=dev)  # slot stride > rows*cols
    ring_b = torch.zeros((R, 12), dtype=torch.bool, device=dev)
    cur_i = torch.zeros(20, dtype=torch.int32, device=dev)
    cur_f = torch.zeros(9, dtype=torch.float32, device=dev)
    cur_b = torch.zeros(12, dtype=torch.bool, device=dev)
    meta = torch.zeros(4, dtype=torch.int64, device=dev)
    S = _lib.ReplaySeg
    segs = (S * 3)(S(src_i.data_ptr(), 7, ring_i.data_ptr(), cur_i.data_ptr(), 20, 4, 5, 4, 0),
                   S(src_f.data_ptr(), 9, ring_f.data_ptr(), cur_f.data_ptr(), 11, 1, 9, 4, 0),
                   S(src_b.data_ptr(), 6, ring_b.data_ptr(), None, 12, 3, 4, 1, 0))
    ref_i, ref_f, ref_b = ring_i.cpu().numpy(), ring_f.cpu().numpy(), ring_b.cpu().numpy()
    pos = filled = 0
    seen_self = False
    for call in range(7):
        src_i.copy_(torch.randint(-1000, 1000, src_i.shape, generator=g, device=dev, dtype=torch.int32))
        src_f.normal_(generator=g)
        src_b.copy_(torch.rand(src_b.shape, generator=g, device=dev) > 0.5)
        _lib.check(lib.vn_replay_push_draw(segs, 3, _lib.ptr(meta), R, ctypes.c_uint64(seed),
                                           _lib.stream_ptr(torch.device(dev))), "vn_replay_push_draw")
        si, sf, sb = src_i.cpu().numpy(), src_f.cpu().numpy(), src_b.cpu().numpy()
        ref_i[pos, :20] = si[:4, :5].reshape(-1)
        ref_f[pos, :9] = sf
        ref_b[pos, :12] = sb[:3, :4].reshape(-1)
        filled = min(filled + 1, R)
        r = philox4x32_10(call & 0xFFFFFFFF, call >> 32, 0, 4, k0, k1)[0]
        k = int(uniform_below(r, filled))
        seen_self |= k == pos
        torch.cuda.synchronize()
        assert np.array_equal(ring_i.cpu().numpy(), ref_i), call
        assert np.array_equal(ring_f.cpu().numpy(), ref_f), call
        assert np.array_equal(ring_b.cpu().numpy(), ref_b), call
        assert np.array_equal(cur_i.cpu().numpy(), ref_i[k]), (call, k)
        assert np.array_equal(cur_f.cpu().numpy(), ref_f[k, :9]), (call, k)
        pos = (pos + 1) % R
        assert meta.cpu().tolist() == [pos, filled, call + 1, k], call
    assert seen_self  # the k == slot-being-written path ran (cur taken from the source)
    assert not cur_b.any()  # a NULL cur is not written


def _ref_trainer(graph, replay_size=4, E=16, T=5, S=8, seed=3, **kw):
    """thor-cached-auxiliary's trainer settings (vnav/train.py): LSTM + aux heads + UNREAL,
    both batches replayed."""
    import vnav
    env = _unreal_env(E, seed=5)
    return vnav.A2CTrainer(env, num_steps=T, seed=seed, max_time_steps=1e9, recurrent=True, aux_weight=0.1,
                           unreal=True, unreal_envs=S, aux_source="replay", unreal_source="replay",
                           replay_size=replay_size, cuda_graph=graph, entropy_coefficient=0.001, **kw)


@pytest.mark.parametrize("E,S,merged", [(16, 8, False), (4, 4, False), (4, 4, True)])
def test_cuda_graph_with_replay_sources_is_bit_identical(E, S, merged):
    """The registered experiment's update (replayed aux batch + replayed UNREAL pass on a side
    stream; at S == E the aux heads inside the UNREAL pass) captured once in a hipGraph and
    replayed: parameters, RMSprop state, ring, meta and the metrics equal the eager updates
    bitwise (the pc / aux statistics to rounding: atomics)."""
    def run(graph):
        if merged:
            os.environ["VN_REPLAY_MERGED"] = "1"
        try:
            tr = _ref_trainer(graph, E=E, S=S)
        finally:
            os.environ.pop("VN_REPLAY_MERGED", None)
        assert tr._merged_replay == merged
        ms = [tr.step(sync=True) for _ in range(7)]
        torch.cuda.synchronize()
        return tr, ms

    a, ma = run(False)
    b, mb = run(True)
    assert b._graph is not None  # the updates after the first replayed the captured graph
    assert torch.equal(a.params, b.params) and torch.equal(a.square_avg, b.square_avg)
    assert torch.equal(a.replay_meta, b.replay_meta) and torch.equal(a.replay_rows, b.replay_rows)
    assert a.replay_filled == 4
    for key in a.ur:
        assert torch.equal(a.ur[key], b.ur[key]), key
    for x, y in zip(ma, mb):
        for k in ("value_loss", "rp_loss", "vr_loss", "grad_norm", "entropy"):
            assert x[k] == y[k], (k, x[k], y[k])
        # the pc and aux loss statistics sum per-workgroup partials with atomics (metrics only)
        for k in ("pc_loss", "aux_loss"):
            np.testing.assert_allclose(x[k], y[k], rtol=1e-5)


def test_merged_replay_pass_matches_two_passes():
    """S == E (the logged run's 4 envs), opt-in `VN_REPLAY_MERGED`: the aux heads on the replayed
    UNREAL pass's trunk forward, their dX4 joining its trunk backward (one forward + backward of the
    replayed rollout) against the separate aux-replay pass (the default): the same update to rounding (the trunk
    gradients of the two losses summed in another order, over three updates of drift) — every
    gradient block to 1e-4 of its scale (the suite's gradient tolerance; measured 1.3e-5), the
    aux / UNREAL statistics to 1e-4, the ring bitwise."""
    import os

    def run(separate):
        if not separate:
            os.environ["VN_REPLAY_MERGED"] = "1"
        try:
            tr = _ref_trainer(False, E=4, S=4)
        finally:
            os.environ.pop("VN_REPLAY_MERGED", None)
        assert tr._merged_replay == (not separate)
        for _ in range(3):  # fill the ring, then one compared update
            batch, _ = tr.sample_training_batch()
            tr.update(batch)
        torch.cuda.synchronize()
        return tr

    a, b = run(False), run(True)
    assert torch.equal(a.replay_meta, b.replay_meta) and torch.equal(a.replay_rows, b.replay_rows)
    ga, gb = a.net.to_reference(a.grads), b.net.to_reference(b.grads)
    bad = {}
    for k in gb:
        ref = gb[k].numpy().astype(np.float64)
        sc = np.abs(ref).max()
        if sc == 0:
            continue
        e = np.abs(ga[k].numpy() - ref).max() / sc
        if e > 1e-4:
            bad[k] = "%.3g" % e
    assert not bad, bad
    torch.testing.assert_close(a.aux_stats, b.aux_stats, rtol=1e-4, atol=0)
    torch.testing.assert_close(a.unreal_stats, b.unreal_stats, rtol=1e-4, atol=1e-9)


@pytest.mark.parametrize("merged", [False, True])
def test_side_stream_pass_equals_inline_pass(merged):
    """The replayed UNREAL pass on its side stream (beside the A2C backward) against the same
    pass run on the main stream before it (`VN_UNREAL_INLINE`): every buffer the two streams
    write is disjoint, so four updates give the same parameters, RMSprop state and ring
    bitwise — a race between the streams would show up here as a difference (the pc / aux
    statistics to rounding: atomics). With `VN_REPLAY_MERGED` the aux heads ride in the pass."""
    def run(inline):
        env = {"VN_UNREAL_INLINE": "1"} if inline else {}
        if merged:
            env["VN_REPLAY_MERGED"] = "1"
        os.environ.update(env)
        try:
            tr = _ref_trainer(False, E=4 if merged else 16, S=4 if merged else 8)
        finally:
            for k in env:
                os.environ.pop(k, None)
        assert tr._unreal_inline == inline and tr._merged_replay == merged
        for _ in range(4):
            tr.step(sync=True)
        torch.cuda.synchronize()
        return tr

    a, b = run(False), run(True)
    assert torch.equal(a.params, b.params) and torch.equal(a.square_avg, b.square_avg)
    assert torch.equal(a.replay_meta, b.replay_meta)
    torch.testing.assert_close(a.unreal_stats, b.unreal_stats, rtol=1e-5, atol=1e-9)
    torch.testing.assert_close(a.aux_stats, b.aux_stats, rtol=1e-5, atol=0)


def test_grad_norm_join_equals_adds_then_norm():
    """vn_grad_norm_join (the side passes' gradients added inside the norm's first pass) against
    the two adds followed by vn_grad_norm: the same gradient and scalars bitwise."""
    from vnav import _lib
    lib = _lib.load()
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 1_000_003
    grads = torch.randn(n, generator=g, device="cuda")
    a0 = torch.randn(n, generator=g, device="cuda")
    a1 = torch.randn(n, generator=g, device="cuda")
    partial = torch.zeros(512, dtype=torch.float64, device="cuda")
    s1, s2 = torch.zeros(2, device="cuda"), torch.zeros(2, device="cuda")
    st = _lib.stream_ptr(torch.device("cuda"))
    ref = grads.clone()
    ref[1000:700000] += a0[1000:700000]
    ref[0:500000] += a1[0:500000]
    P = _lib.ptr
    _lib.check(lib.vn_grad_norm(P(ref), n, ctypes.c_float(0.5), ctypes.c_float(0.5), P(partial), P(s1), st), "norm")
    _lib.check(lib.vn_grad_norm_join(P(grads), n, P(a0), 1000, 700000, P(a1), 0, 500000, ctypes.c_float(0.5),
                                     ctypes.c_float(0.5), P(partial), P(s2), st), "join")
    torch.cuda.synchronize()
    assert torch.equal(grads, ref) and torch.equal(s1, s2)
    with pytest.raises(_lib.VnavError):
        lib_rc = lib.vn_grad_norm_join(P(grads), n, P(a0), 0, n + 1, None, 0, 0, ctypes.c_float(1.0),
                                       ctypes.c_float(0.5), P(partial), P(s2), st)
        _lib.check(lib_rc, "vn_grad_norm_join")


@pytest.mark.parametrize("E,S,merged", [(16, 8, False), (4, 4, True)])
def test_side_stream_guard_passes_and_trips_on_overlap(E, S, merged):
    """The replayed UNREAL pass's side stream is race-free only while its buffers and gradient
    block are disjoint from the main stream's: the debug check passes on the trainer's own
    layout (every update of a debug run; at S == E with the aux heads' buffers and block on the
    side stream) and raises on an aliased buffer and on a join range reaching into the pc / rp
    block."""
    if merged:
        os.environ["VN_REPLAY_MERGED"] = "1"
    try:
        tr = _ref_trainer(False, replay_size=2, E=E, S=S)
    finally:
        os.environ.pop("VN_REPLAY_MERGED", None)
    assert tr._merged_replay == merged
    tr.debug_streams = True
    for _ in range(2):
        tr.step(sync=True)
    tr._check_side_stream_disjoint()
    ws = tr.pc_ws
    tr.pc_ws = tr.workspace[:ws.numel()]  # a side-stream buffer carved from the main workspace
    with pytest.raises(RuntimeError, match="pc_ws"):
        tr._check_side_stream_disjoint()
    tr.pc_ws = ws
    end = tr._ur_add_end
    tr._ur_add_end = tr.net.n_params  # the join would add over the side stream's pc / rp block
    with pytest.raises(RuntimeError, match="join range"):
        tr._check_side_stream_disjoint()
    tr._ur_add_end = end
    tr._check_side_stream_disjoint()


def test_resume_aux_only_replay_checkpoint_restarts_the_unreal_ring():
    """A checkpoint saved with aux-only replay (unreal_source='rollout') loaded into the
    registered experiment's trainer (both replayed): its ring has no UNREAL record, so the ring
    restarts empty with a warning (restoring the frame rows alone would draw slots whose UNREAL
    record is zeros) and training continues; a checkpoint of the same settings resumes exactly."""
    import vnav
    env = _unreal_env(16, seed=5)
    a = vnav.A2CTrainer(env, num_steps=5, seed=3, max_time_steps=1e9, recurrent=True, aux_weight=0.1, unreal=True,
                        unreal_envs=8, aux_source="replay", unreal_source="rollout", replay_size=4)
    for _ in range(3):
        a.step(sync=True)
    sd = copy.deepcopy(a.state_dict())
    assert "replay_meta" in sd and not any(k.startswith("ur_") for k in sd)
    b = _ref_trainer(False)
    with pytest.warns(UserWarning, match="replay ring restarts empty"):
        b.load_state_dict(sd)
    assert b.replay_filled == 0 and torch.equal(b.params, a.params)
    m = b.step(sync=True)
    assert all(np.isfinite(m[k]) for k in ("rp_loss", "vr_loss", "pc_loss", "aux_loss"))
    assert b.replay_filled == 1
    # same settings: exact resume through the device meta
    sd2 = copy.deepcopy(b.state_dict())
    m1 = [b.step(sync=True) for _ in range(2)]
    c = _ref_trainer(False)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        c.load_state_dict(sd2)
    m2 = [c.step(sync=True) for _ in range(2)]
    assert torch.equal(b.params, c.params) and torch.equal(b.replay_meta, c.replay_meta)
    for x, y in zip(m1, m2):
        assert x["rp_loss"] == y["rp_loss"] and x["vr_loss"] == y["vr_loss"]
        np.testing.assert_allclose(x["aux_loss"], y["aux_loss"], rtol=1e-5)  # atomics (metric only)


def test_update_without_batch_pushes_and_uses_the_replayed_aux_batch():
    """update(None) after a bare rollout() with aux_source='replay': the rollout is pushed into
    the ring and the drawn aux batch is used, exactly as sample_training_batch() + update(batch)."""
    import vnav
    from test_aux_gpu import _aux_scene

    def make():
        env = vnav.VectorEnv([_aux_scene(0)], 64, seed=2, max_episode_steps=50)
        return vnav.A2CTrainer(env, num_steps=5, seed=1, max_time_steps=1e9, aux_weight=0.1, recurrent=True,
                               aux_source="replay", replay_size=3)

    a, b = make(), make()
    for _ in range(3):
        batch, _ = a.sample_training_batch()
        a.update(batch)
        b.rollout()
        b.update(None)
    torch.cuda.synchronize()
    assert b.replay_filled == 3
    assert torch.equal(a.replay_meta, b.replay_meta)
    # the aux loss statistic sums per-workgroup partials with atomics (metric only)
    torch.testing.assert_close(a.aux_stats, b.aux_stats, rtol=1e-5, atol=0)
    assert float(b.aux_stats.abs().sum()) > 0
    assert torch.equal(a.params, b.params)


def test_bighouse_reference_rp_of_7776_inputs_loads_the_rest():
    """BigHouseModel builds rp as Linear(9*9*32*3, 3) (bignet.py:94), which fits only 100x100
    frames; a reference state dict carrying it loads into BigHousePolicy(unreal=True) at 84x84
    with a warning: every other tensor is loaded, rp keeps this policy's initialisation."""
    from vnav.policy import BigHousePolicy
    src = BigHousePolicy(3, 4, recurrent=True, unreal=True, seed=1)
    sd = {k: v.clone() for k, v in src.reference_state_dict().items()}
    sd["rp.weight"] = torch.randn(3, 9 * 9 * 32 * 3)
    dst = BigHousePolicy(3, 4, recurrent=True, unreal=True, seed=2)
    rp0 = {k: v.clone() for k, v in dst.reference_state_dict().items() if k.startswith("rp.")}
    with pytest.warns(UserWarning, match="rp left at its initialisation"):
        dst.load_reference_state_dict(sd)
    out = dst.reference_state_dict()
    for k, v in out.items():
        if k.startswith("rp."):
            assert torch.equal(v, rp0[k]), k
        else:
            assert torch.equal(v, sd[k]), k
