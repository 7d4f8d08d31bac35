"""The persistent specialised kernels against the generic products they replaced (selected
back per call by an environment switch): the parity-class kernel (`parity_dgrad_x6_kernel`,
`VN_DGRAD_GENERIC`; at 300x400 its banded form `parity_dgrad_band_x6_kernel`) for conv3's
input gradient (k4 s2, 64 -> 2 x 32 channels) and the aux
heads' first transposed conv (32 -> 48 channels, bias + ReLU), and conv3's weight gradient
(`conv3_wgrad_x6_kernel`, `VN_WGRAD_GENERIC`). Both compute the same exact
split-bf16 products in another summation order, so every parameter gradient — conv3's
input gradient feeds conv2's and conv1's — agrees to rounding (1e-5 of scale). Batch sizes
cover a partial last work item (84x84 packs 4 images per item) and persistent-grid wraps
(more items than resident workgroups). The reference-level checks of these gradients are
tests/test_policy_gpu.py (84x84 golden, 174x174 float64 oracle)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grads(pol, img, gl, cl, cv, generic):
    if generic:
        os.environ[generic] = "1"
    try:
        pol.params.grad = None
        logits, value, _ = pol(((img, gl), None), None, None)
        ((logits * cl).sum() + (value * cv).sum()).backward()
        torch.cuda.synchronize()
        return pol.params.grad.clone()
    finally:
        if generic:
            os.environ.pop(generic, None)


@pytest.mark.parametrize("switch", ["VN_DGRAD_GENERIC", "VN_WGRAD_GENERIC"])
@pytest.mark.parametrize("hw,N", [((84, 84), 37), ((84, 84), 1030), ((174, 174), 5), ((174, 174), 300),
                                  ((300, 400), 31)])
def test_conv3_kernels_match_generic_products(hw, N, switch):
    """VN_DGRAD_GENERIC: conv3's input gradient; VN_WGRAD_GENERIC: conv3's weight and bias
    gradient (`conv3_wgrad_x6_kernel`, per-workgroup slabs + fixed-order reduce) against the
    split-K product over the gathered im2col."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(11)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(1)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)
    fast = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic=None))
    gen = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic=switch))
    bad = {}
    for k in gen:
        b = gen[k].numpy().astype(np.float64)
        e = np.abs(fast[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad
    # the kernels ran (not no-ops): conv3's input gradient reaches conv2's weights, and
    # conv3's own weight and bias gradients are live
    for k in ("shared_base.0.2.weight", "conv_base.0.0.weight", "conv_base.0.0.bias"):
        assert np.abs(fast[k].numpy()).max() > 0, k


@pytest.mark.parametrize("switch", ["VN_DGRAD_GENERIC", "VN_WGRAD_GENERIC"])
@pytest.mark.parametrize("hw,N", [((84, 84), 37), ((174, 174), 300), ((300, 400), 3), ((300, 400), 31)])
def test_aux_first_layer_matches_generic_products(hw, N, switch):
    """The aux heads' predictions and every parameter gradient of their MSE, both paths:
    VN_DGRAD_GENERIC for the first transposed conv's forward (parity kernel),
    VN_WGRAD_GENERIC for its weight gradient (`conv_wgrad_x6_kernel` with X4 as the reduced
    map and the 48-channel dA1 under it, no bias column)."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(12)
    pol = GoalNavPolicy(3, 4, hw, aux=True)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(2)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)

    # the switch is set for the forward and for the backward separately: the predictions compare
    # the two forwards, the gradients the two backwards over the SAME forward (with two forwards,
    # an A1 value within rounding of 0 could take the other side of its ReLU in one of them and
    # move the second layer's gradient by one pixel's term: seen at 1e-4 of scale at 174x174,
    # N = 300, once conv3's forward summed in another order)
    def run(generic_fwd, generic_bwd):
        try:
            if generic_fwd:
                os.environ[switch] = "1"
            pol.params.grad = None
            preds, _ = pol.forward_deconv(((img, gl), None))
            torch.cuda.synchronize()
            os.environ.pop(switch, None)
            if generic_bwd:
                os.environ[switch] = "1"
            sum((p * p).mean() for p in preds).backward()
            torch.cuda.synchronize()
            return [p.detach().cpu() for p in preds], pol.net.to_reference(pol.params.grad.clone())
        finally:
            os.environ.pop(switch, None)

    (pf, gf), (pg, _) = run(False, False), run(True, True)
    _, gg = run(False, True)
    for a, b in zip(pf, pg):
        e = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
        assert e < 1e-5, e
    bad = {}
    for k in gg:
        b = gg[k].numpy().astype(np.float64)
        if np.abs(b).max() == 0.0:
            continue
        e = np.abs(gf[k].numpy() - b).max() / np.abs(b).max()
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad


@pytest.mark.parametrize("hw,N", [((174, 174), 17), ((174, 174), 300), ((174, 174), 1030), ((300, 400), 17),
                                  ((300, 400), 129)])
def test_conv2_ring_forward_matches_generic_product(hw, N):
    """conv2's forward at 174x174 (42x42x32 -> 20x20x32) through the ring kernel
    (`conv2_fwd_ring_kernel`: frames streamed band by band, X1 rows split once into an LDS
    ring) and at 300x400 (74x99x32 -> 36x48x32) through the banded kernel
    (`conv2_fwd_x6_kernel`: bands of output rows, their X1 rows split once into LDS planes)
    against the generic im2col product (`VN_CONV2F_GENERIC`): the X2 maps of every frame
    (the kernel's whole output) to rounding, 2e-6 of scale, and the logits / value. N = 17 is
    the smallest batch that takes them (34 frames: most workgroups idle), 300 and 1030 wrap the
    persistent grid (several frames per workgroup: the ring crosses frame boundaries). Every
    parameter gradient is compared at N <= 300: both paths sum the same exact split products in
    another order, and at 1030 samples (26 M X2 values) a few values within rounding of 0 take
    the other side of a ReLU, which moves conv3's gradients by one sample's term (the oracle
    tests in test_prod_oracle_gpu.py run the float64 backward with the GPU's own masks)."""
    from vnav.policy import GoalNavPolicy, frames_from_batch
    torch.manual_seed(13)
    pol = GoalNavPolicy(3, 4, hw)
    net = pol.net
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(3)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)
    (h1, w1), (h2, w2) = {174: ((42, 42), (20, 20)), 300: ((74, 99), (36, 48))}[hw[0]]
    m1, x1, x2 = 2 * h1 * w1, 2 * h1 * w1 * 32, 2 * h2 * w2 * 32  # per-sample act regions (vn_policy.hip, acts_at)

    def run(generic):
        if generic:
            os.environ["VN_CONV2F_GENERIC"] = "1"
        try:
            acts = net.new_acts(N)
            out = torch.zeros((N, 8), device="cuda")
            net.forward(pol.params.detach(), frames_from_batch(img.view((N,) + hw + (3,)), gl.view((N,) + hw + (3,))),
                        N, acts, N, 0, out)
            X2 = acts[N * (m1 + x1):N * (m1 + x1 + x2)].clone()
            grads = None
            if N <= 300:
                pol.params.grad = None
                logits, value, _ = pol(((img, gl), None), None, None)
                ((logits * cl).sum() + (value * cv).sum()).backward()
                grads = net.to_reference(pol.params.grad.clone())
            torch.cuda.synchronize()
            return X2, out[:, :5].clone(), grads
        finally:
            os.environ.pop("VN_CONV2F_GENERIC", None)

    (xf, of, gf), (xg, og, gg) = run(False), run(True)
    assert float(xg.abs().max()) > 0
    e = float((xf - xg).abs().max()) / float(xg.abs().max())
    # both sum 512 exact products per output in fp32, in another order (the banded kernel adds
    # four kernel-row partials): ~8 ulp of the map's scale at 300x400 (1.02e-6 measured)
    assert e < 2e-6, e
    e = float((of - og).abs().max()) / max(float(og.abs().max()), 1e-30)
    assert e < 1e-5, e
    if gg is not None:
        bad = {}
        for k in gg:
            b = gg[k].numpy().astype(np.float64)
            e = np.abs(gf[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
            if e > 1e-5:
                bad[k] = "%.3g" % e
        assert not bad, bad


@pytest.mark.parametrize("N", [1, 4, 13, 16])
def test_conv12_small_matches_two_kernels(N):
    """conv1 + conv2 of a few envs at 174x174 in one launch (`conv12_small_kernel`: one
    workgroup per (frame, band) item runs conv1 on the band's X1 rows into LDS planes, then
    conv2 on them) against the two launches it replaces (`VN_CONV12_SMALL_OFF`:
    conv1_fwd_x3_kernel, then the banded conv2_fwd_x6_kernel): X1 and the ReLU bitmask bitwise
    (the same products in the same order, every X1 row stored by one workgroup), X2 to rounding
    (the ring kernel's two kernel-row halves vs the banded kernel's four partials: 2e-6 of
    scale), the logits / value to 1e-5, and every parameter gradient to 1e-5 of scale."""
    from vnav.policy import GoalNavPolicy, frames_from_batch
    torch.manual_seed(17)
    hw = (174, 174)
    pol = GoalNavPolicy(3, 4, hw)
    net = pol.net
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(7)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)
    m1, x1, x2 = 2 * 42 * 42, 2 * 42 * 42 * 32, 2 * 20 * 20 * 32

    def run(off):
        if off:
            os.environ["VN_CONV12_SMALL_OFF"] = "1"
        try:
            acts = net.new_acts(N)
            acts.fill_(float("nan"))
            out = torch.zeros((N, 8), device="cuda")
            net.forward(pol.params.detach(), frames_from_batch(img.view((N,) + hw + (3,)), gl.view((N,) + hw + (3,))),
                        N, acts, N, 0, out)
            M1 = acts[:N * m1].view(torch.int32).clone()
            X1 = acts[N * m1:N * (m1 + x1)].clone()
            X2 = acts[N * (m1 + x1):N * (m1 + x1 + x2)].clone()
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            return M1, X1, X2, out[:, :5].clone(), net.to_reference(pol.params.grad.clone())
        finally:
            os.environ.pop("VN_CONV12_SMALL_OFF", None)

    (mf, xf1, xf2, of, gf), (ms, xs1, xs2, os_, gs) = run(False), run(True)
    assert not torch.isnan(xf1).any() and not torch.isnan(xf2).any(), "unwritten activations"
    assert torch.equal(mf, ms) and torch.equal(xf1, xs1)
    e = float((xf2 - xs2).abs().max()) / float(xs2.abs().max())
    assert e < 2e-6, e
    e = float((of - os_).abs().max()) / max(float(os_.abs().max()), 1e-30)
    assert e < 1e-5, e
    bad = {}
    for k in gs:
        b = gs[k].numpy().astype(np.float64)
        e = np.abs(gf[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad


@pytest.mark.parametrize("hw,N", [((84, 84), 1), ((84, 84), 16), ((174, 174), 4), ((174, 174), 13)])
def test_conv34_small_matches_generic_products(hw, N):
    """conv3 + conv4 of a few envs (n <= 16) in one launch (`conv34_small_kernel`: exact fp32
    products per pixel, the k quarters summed in a fixed order) against the x6 products
    (`VN_CONV34_GENERIC`): logits, value and every parameter gradient to 1e-5 of scale."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(14)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(4)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)

    def run(generic):
        if generic:
            os.environ["VN_CONV34_GENERIC"] = "1"
        try:
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            return (logits.detach().cpu(), value.detach().cpu()), pol.net.to_reference(pol.params.grad.clone())
        finally:
            os.environ.pop("VN_CONV34_GENERIC", None)

    (of, gf), (og, gg) = run(False), run(True)
    for a, b in zip(of, og):
        e = float((a - b).abs().max()) / max(float(b.abs().max()), 1e-30)
        assert e < 1e-5, e
    bad = {}
    for k in gg:
        b = gg[k].numpy().astype(np.float64)
        e = np.abs(gf[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad


@pytest.mark.parametrize("N", [3, 300])
def test_conv2_band_dgrad_matches_class_products(N):
    """300x400 (74x99 conv1 map, odd width): conv2's input gradient on the banded x6 kernel
    (`conv2_dgrad_band_x6_kernel`: bands of 10 conv1 rows, the last one 4, class widths 50 / 49)
    against the four parity-class products (VN_DGRAD_GENERIC). It feeds conv1's weight
    gradient, which must agree to 1e-5 of scale; N = 300 wraps the persistent grid."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(13)
    hw = (300, 400)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(3)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)
    fast = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic=None))
    gen = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic="VN_DGRAD_GENERIC"))
    bad = {}
    for k in gen:
        b = gen[k].numpy().astype(np.float64)
        e = np.abs(fast[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad
    assert np.abs(fast["shared_base.0.0.weight"].numpy()).max() > 0


@pytest.mark.parametrize("hw,N", [((84, 84), 300), ((174, 174), 130), ((174, 174), 7), ((300, 400), 37)])
def test_conv1_resident_weights_matches_lds_fragments(hw, N):
    """conv1's forward with the split weights resident in registers (`conv1_fwd_x3r_kernel`,
    contiguous bf16 band rows, buffer-descriptor prefetch, med3 ReLU bits) against the
    LDS-fragment kernel it replaces (`VN_CONV1F_LDSW`): the same products in the same three
    chains and the same final sum, so X1 and the ReLU bitmask are bitwise equal (every frame,
    every band, the short last band of 174x174 and 300x400 included)."""
    from vnav.policy import GoalNavPolicy, frames_from_batch
    torch.manual_seed(23)
    pol = GoalNavPolicy(3, 4, hw)
    net = pol.net
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(5)
    img = torch.randint(0, 256, (N,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    oh, ow = (hw[0] - 7) // 4 + 1, (hw[1] - 7) // 4 + 1
    m1, x1 = 2 * oh * ow, 2 * oh * ow * 32

    def run(ldsw):
        if ldsw:
            os.environ["VN_CONV1F_LDSW"] = "1"
        try:
            acts = net.new_acts(N)
            acts.fill_(float("nan"))
            out = torch.zeros((N, 8), device="cuda")
            net.forward(pol.params.detach(), frames_from_batch(img, gl), N, acts, N, 0, out)
            torch.cuda.synchronize()
            return acts[:N * m1].view(torch.int32).clone(), acts[N * m1:N * (m1 + x1)].clone(), out[:, :5].clone()
        finally:
            os.environ.pop("VN_CONV1F_LDSW", None)

    (mr, xr, orr), (ml, xl, ol) = run(False), run(True)
    assert not torch.isnan(xr).any(), "unwritten X1"
    assert float(xl.abs().max()) > 0 and int((ml != 0).sum()) > 0
    assert torch.equal(mr, ml), int((mr != ml).sum())
    assert torch.equal(xr, xl), float((xr - xl).abs().max())
    assert torch.equal(orr, ol)


@pytest.mark.parametrize("N", [3, 130, 1031])
def test_conv2_ring_prefetch_matches_load_before_split(N):
    """conv2's forward ring kernel at 174x174 with band k + 2 prefetched through band k + 1's
    MFMAs (the default) against the form that loads each band just before its split
    (`VN_CONV2F_RING2_NOPF`): the same sums in the same order, X2 bitwise, including items past
    a workgroup's last band (the prefetch repeats the last item) and persistent-grid wraps."""
    from vnav.policy import GoalNavPolicy, frames_from_batch
    torch.manual_seed(29)
    hw = (174, 174)
    pol = GoalNavPolicy(3, 4, hw)
    net = pol.net
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(9)
    img = torch.randint(0, 256, (N,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N,) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    m1, x1, x2 = 2 * 42 * 42, 2 * 42 * 42 * 32, 2 * 20 * 20 * 32

    def run(nopf):
        if nopf:
            os.environ["VN_CONV2F_RING2_NOPF"] = "1"
        try:
            acts = net.new_acts(N)
            acts.fill_(float("nan"))
            out = torch.zeros((N, 8), device="cuda")
            net.forward(pol.params.detach(), frames_from_batch(img, gl), N, acts, N, 0, out)
            torch.cuda.synchronize()
            return acts[N * (m1 + x1):N * (m1 + x1 + x2)].clone(), out[:, :5].clone()
        finally:
            os.environ.pop("VN_CONV2F_RING2_NOPF", None)

    (xp, op), (xn, on) = run(False), run(True)
    assert not torch.isnan(xp).any() and float(xp.abs().max()) > 0
    assert torch.equal(xp, xn), float((xp - xn).abs().max())
    assert torch.equal(op, on)


@pytest.mark.parametrize("hw,N", [((174, 174), 61), ((300, 400), 9)])
def test_conv1_wgrad_lean_matches_masked_form(hw, N):
    """conv1's weight gradient with scalar lane masks for the dZ validity and no per-step
    B-fragment masking (`conv1_wgrad_x3_kernel<..., LEAN = true>`: pad slots left as read, the
    bias lane reading 8 bf16 ones) against the masked form (`VN_CONV1WG_NOLEAN`): the same
    products into the kept slots in the same order, so every parameter gradient is bitwise equal."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(31)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(11)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)

    def run(nolean):
        if nolean:
            os.environ["VN_CONV1WG_NOLEAN"] = "1"
        try:
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            return pol.params.grad.clone()
        finally:
            os.environ.pop("VN_CONV1WG_NOLEAN", None)

    gl_, gm = run(False), run(True)
    w, b = pol.net.offsets["conv1"]
    assert float(gm[w:w + 32 * 148].abs().max()) > 0 and float(gm[b:b + 32].abs().max()) > 0
    assert torch.equal(gl_, gm), float((gl_ - gm).abs().max())


@pytest.mark.parametrize("hw,N", [((84, 84), 37), ((174, 174), 77)])
def test_conv2_dgrad_rotated_matches_original(hw, N):
    """conv2's input gradient with the rotated item loop (stage the next frame after this frame's
    tiles; fixed tile-pair count, lanes past the class map storing to the slab's sink) against
    the original loop (`VN_CONV2DG_NOROT`): the same products and order, every parameter
    gradient bitwise equal (conv1's weight gradient reads the dX1 it writes)."""
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(37)
    pol = GoalNavPolicy(3, 4, hw)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator(device="cuda").manual_seed(13)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
    cl = torch.randn((N, 1, 4), device="cuda", generator=g)
    cv = torch.randn((N, 1, 1), device="cuda", generator=g)

    def run(norot):
        if norot:
            os.environ["VN_CONV2DG_NOROT"] = "1"
        try:
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            return pol.params.grad.clone()
        finally:
            os.environ.pop("VN_CONV2DG_NOROT", None)

    gr, go = run(False), run(True)
    w, _ = pol.net.offsets["conv1"]
    assert float(go[w:w + 32 * 148].abs().max()) > 0
    assert torch.equal(gr, go), float((gr - go).abs().max())

