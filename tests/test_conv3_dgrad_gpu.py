"""conv3's input gradient (k4 s2, 64 -> 2 x 32 channels): the persistent all-classes kernel
(`conv3_dgrad_x6_kernel`, vn_policy.hip) against the four generic parity-class products it
replaced (`VN_CONV3_DGRAD_GENERIC`, read per backward call). Both compute the same exact
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
        os.environ["VN_CONV3_DGRAD_GENERIC"] = "1"
    try:
        pol.params.grad = None
        logits, value, _ = pol(((img, gl), None), None, None)
        ((logits * cl).sum() + (value * cv).sum()).backward()
        torch.cuda.synchronize()
        return pol.params.grad.clone()
    finally:
        os.environ.pop("VN_CONV3_DGRAD_GENERIC", None)


@pytest.mark.parametrize("hw,N", [((84, 84), 37), ((84, 84), 1030), ((174, 174), 5), ((174, 174), 300)])
def test_conv3_dgrad_kernel_matches_class_products(hw, N):
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
    fast = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic=False))
    gen = pol.net.to_reference(_grads(pol, img, gl, cl, cv, generic=True))
    bad = {}
    for k in gen:
        b = gen[k].numpy().astype(np.float64)
        e = np.abs(fast[k].numpy() - b).max() / max(np.abs(b).max(), 1e-30)
        if e > 1e-5:
            bad[k] = "%.3g" % e
    assert not bad, bad
    # the kernel ran (not a no-op): conv3's input gradient reaches conv2's weights
    assert np.abs(fast["shared_base.0.2.weight"].numpy()).max() > 0
