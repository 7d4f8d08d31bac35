"""A/B helper for conv2's banded forward kernel (conv2_fwd_x6_kernel, 300x400 training batches
and 174x174 few-env batches with VN_CONV12_SMALL_OFF): hashes of the logits / value and of the
parameter gradients of a forward + backward, so two library builds can be compared bit for bit."""
import hashlib
import os
import sys

import torch

R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "a2cat-vn-pytorch_amd"))
import vnav  # noqa: E402


def h(t):
    return hashlib.sha1(t.detach().contiguous().cpu().numpy().tobytes()).hexdigest()[:12]


os.environ["VN_CONV12_SMALL_OFF"] = "1"
for hw, N in (((300, 400), 17), ((300, 400), 129), ((174, 174), 5)):
    torch.manual_seed(1)
    pol = vnav.GoalNavPolicy(3, 4, hw, aux=True)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    g = torch.Generator().manual_seed(2)
    img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, generator=g).cuda()
    gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, generator=g).cuda()
    logits, value, _ = pol(((img, gl), None), None, None)
    (logits.sum() + value.sum()).backward()
    torch.cuda.synchronize()
    print(hw, N, "out", h(logits), h(value), "grad", h(pol.params.grad), flush=True)
