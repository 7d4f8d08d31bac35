"""Max relative errors of tests/test_aux_gpu.py::test_aux_grads_large_batch_consistency_174
(1040-sample gradient vs the mean of 26 batches of 40) per parameter, with the conv2 ring
kernel and with the generic im2col product (VN_CONV2F_GENERIC). Diagnostic."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def run():
    from vnav.policy import GoalNavPolicy
    torch.manual_seed(1)
    pol = GoalNavPolicy(3, 4, (174, 174), aux=True)
    with torch.no_grad():
        pol.params.add_(torch.randn_like(pol.params) * 0.01)
    B, C = 1040, int(os.environ.get('AUX_C', '208'))
    rng = np.random.RandomState(9)
    img = torch.as_tensor(rng.randint(0, 256, size=(B, 1, 174, 174, 3)).astype(np.uint8)).cuda()
    gl = torch.as_tensor(rng.randint(0, 256, size=(B, 1, 174, 174, 3)).astype(np.uint8)).cuda()
    shapes = [p.shape[2:] for p in pol.forward_deconv(((img[:1], gl[:1]), None))[0]]
    targets = [torch.as_tensor(rng.rand(B, 1, *sh).astype(np.float32)).cuda() for sh in shapes]

    def grads(lo, hi):
        pol.params.grad = None
        preds, _ = pol.forward_deconv(((img[lo:hi], gl[lo:hi]), None))
        loss = sum(torch.nn.functional.mse_loss(p, t[lo:hi]) for p, t in zip(preds, targets))
        loss.backward()
        return pol.params.grad.detach().clone()

    full = grads(0, B)
    parts = [grads(k, k + C).double() for k in range(0, B, C)]
    gmean = sum(parts) / (B // C)
    mine, ref = pol.net.to_reference(full), pol.net.to_reference(gmean.float())
    out = {}
    for k in ref:
        b = ref[k].numpy().astype(np.float64)
        if np.abs(b).max() == 0.0:
            continue
        out[k] = float(np.abs(mine[k].numpy() - b).max() / np.abs(b).max())
    return out


if __name__ == "__main__":
    r = run()
    os.environ["VN_CONV2F_GENERIC"] = "1"
    g = run()
    for k in r:
        print("%-40s ring %.3g  generic %.3g" % (k, r[k], g[k]))
