"""Is conv2's ring-kernel output independent of the batch a frame is computed in? X2 of
samples [lo, lo+C) computed within a batch of B and as a batch of C (bitwise). Diagnostic."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)
import torch  # noqa: E402


def main():
    from vnav.policy import PolicyNet, frames_from_batch
    torch.cuda.set_device(0)
    net = PolicyNet((174, 174), 4)
    params = net.init_params(3)
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1040
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randint(0, 256, (B, 174, 174, 3), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (B, 174, 174, 3), dtype=torch.uint8, device="cuda", generator=g)
    m1, x1, x2 = 2 * 42 * 42, 2 * 42 * 42 * 32, 2 * 20 * 20 * 32

    def x2_of(lo, n):
        acts = net.new_acts(n)
        out = torch.zeros((n, 8), device="cuda")
        net.forward(params, frames_from_batch(img[lo:lo + n], gl[lo:lo + n]), n, acts, n, 0, out)
        torch.cuda.synchronize()
        return acts[n * (m1 + x1):n * (m1 + x1 + x2)].view(n, -1).clone()

    full = x2_of(0, B)
    for lo, c in ((0, 40), (520, 40), (B - 40, 40), (3, 17), (100, 300)):
        part = x2_of(lo, c)
        d = (full[lo:lo + c] - part).abs()
        print({"lo": lo, "n": c, "bitwise_equal": bool(torch.equal(full[lo:lo + c], part)),
               "max_abs_diff": float(d.max()), "n_diff": int((d > 0).sum())})
    again = x2_of(0, B)
    print({"rerun_bitwise_equal": bool(torch.equal(full, again))})


if __name__ == "__main__":
    main()
