"""A/B of conv2's forward at 174x174 in one process: the policy trunk forward over 4096
samples (8192 frames, one rollout step of the bench's 174x174 leg) with the ring kernels (two
workgroups per CU; VN_CONV2F_RING1: one) and with the generic im2col product (VN_CONV2F_GENERIC), alternating; prints the forward's device
time per call for both and the max relative difference of the conv_merge features. Run under
rocprofv3 --kernel-trace --stats for per-kernel times.

    python tools/ab/conv2f_ab.py [samples] [reps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "a2cat-vn-pytorch_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    from vnav.policy import PolicyNet, frames_from_batch
    torch.cuda.set_device(0)
    net = PolicyNet((174, 174), 4)
    params = net.init_params(0)
    g = torch.Generator(device="cuda").manual_seed(0)
    img = torch.randint(0, 256, (n, 174, 174, 3), dtype=torch.uint8, device="cuda", generator=g)
    gl = torch.randint(0, 256, (n, 174, 174, 3), dtype=torch.uint8, device="cuda", generator=g)
    fr = frames_from_batch(img, gl)
    acts = net.new_acts(n)
    out = torch.zeros((n, 8), device="cuda")
    res = {}
    feats = {}
    for rnd in range(2):
        for mode in ("ring", "ring1", "generic"):
            os.environ.pop("VN_CONV2F_GENERIC", None)
            os.environ.pop("VN_CONV2F_RING1", None)
            if mode == "generic":
                os.environ["VN_CONV2F_GENERIC"] = "1"
            elif mode == "ring1":
                os.environ["VN_CONV2F_RING1"] = "1"
            net.forward(params, fr, n, acts, n, 0, out)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                net.forward(params, fr, n, acts, n, 0, out)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / reps)
            feats[mode] = net.x5(acts, n).clone()
    os.environ.pop("VN_CONV2F_GENERIC", None)
    os.environ.pop("VN_CONV2F_RING1", None)
    d = (feats["ring"] - feats["generic"]).abs().max() / feats["generic"].abs().max()
    print({"samples": n, "forward_ms": res, "x5_max_rel_diff": float(d),
           "ring_vs_ring1_bitwise": bool(torch.equal(feats["ring"], feats["ring1"]))})


if __name__ == "__main__":
    main()
