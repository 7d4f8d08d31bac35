"""Which gradient blocks go non-finite for GoalNavPolicy(aux=True) at 174x174, N samples, and
under which kernel switches (debug aid)."""
import os, sys, torch
sys.path.insert(0, "a2cat-vn-pytorch_amd"); sys.path.insert(0, ".")
from vnav.policy import GoalNavPolicy
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1031
hw = (174, 174)
for flags in ([], ["VN_CONV1F_LDSW"], ["VN_CONV1WG_NOLEAN"], ["VN_CONV2DG_NOROT"], ["VN_CONV2F_RING2_NOPF"]):
    for aux in (True, False):
        for f in flags: os.environ[f] = "1"
        torch.manual_seed(41)
        pol = GoalNavPolicy(3, 4, hw, recurrent=False, aux=aux)
        with torch.no_grad():
            pol.params.add_(torch.randn_like(pol.params) * 0.01)
        g = torch.Generator(device="cuda").manual_seed(17)
        img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
        gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
        cl = torch.randn((N, 1, 4), device="cuda", generator=g)
        cv = torch.randn((N, 1, 1), device="cuda", generator=g)
        pol.params.grad = None
        logits, value, _ = pol(((img, gl), None), None, None)
        ok_out = bool(torch.isfinite(logits).all() and torch.isfinite(value).all())
        ((logits * cl).sum() + (value * cv).sum()).backward()
        torch.cuda.synchronize()
        gr = pol.params.grad
        bad = []
        for name, (w, b) in pol.net.offsets.items():
            co, k = pol.net.shapes[name]
            if co and not (torch.isfinite(gr[w:w + co * k]).all() and torch.isfinite(gr[b:b + co]).all()):
                bad.append(name)
        print(flags, "aux", aux, "N", N, "outputs finite", ok_out, "non-finite grad blocks", bad,
              "all finite", bool(torch.isfinite(gr).all()), flush=True)
        for f in flags: os.environ.pop(f, None)
        del pol
