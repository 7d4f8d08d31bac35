import os, sys, torch
sys.path.insert(0, "a2cat-vn-pytorch_amd"); sys.path.insert(0, ".")
from vnav.policy import GoalNavPolicy
for aux in (False, True):
    for N in (1, 77, 1031):
        torch.manual_seed(41)
        hw = (174, 174)
        pol = GoalNavPolicy(3, 4, hw, recurrent=False, aux=aux)
        with torch.no_grad():
            pol.params.add_(torch.randn_like(pol.params) * 0.01)
        g = torch.Generator(device="cuda").manual_seed(17)
        img = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
        gl = torch.randint(0, 256, (N, 1) + hw + (3,), dtype=torch.uint8, device="cuda", generator=g)
        cl = torch.randn((N, 1, 4), device="cuda", generator=g)
        cv = torch.randn((N, 1, 1), device="cuda", generator=g)
        outs = []
        for rep in range(3):
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            outs.append(pol.params.grad.clone())
        d = [float((outs[0] - o).abs().max()) for o in outs[1:]]
        print("aux", aux, "N", N, "max diff vs run0:", d, "finite", bool(torch.isfinite(outs[0]).all()), flush=True)
