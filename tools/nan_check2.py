"""det_check's sequence (six policies in one process) with the non-finite gradient blocks of every
run printed (debug aid)."""
import os, sys, torch
sys.path.insert(0, "a2cat-vn-pytorch_amd"); sys.path.insert(0, ".")
from vnav.policy import GoalNavPolicy
seq = [(False, 1), (False, 77), (False, 1031), (True, 1), (True, 77), (True, 1031)]
if len(sys.argv) > 1:
    seq = seq[int(sys.argv[1]):]
for aux, N in seq:
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
    for rep in range(3):
        pol.params.grad = None
        logits, value, _ = pol(((img, gl), None), None, None)
        ok = bool(torch.isfinite(logits).all() and torch.isfinite(value).all())
        ((logits * cl).sum() + (value * cv).sum()).backward()
        torch.cuda.synchronize()
        gr = pol.params.grad
        bad = [n for n, (w, b) in pol.net.offsets.items() if pol.net.shapes[n][0] and not (
            torch.isfinite(gr[w:w + pol.net.shapes[n][0] * pol.net.shapes[n][1]]).all() and
            torch.isfinite(gr[b:b + pol.net.shapes[n][0]]).all())]
        nf = int((~torch.isfinite(gr)).sum())
        print("aux", aux, "N", N, "rep", rep, "outputs finite", ok, "non-finite", nf, bad, flush=True)
