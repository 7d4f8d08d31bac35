"""Repeat det_check's sequence (six policies per pass) and report every non-finite gradient, with
the kernel switches of the pass (debug aid for an intermittent non-finite gradient seen once)."""
import os, sys, torch
sys.path.insert(0, "a2cat-vn-pytorch_amd"); sys.path.insert(0, ".")
from vnav.policy import GoalNavPolicy
passes = [[], ["VN_CONV1F_LDSW", "VN_CONV1WG_NOLEAN", "VN_CONV2DG_NOROT", "VN_CONV2F_RING2_NOPF", "VN_CONV3F_GATHER"]] * 3
seq = [(False, 1), (False, 77), (False, 1031), (True, 1), (True, 77), (True, 1031)]
bad_total = 0
for pi, flags in enumerate(passes):
    for f in flags: os.environ[f] = "1"
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
        ref = None
        for rep in range(3):
            pol.params.grad = None
            logits, value, _ = pol(((img, gl), None), None, None)
            ((logits * cl).sum() + (value * cv).sum()).backward()
            torch.cuda.synchronize()
            gr = pol.params.grad.clone()
            nf = int((~torch.isfinite(gr)).sum())
            if nf:
                bad = [n for n, (w, b) in pol.net.offsets.items() if pol.net.shapes[n][0] and not (
                    torch.isfinite(gr[w:w + pol.net.shapes[n][0] * pol.net.shapes[n][1]]).all() and
                    torch.isfinite(gr[b:b + pol.net.shapes[n][0]]).all())]
                print("NONFINITE pass", pi, flags, "aux", aux, "N", N, "rep", rep, nf, bad, flush=True)
                bad_total += 1
            if ref is None:
                ref = gr
            elif not torch.equal(ref.nan_to_num(7.0), gr.nan_to_num(7.0)):
                print("NONDETERMINISTIC pass", pi, flags, "aux", aux, "N", N, "rep", rep,
                      float((ref - gr).abs().nan_to_num(0).max()), flush=True)
                bad_total += 1
        del pol
    for f in flags: os.environ.pop(f, None)
    print("pass", pi, "done", flush=True)
print("bad", bad_total)
