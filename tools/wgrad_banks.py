"""LDS bank model of conv_wgrad_x6_kernel (csrc/vn_policy.hip): the split dZ / X planes'
staging stores (ds_write_b64: 4 groups of 16 contiguous lanes, bank = dword mod 32) under
the former slot order (row i / Q) and wg_slot's (rows r, r + D per 16-lane group), and the
transpose reads of both operands (ds_read_b64_tr_b16: 2 groups of 32 lanes, bank = dword mod
64), per MI355X_MICROARCH.md's LDS table. Extra LDS cycles / instruction groups.

    python tools/wgrad_banks.py
"""
from collections import defaultdict


def wg_slot(i, Q, rstride, rows):
    D = 4 if (Q == 8 and rstride % 32 == 20) else 2 if (Q == 8 and rstride % 32 == 24) else 0
    c, t = i % Q, i // Q
    if D == 0:
        return t, c
    full = rows // (2 * D) * (2 * D)
    m = t % (2 * D)
    return (t - m + (m >> 1) + (m & 1) * D if t < full else t), c


def writes(rows, Q, pstride, permuted):
    ex = n = 0
    for base in range(0, rows * Q, 16):
        b = defaultdict(set)
        for i in range(base, min(base + 16, rows * Q)):
            r, c = wg_slot(i, Q, pstride // 2, rows) if permuted else (i // Q, i % Q)
            d = (r * pstride + 4 * c) // 2
            for x in (d, d + 1):
                b[x % 32].add(x)
        ex += max(len(v) for v in b.values()) - 1
        n += 1
    return ex, n


def reads(IH, IW, OH, OW, CO, BR, IMG, CX):
    kperm = CX == 32
    PZ, PX = CO + (16 if kperm else 8), CX + 8
    XR = min(2 * BR + 2, IH)
    NPX, KP, BP = XR * IW, IMG * BR * OW, BR * OW
    out = {"z": [0, 0], "x": [0, 0]}
    for wave in range(8):
        for ks in range((KP + 31) // 32):
            for s in range(2):
                for half in range(2):
                    zb = [defaultdict(set) for _ in range(CO // 16)]
                    xb = [defaultdict(set) for _ in range(2 * (CX // 16))]
                    for lane in range(32 * half, 32 * half + 32):
                        Gq, q, p = lane >> 4, (lane >> 2) & 3, lane & 3
                        k = ks * 32 + 16 * (Gq >> 1) + 8 * s + 4 * (Gq & 1) + q if kperm else ks * 32 + 8 * Gq + 4 * s + q
                        im, o = k // BP, k % BP
                        oy, ox = o // OW, o % OW
                        ok = k < KP
                        for mt in range(CO // 16):
                            d = ((k if ok else KP) * PZ + 16 * mt + 4 * p) // 2
                            for x in (d, d + 1):
                                zb[mt][x % 64].add(x)
                        for nt in range(2 * (CX // 16)):
                            tap = 2 * wave + nt // (CX // 16)
                            row = im * NPX + (2 * oy + (tap >> 2)) * IW + 2 * ox + (tap & 3) if ok else IMG * NPX
                            d = (row * PX + 16 * (nt % (CX // 16)) + 4 * p) // 2
                            for x in (d, d + 1):
                                xb[nt][x % 64].add(x)
                    for key, bs in (("z", zb), ("x", xb)):
                        for b in bs:
                            out[key][0] += max(len(v) for v in b.values()) - 1
                            out[key][1] += 1
    return out


def main():
    for name, a in (("conv2 174 WgSpec<42,42,20,20,32,1,4,1>", (42, 42, 20, 20, 32, 4, 1, 32)),
                    ("conv3 174 WgSpec<20,20,9,9,64,2,9,1>", (20, 20, 9, 9, 64, 9, 1, 32)),
                    ("aux 174 WgSpec<20,20,9,9,32,1,9,1,48>", (20, 20, 9, 9, 32, 9, 1, 48))):
        IH, IW, OH, OW, CO, BR, IMG, CX = a
        kperm = CX == 32
        PZ, PX = CO + (16 if kperm else 8), CX + 8
        KP = IMG * BR * OW
        NPX = min(2 * BR + 2, IH) * IW * IMG
        r = reads(*a)
        print("%-40s z writes %s -> %s, x writes %s -> %s; tr reads z %s x %s" % (
            name, writes(KP, CO // 4, PZ, False), writes(KP, CO // 4, PZ, True),
            writes(NPX, CX // 4, PX, False), writes(NPX, CX // 4, PX, True), tuple(r["z"]), tuple(r["x"])))


if __name__ == "__main__":
    main()
