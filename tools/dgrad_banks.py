"""LDS bank model of the k4 s2 input-gradient kernels' split planes: conv2_dgrad_x6_kernel
(csrc/vn_conv1.h; 84x84: 20x20 conv1 map, 174x174: 42x42) and parity_dgrad_x6_kernel
(csrc/vn_policy.hip; conv3's dZ3 9x9 -> 20x20 with 64 channels, the aux / pixel-control
first deconvs with 32). Counts, per wave-instruction, the extra LDS cycles of
  * the A-fragment ds_read_b128 (4 groups of 16 lanes, MI355X_MICROARCH.md §LDS:
    {0-3,12-15,20-27}, ...; a 16-B quad's bank = quad mod 16), lane (i16, q) = (class pixel
    of the 16-pixel tile, quad), for every tile and tap,
  * the staging ds_write_b64 (4 x 16 contiguous lanes, bank = dword mod 32),
for the former layout (pixel rows padded to KC + 8 bf16, one shared zero row for
out-of-range taps) and the current one (row (oy + 1) XC + ox + 1: consecutive rows per tile,
quads rotated per row, dg_quad_off).

    python tools/dgrad_banks.py
"""
from collections import defaultdict

G128 = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
        [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31],
        [32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59],
        [36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63]]


def new_quad(r, qq, nq):
    return r * nq + ((qq + 2 * (r >> 2)) & 3 if nq == 4 else (qq + r) & 7)


def old_quad(r, qq, kc):
    return r * (kc + 8) // 8 + qq


def model(SH, SW, KC, img, layout):
    XC, YC = SW + 1, SH + 1
    NP, NPC = SH * SW, YC * XC
    nq = KC // 8
    tiles = (img * NPC + 15) // 16
    zero = img * NP
    rd = rb = 0
    for t in range(tiles):
        for tap in range(4):
            ty, tx = tap >> 1, tap & 1
            rows = []
            for i16 in range(16):
                pc = t * 16 + i16
                if layout == "new":
                    rows.append(pc + (1 - ty) * XC + (1 - tx))
                    continue
                im, r = pc // NPC, pc % NPC
                oy, ox = r // XC - ty, r % XC - tx
                ok = pc < img * NPC and 0 <= oy < SH and 0 <= ox < SW
                rows.append(im * NP + oy * SW + ox if ok else zero)
            for h in range(KC // 32):
                for g in G128:
                    banks = defaultdict(set)
                    for lane in g:
                        qq = (lane >> 4) + 4 * h
                        a = new_quad(rows[lane & 15], qq, nq) if layout == "new" else old_quad(rows[lane & 15], qq, KC)
                        banks[a % 16].add(a)
                    rd += max(len(v) for v in banks.values()) - 1
                    rb += 1
    wr = wb = 0
    c4 = KC // 4
    n = img * NP * c4
    for base in range(0, n, 16):
        banks = defaultdict(set)
        for i in range(base, min(base + 16, n)):
            pix, c = i // c4, i % c4
            im, rem = pix // NP, pix % NP
            if layout == "new":
                r = im * NPC + (rem // SW + 1) * XC + rem % SW + 1
                d = new_quad(r, c >> 1, nq) * 4 + (c & 1) * 2
            else:
                d = (pix * (KC + 8) + 4 * c) // 2
            for x in (d, d + 1):
                banks[x % 32].add(x)
        wr += max(len(v) for v in banks.values()) - 1
        wb += 1
    return rd / rb, wr / wb


def main():
    cases = (("conv2_dgrad 84x84 (dZ2 9x9, 32 ch)", 9, 9, 32, 1),
             ("conv2_dgrad 174x174 (dZ2 20x20, 32 ch)", 20, 20, 32, 1),
             ("parity_dgrad conv3 174x174 (dZ3 9x9, 64 ch, 2 images)", 9, 9, 64, 2),
             ("parity_dgrad aux/pc 174x174 (X4 9x9, 32 ch, 2 images)", 9, 9, 32, 2),
             ("parity_dgrad aux 84x84 (X4 3x3, 32 ch, 4 images)", 3, 3, 32, 4))
    for name, sh, sw, kc, img in cases:
        o, n = model(sh, sw, kc, img, "old"), model(sh, sw, kc, img, "new")
        print("%-55s extra cycles per group: reads %.2f -> %.2f, writes %.2f -> %.2f" % (name, o[0], n[0], o[1], n[1]))


if __name__ == "__main__":
    main()
