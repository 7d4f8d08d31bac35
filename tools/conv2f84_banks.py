"""Exhaustive LDS bank check of conv2_fwd_x6_kernel's X1 planes at 84x84 frames (20x20 -> 9x9,
vn_conv1.h Conv2FwdBand): the row-major tiles at pixel stride 40 against the 2x8 tiles
(`pix2x8`) on unpadded pixels with the odd-x plane 352 bf16 and rows 680 bf16 apart. Same
model as tools/ring_banks.py: the 4 lane groups of a B-fragment ds_read_b128 (bank of a 16-B
quad = quad mod 16, identical addresses broadcast) and 16-lane groups of the split's
ds_write_b64 (bank = dword mod 32). Prints the extra LDS cycles summed over one frame.

    python tools/conv2f84_banks.py
"""
from collections import defaultdict

GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
          [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31],
          [32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59],
          [36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63]]
IW, OW, WH = 20, 9, 10


def layouts():
    yield "row-major, PSX 40", dict(PSX=40, PO=WH * 40, RSP=2 * WH * 40, tiled=False)
    yield "2x8 tiles, PSX 32", dict(PSX=32, PO=352, RSP=680, tiled=True)


def pixel(L, t, i):
    if not L["tiled"]:
        p = min(t * 16 + i, OW * OW - 1)
        return p // OW, p % OW
    if t < 4:
        return 2 * t + (i >> 3), i & 7
    if t == 4:
        return (8, i) if i < 8 else (i - 8, 8)
    return 8, 8


def extra(addrs, nbanks):
    banks = defaultdict(set)
    for a in addrs:
        banks[a % nbanks].add(a)
    return max(len(v) for v in banks.values()) - 1


def main():
    for name, L in layouts():
        rd = 0
        for ky in range(4):
            for t in range(6):
                for kx in range(4):
                    for g in GROUPS:
                        quads = []
                        for lane in g:
                            oy, ox = pixel(L, t, lane & 15)
                            e = (2 * oy + ky) * L["RSP"] + ox * L["PSX"] + 8 * (lane >> 4)
                            e += (kx & 1) * L["PO"] + (kx >> 1) * L["PSX"]
                            quads.append(e // 8)
                        rd += extra(quads, 16)
        wr = 0
        for base in range(0, IW * IW * 8, 16):
            dws = []
            for i in range(base, base + 16):
                c4, px = i & 7, i >> 3
                y, x = px // IW, px % IW
                d = (y * L["RSP"] + (x & 1) * L["PO"] + (x >> 1) * L["PSX"] + 4 * c4) // 2
                dws += [d, d + 1]
            wr += extra(dws, 32)
        print({"layout": name, "read_extra_cycles": rd, "write_extra_cycles": wr})


if __name__ == "__main__":
    main()
