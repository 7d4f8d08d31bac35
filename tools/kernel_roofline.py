#!/usr/bin/env python3
"""Roofline table of the training kernels of one A2C update from a rocprofv3 kernel trace of
bench.py: per kernel the measured time per update, its algorithmic FLOPs (fp32-equivalent,
one multiply-add = 2) and the bytes it must move through HBM, the rates, and the fraction of
the ceilings that bound it — the fp32 MFMA peak (157.3 TF), the bf16 MFMA rate divided by the
products each fp32 product costs (x6: 2.5 PF / 6, x3: 2.5 PF / 3) and HBM (8 TB/s).

    python tools/kernel_roofline.py TRACE.csv UPDATE_INDEX GEOMETRY(84|174) [E] [T]
"""
import collections
import csv
import re
import sys

FP32 = 157.3e12
BF16 = 2.5e15
HBM = 8.0e12


def geo(h):
    o1 = (h - 7) // 4 + 1
    o2 = (o1 - 4) // 2 + 1
    o3 = (o2 - 4) // 2 + 1
    return o1, o2, o3


def table(h, E, T):
    o1, o2, o3 = geo(h)
    p1, p2, p3 = o1 * o1, o2 * o2, o3 * o3
    fb = h * h * 3
    N = E * T
    F = 2 * N                 # frames in the update (image + goal)
    fs = 2 * E                # frames per rollout step
    fcin = p3 * 32
    xcat = 1032
    f4 = 4
    # name regex -> (per-call FLOPs, per-call bytes, MFMA form)
    return [
        (r"conv1_fwd_x3_kernel", fs * p1 * 32 * 147 * 2, fs * (fb + p1 * 32 * f4 + p1 * 4), "x3"),
        (r"conv2_fwd_x6_kernel|conv2_fwd_ring2?_kernel|NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 1>, DenseRows, EpiBiasAct" % (o1, o1, o2, o2),
         fs * p2 * 32 * 512 * 2, fs * (p1 + p2) * 32 * f4, "x6"),
        (r"NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 2>, DenseRows, EpiBiasAct" % (o2, o2, o3, o3),
         E * p3 * 64 * 1024 * 2, E * (2 * p2 * 32 + p3 * 64) * f4, "x6"),
        (r"EpiBias2", E * 2048 * xcat * 2, (E * xcat + 2048 * xcat + E * 2048) * f4, "x6"),
        (r"conv1_wgrad_x3_kernel<", F * p1 * 32 * 147 * 2, F * (fb + p1 * 32 * f4), "x3"),
        (r"conv2_wgrad_kernel", F * p2 * 32 * 512 * 2, F * (p1 + p2) * 32 * f4, "f32"),
        (r"WgSpec<%d, %d, %d, %d, 32, 1," % (o1, o1, o2, o2), F * p2 * 32 * 512 * 2, F * (p1 + p2) * 32 * f4, "x6"),
        (r"conv2_dgrad_x6_kernel", F * p2 * 32 * 512 * 2, F * (p2 * 32 * f4 + p1 * 32 * f4 + p1 * 4), "x6"),
        (r"RowsOnes, EpiSlab", N * 2048 * (xcat + 1) * 2, N * (2048 + xcat) * f4, "x6"),
        (r"EpiLstmDh", E * 512 * 2048 * 2, (E * 2048 + 2048 * 512 + E * 512) * f4, "x6"),
        (r"Im2colT<NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 2> >, EpiSlab" % (o2, o2, o3, o3),
         N * p3 * 64 * 1024 * 2, N * (2 * p2 * 32 + p3 * 64) * f4, "x6"),
        (r"WgSpec<%d, %d, %d, %d, 64, 2," % (o2, o2, o3, o3), N * p3 * 64 * 1024 * 2, N * (2 * p2 * 32 + p3 * 64) * f4, "x6"),
        (r"DgradA<64, 4, 2, %d, %d" % (o3, o3), N * p3 * 64 * 1024 * 2 / 4, None, "x6"),  # per class: 1/4 of the total
        (r"ParityDg<%d, %d, \d+, \d+, 64, 64, 2>" % (o3, o3), N * p3 * 64 * 1024 * 2, N * (p3 * 64 + 2 * 2 * p2 * 32) * f4, "x6"),
        (r"128, 128, 32, 2, 2, DenseRows, DenseRows, EpiMask>", N * 512 * 2048 * 2, (N * 2048 + N * 512 * 2) * f4, "x6"),
    ]


def main():
    path, upd, h = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    E = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    T = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ups, cur = [], []
    for r in rows:
        cur.append(r)
        if "rmsprop" in r["Kernel_Name"]:
            ups.append(cur)
            cur = []
    u = ups[upd - 1]
    agg = collections.defaultdict(lambda: [0, 0.0, ""])
    for r in u:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        kname = r["Kernel_Name"].replace("vn::", "")
        for pat, fl, by, form in table(h, E, T):
            if re.search(pat, kname):
                a = agg[pat]
                a[0] += 1
                a[1] += d
                a[2] = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("vn::", "")[:60]
                break
    total = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in u)
    print("update %d (%dx%d, E=%d, T=%d): %d dispatches, %.2f ms of kernel time" % (upd, h, h, E, T, len(u), total * 1e3))
    print("| kernel | calls | ms / update | GFLOP | GB | TFLOP/s | of fp32 peak | MFMA form | of its bf16 ceiling | "
          "TB/s | of HBM |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for pat, fl, by, form in table(h, E, T):
        if pat not in agg:
            continue
        c, t, name = agg[pat]
        flops = fl * c
        tf = flops / t / 1e12
        ceil = {"x6": BF16 / 6, "x3": BF16 / 3, "f32": FP32}[form]
        gb = by * c / 1e9 if by else None
        bw = by * c / t / 1e12 if by else None
        print("| `%s` | %d | %.2f | %.0f | %s | %.1f | %.2f | %s | %.2f | %s | %s |" % (
            name, c, t * 1e3, flops / 1e9, "%.1f" % gb if gb else "—", tf, tf * 1e12 / FP32, form,
            tf * 1e12 / ceil, "%.2f" % bw if bw else "—", "%.2f" % (bw * 1e12 / HBM) if bw else "—"))


if __name__ == "__main__":
    main()
