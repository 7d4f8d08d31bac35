#!/usr/bin/env python3
"""Roofline table of the training kernels of one A2C update from a rocprofv3 kernel trace of
bench.py: per kernel group the measured time per update, its executed FLOPs (fp32-equivalent,
one multiply-add = 2) and the bytes it must move through HBM, the rates, and the fraction of
the ceilings that bound it — the fp32 MFMA peak (157.3 TF), the bf16 MFMA rate divided by the
products each fp32 product costs (x6: 2.5 PF / 6, x3: 2.5 PF / 3) and HBM (8 TB/s).

    python tools/kernel_roofline.py TRACE.csv UPDATE_INDEX H W [E] [T] [GOAL_FWD] [GOAL_BWD]

GOAL_FWD / GOAL_BWD: the fraction of goal frames whose shared_base ran in the rollout forward /
the update's backward (bench.py's goal_frames_computed; 1 without goal-run deduplication).
The update is split at each rmsprop kernel; UPDATE_INDEX counts from 1.
"""
import collections
import csv
import re
import sys

FP32 = 157.3e12
BF16 = 2.5e15
HBM = 8.0e12


def geo(h, w):
    o1 = ((h - 7) // 4 + 1, (w - 7) // 4 + 1)
    o2 = ((o1[0] - 4) // 2 + 1, (o1[1] - 4) // 2 + 1)
    o3 = ((o2[0] - 4) // 2 + 1, (o2[1] - 4) // 2 + 1)
    return o1, o2, o3


def table(h, w, E, T, gf=1.0, gb=1.0):
    """(regex, FLOPs per update, HBM bytes per update or None, MFMA form) per kernel group."""
    (a1, b1), (a2, b2), (a3, b3) = geo(h, w)
    p1, p2, p3 = a1 * b1, a2 * b2, a3 * b3
    fb = h * w * 3
    N = E * T
    Ff = N * (1 + gf) + 2 * E  # conv1 / conv2 forward frames: the rollout + the bootstrap
    Fb = N * (1 + gb)          # frames of the conv1 / conv2 backward
    fcin = p3 * 32
    xcat = 1032
    f4 = 4
    c1 = p1 * 32 * 147 * 2     # FLOPs per frame
    c2 = p2 * 32 * 512 * 2
    c3 = p3 * 64 * 1024 * 2    # per sample
    x1, x2 = p1 * 32 * f4, p2 * 32 * f4
    lstm = E * 2048 * xcat * 2
    return [
        (r"conv1_fwd_x3r?_kernel", Ff * c1, Ff * (fb + x1 + p1 * 4), "x3"),
        (r"conv2_fwd_x6_kernel|conv2_fwd_ring2?_kernel|(NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 1>|FrameListIm2col<%d, %d, %d, %d>), "
         r"DenseRows, (EpiBiasAct|EpiBiasActFrames)" % (a1, b1, a2, b2, a1, b1, a2, b2), Ff * c2, Ff * (x1 + x2), "x6"),
        (r"(NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 2>|NhwcIm2colGoalF?<32, 4, 4, 2, %d, %d, %d, %d>), DenseRows, "
         r"EpiBiasAct" % (a2, b2, a3, b3, a2, b2, a3, b3), (N + E) * c3, (N + E) * (2 * x2 + p3 * 64 * f4), "x6"),
        (r"EpiBias2", (T + 1) * lstm, (T + 1) * (E * xcat + 2048 * xcat + E * 2048) * f4, "x6"),
        (r"conv1_wgrad_x3_kernel<", Fb * c1, Fb * (fb + x1), "x3"),
        (r"conv2_wgrad_kernel", Fb * c2, Fb * (x1 + x2), "f32"),
        (r"WgSpec<%d, %d, %d, %d, 32, 1," % (a1, b1, a2, b2), Fb * c2, Fb * (x1 + x2), "x6"),
        (r"conv2_dgrad_x6_kernel|conv2_dgrad_band_x6_kernel", Fb * c2, Fb * (x2 + x1 + p1 * 4), "x6"),
        (r"DgradA<32, 4, 2, %d, %d" % (a2, b2), Fb * c2 / 4, None, "x6"),  # per class product
        (r"goal_dz2_reduce_kernel", 0, N * x2 + N * gb * 2 * x2, "hbm"),
        (r"RowsOnes, EpiSlab", N * 2048 * (xcat + 1) * 2, N * (2048 + xcat) * f4, "x6"),
        (r"EpiLstmDh", T * E * 512 * 2048 * 2, T * (E * 2048 + 2048 * 512 + E * 512) * f4, "x6"),
        (r"Im2colT<(NhwcIm2col<32, 4, 4, 2, %d, %d, %d, %d, 2>|NhwcIm2colGoal<32, 4, 4, 2, %d, %d, %d, %d>) >, EpiSlab"
         % (a2, b2, a3, b3, a2, b2, a3, b3), N * c3, N * (2 * x2 + p3 * 64 * f4), "x6"),
        (r"WgSpec<%d, %d, %d, %d, 64, 2," % (a2, b2, a3, b3), N * c3, N * (2 * x2 + p3 * 64 * f4), "x6"),
        (r"DgradA<64, 4, 2, %d, %d" % (a3, b3), N * c3 / 4, None, "x6"),  # per class product
        (r"ParityDg<%d, %d, \d+, \d+, 64, 64, 2>" % (a3, b3), N * c3, N * (p3 * 64 * f4 + 2 * 2 * x2), "x6"),
        (r"128, 128, 32, 2, 2, DenseRows, DenseRows, EpiMask>", N * 512 * 2048 * 2, (N * 2048 + N * 512 * 2) * f4,
         "x6"),
        (r"DenseRows, DenseRows, EpiBiasAct>", (N + E) * fcin * 512 * 2, (N + E) * (fcin + 512) * f4, "x6"),
    ]


def main():
    path, upd = sys.argv[1], int(sys.argv[2])
    h, w = int(sys.argv[3]), int(sys.argv[4])
    E = int(sys.argv[5]) if len(sys.argv) > 5 else 4096
    T = int(sys.argv[6]) if len(sys.argv) > 6 else 20
    gf = float(sys.argv[7]) if len(sys.argv) > 7 else 1.0
    gb = float(sys.argv[8]) if len(sys.argv) > 8 else gf
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ups, cur = [], []
    for r in rows:
        cur.append(r)
        if "rmsprop" in r["Kernel_Name"]:
            ups.append(cur)
            cur = []
    u = ups[upd - 1]
    tab = table(h, w, E, T, gf, gb)
    agg = collections.defaultdict(lambda: [0, 0.0, ""])
    for r in u:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        kname = r["Kernel_Name"].replace("vn::", "")
        for pat, fl, by, form in tab:
            if re.search(pat, kname):
                a = agg[pat]
                a[0] += 1
                a[1] += d
                a[2] = re.sub(r"\(.*$", "", r["Kernel_Name"]).replace("void ", "").replace("vn::", "")[:60]
                break
    total = sum((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in u)
    print("update %d (%dx%d, E=%d, T=%d, goal frames computed: forward %.3f, backward %.3f): %d dispatches, "
          "%.2f ms of kernel time" % (upd, h, w, E, T, gf, gb, len(u), total * 1e3))
    print("| kernel | calls | ms / update | GFLOP (executed) | GB | TFLOP/s | of fp32 peak | MFMA form | "
          "of its issued ceiling | TB/s | of HBM |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    for pat, fl, by, form in tab:
        if pat not in agg:
            continue
        c, t, name = agg[pat]
        nper = c if "DgradA" in pat else 1  # per-class products: FLOPs are per call
        flops = fl * nper
        tf = flops / t / 1e12
        ceil = {"x6": BF16 / 6, "x3": BF16 / 3, "f32": FP32, "hbm": None}[form]
        bw = by / t / 1e12 if by else None
        print("| `%s` | %d | %.2f | %.0f | %s | %.1f | %.2f | %s | %s | %s | %s |" % (
            name, c, t * 1e3, flops / 1e9, "%.1f" % (by / 1e9) if by else "—", tf, tf * 1e12 / FP32, form,
            "%.2f" % (tf * 1e12 / ceil) if ceil else "—", "%.2f" % bw if bw else "—",
            "%.2f" % (bw * 1e12 / HBM) if bw else "—"))


if __name__ == "__main__":
    main()
