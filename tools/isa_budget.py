#!/usr/bin/env python3
"""Per-basic-block instruction budget of one kernel in a hipcc -S (gfx950) listing.

    hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -o vn_policy.s csrc/vn_policy.hip
    python tools/isa_budget.py vn_policy.s conv1_fwd_x3_kernelILi174 [--md]

Counts, per basic block (label to label): MFMA, VALU (v_* other than MFMA; v_cvt / v_perm /
v_cndmask / v_lshl / v_or / v_and / v_add / v_fma / v_max split out), LDS reads and writes,
global/buffer loads and stores, s_waitcnt (with their vmcnt / lgkmcnt arguments), s_barrier,
SALU and branches. Blocks that end in a backward branch are marked as loop latches; the
static counts of the tile loop body (the block(s) holding the MFMAs) are the per-tile budget.
"""
import re
import sys
from collections import Counter, OrderedDict

CATS = [
    ("mfma", re.compile(r"^v_mfma")),
    ("ds_read", re.compile(r"^ds_read|^ds_load")),
    ("ds_write", re.compile(r"^ds_write|^ds_store")),
    ("vmem_load", re.compile(r"^(global_load|buffer_load|flat_load)")),
    ("vmem_store", re.compile(r"^(global_store|buffer_store|flat_store)")),
    ("smem", re.compile(r"^s_load|^s_buffer_load")),
    ("waitcnt", re.compile(r"^s_waitcnt")),
    ("barrier", re.compile(r"^s_barrier")),
    ("branch", re.compile(r"^s_(cbranch|branch)")),
    ("nop", re.compile(r"^s_nop")),
    ("v_cvt", re.compile(r"^v_cvt")),
    ("v_perm/bfe/alignbit", re.compile(r"^v_(perm|bfe|alignbit|alignbyte|bfi)")),
    ("v_add/sub/mad int", re.compile(r"^v_(add|sub|mad|mul|lshl_add|add3|lshl_or|or3|and_or|subrev)_(u|i|co|nc|lshl)")),
    ("v_shift/logic", re.compile(r"^v_(lshl|lshr|ashr|and|or|xor|not)")),
    ("v_cndmask/cmp", re.compile(r"^v_(cndmask|cmp)")),
    ("v_f32 arith", re.compile(r"^v_(add|sub|mul|fma|fmac|max|min|pk_add|pk_fma|pk_mul|max3|min3|med3)_f32")),
    ("v_mov/accvgpr", re.compile(r"^v_(mov|accvgpr|readfirstlane|readlane|writelane)")),
    ("v_other", re.compile(r"^v_")),
    ("salu", re.compile(r"^s_")),
]


def kernel_lines(path, needle):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and re.match(r"^_Z\S*:", l) and needle in l.split(":")[0]:
            start = i
            name = l.split(":")[0]
        elif start is not None and (l.startswith(".Lfunc_end") or re.match(r"^\s*\.size\s", l)):
            return name, lines[start:i]
    raise SystemExit(f"kernel containing {needle!r} not found")


def blocks(body):
    out = OrderedDict()
    cur = "entry"
    out[cur] = []
    for l in body[1:]:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            m = re.match(r"^(\.LBB\S+):", s)
            if m:
                cur = m.group(1)
                out[cur] = []
            continue
        out[cur].append(s.split(";")[0].strip())
    return out


def classify(ins):
    op = ins.split()[0]
    for name, rx in CATS:
        if rx.match(op):
            return name
    return "other"


def main():
    path, needle = sys.argv[1], sys.argv[2]
    md = "--md" in sys.argv
    name, body = kernel_lines(path, needle)
    bl = blocks(body)
    order = list(bl)
    total = Counter()
    print(f"# {name}\n")
    hdr = ["block", "n", "latch"] + [c for c, _ in CATS]
    if md:
        print("| " + " | ".join(hdr) + " |")
        print("|" + "---|" * len(hdr))
    for b, ins in bl.items():
        c = Counter(classify(i) for i in ins)
        total.update(c)
        latch = ""
        for i in ins:
            m = re.match(r"s_c?branch\S*\s+(\.LBB\S+)", i)
            if m and m.group(1) in bl and order.index(m.group(1)) <= order.index(b):
                latch = "<-" + m.group(1)
        waits = [i for i in ins if i.startswith("s_waitcnt")]
        row = [b, str(len(ins)), latch] + [str(c.get(k, 0)) for k, _ in CATS]
        if md:
            print("| " + " | ".join(row) + " |")
        else:
            print(" ".join(f"{h}={v}" for h, v in zip(hdr, row) if v not in ("0", "")))
            if c.get("mfma"):
                print("   waits:", "; ".join(w.replace("s_waitcnt ", "") for w in waits))
    print("\ntotal:", dict(total))


if __name__ == "__main__":
    main()
