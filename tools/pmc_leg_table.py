#!/usr/bin/env python3
"""Per-kernel PMC table of one bench leg (tools/pmc_leg.sh): the dispatches between the two
vn_trace_marker launches (exactly one update), summed per kernel name, and the derived ratios
VALU/MFMA instructions, wait = SQ_WAIT_ANY / SQ_WAVE_CYCLES, MFMA busy =
SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), LDS bank-conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE. Usage: python tools/pmc_leg_table.py DIR"""
import collections
import csv
import glob
import re
import sys

root = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sorted(glob.glob(root + "/k*/")):
    rows = {}
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rec = rows.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})
            rec[r["Counter_Name"]] = rec.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    marks = sorted(i for i, v in rows.items() if "trace_marker" in v["name"])
    if len(marks) != 2:
        continue
    for i, v in rows.items():
        if marks[0] < i < marks[1]:
            name = re.sub(r"\(.*$", "", v["name"]).replace("void ", "").replace("vn::", "")
            for c, x in v.items():
                if c != "name":
                    per[name][c] += x
            per[name]["_disp"] += 0  # present


def ratio(a, b):
    return a / b if b else float("nan")


print("| kernel | VALU/MFMA | wait | MFMA busy | LDS conflict share |")
print("|---|---|---|---|---|")
busy = lambda v: ratio(v["SQ_VALU_MFMA_BUSY_CYCLES"], 1024 * v["GRBM_GUI_ACTIVE"] / 8)  # noqa: E731
for name, v in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0)):
    if v.get("SQ_INSTS_MFMA", 0) == 0 and v.get("SQ_INSTS_VALU", 0) < 1e6:
        continue
    print("| `%s` | %.1f | %.2f | %.2f | %.2f |" % (name[:80], ratio(v["SQ_INSTS_VALU"], v["SQ_INSTS_MFMA"]),
                                                     ratio(v["SQ_WAIT_ANY"], v["SQ_WAVE_CYCLES"]), busy(v),
                                                     ratio(v["SQ_LDS_BANK_CONFLICT"], v["SQ_LDS_IDX_ACTIVE"])))
