#!/usr/bin/env python3
"""Per-kernel averages (per dispatch) of the counters in gpurun_out/pmcs_k*/ (tools/pmc_sets.sh),
one row per kernel name (truncated), one column per counter.
Usage: python tools/pmc_kernel_table.py [gpurun_out] [name-width]"""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
width = int(sys.argv[2]) if len(sys.argv) > 2 else 70
vals = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(lambda: collections.defaultdict(set))
for f in glob.glob(root + "/pmcs_k*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k, c = r["Kernel_Name"][:width], r["Counter_Name"]
        vals[k][c] += float(r["Counter_Value"])
        disp[k][c].add(r["Dispatch_Id"])
counters = sorted({c for k in vals for c in vals[k]})
print("kernel".ljust(width), *[c[:14].rjust(14) for c in counters])
for k in sorted(vals):
    row = [vals[k][c] / max(1, len(disp[k][c])) if c in vals[k] else float("nan") for c in counters]
    print(k.ljust(width), *["%14.4g" % v for v in row])
