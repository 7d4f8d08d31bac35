#!/usr/bin/env python3
"""Print the top kernels of a rocprofv3 --stats kernel summary (CSV)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:n]:
    print("%9.2f ms %6d %9.1f us %5.1f%%  %s" % (float(r["TotalDurationNs"]) / 1e6, int(r["Calls"]),
                                              float(r["AverageNs"]) / 1e3, float(r["Percentage"]), r["Name"][:120]))
print("total %.2f ms" % (tot / 1e6))
