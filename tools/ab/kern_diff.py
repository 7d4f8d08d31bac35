"""Compare two rocprofv3 kernel_stats CSVs (head, new): total time per kernel, biggest first."""
import csv
import re
import sys


def load(p):
    out = {}
    for r in csv.DictReader(open(p)):
        n = re.sub(r"\(.*$", "", r["Name"]).replace("void ", "").replace("vn::", "")
        out[n] = (int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6)
    return out


h, n = load(sys.argv[1]), load(sys.argv[2])
keys = sorted(set(h) | set(n), key=lambda k: -max(h.get(k, (0, 0))[1], n.get(k, (0, 0))[1]))
th = sum(v[1] for v in h.values())
tn = sum(v[1] for v in n.values())
print("total head %.2f ms  new %.2f ms  (%.1f%%)" % (th, tn, 100 * (tn / th - 1)))
for k in keys[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    ch, th_ = h.get(k, (0, 0.0))
    cn, tn_ = n.get(k, (0, 0.0))
    d = 100 * (tn_ / th_ - 1) if th_ else float("nan")
    print("%9.3f %9.3f %+6.1f%%  %5d %s" % (th_, tn_, d, cn, k[:110]))
