#!/usr/bin/env python3
"""Per-update kernel breakdown from a rocprofv3 kernel trace of bench.py: updates are cut at
each rmsprop kernel; prints the busiest kernels of the chosen updates (1-based)."""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "").replace("vn::", "")
    return n[:110]


def main(path, picks, top=25):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ups, cur = [], []
    for r in rows:
        cur.append(r)
        if "rmsprop" in r["Kernel_Name"]:
            ups.append(cur)
            cur = []
    print("updates found:", len(ups))
    for p in picks:
        u = ups[p - 1]
        # the rollout of an update starts after the previous rmsprop; drop env-only bench leftovers
        span = (int(u[-1]["End_Timestamp"]) - int(u[0]["Start_Timestamp"])) / 1e6
        agg = collections.defaultdict(lambda: [0, 0.0])
        for r in u:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            a = agg[short(r["Kernel_Name"])]
            a[0] += 1
            a[1] += d
        busy = sum(v[1] for v in agg.values())
        print("\n== update %d: %d dispatches, kernel time %.2f ms, span %.2f ms" % (p, len(u), busy, span))
        for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            print("%8.3f ms %5d  %5.1f%%  %s" % (t, c, 100 * t / busy, k))


if __name__ == "__main__":
    main(sys.argv[1], [int(x) for x in sys.argv[2].split(",")], int(sys.argv[3]) if len(sys.argv) > 3 else 25)
