"""Per-dispatch averages of the counters in gpurun_out/pmcs_k*/ (tools/pmc_sets.sh). Usage: python tools/pmc_sets_summary.py [gpurun_out]."""
import collections
import csv
import glob
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(root + "/pmcs_k*/")):
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        rows = list(csv.DictReader(open(f)))
        agg = collections.defaultdict(float)
        for r in rows:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp = len({r["Dispatch_Id"] for r in rows}) or 1
        for k, v in agg.items():
            print("%-40s %.4g" % (k, v / disp))
