"""Split a rocprofv3 kernel trace of a GPU test run per test, and check which kernels each
test dispatched.

    VN_TRACE_TESTS=gpurun_out/tests.tsv rocprofv3 --kernel-trace --output-format csv -d D -o run \
        -- python3 -m pytest tests -m gpu ...
    python tools/test_kernel_map.py D/run_kernel_trace.csv gpurun_out/tests.tsv \
        [--top profiles/r02/train_kernel_stats_v12.csv --k 20 --oracle-tests PATTERN ...] [--md out.md]

tests/conftest.py launches ``vn_trace_marker(k)`` (an empty kernel of k workgroups of 64
lanes) before test k; every kernel dispatched after marker k and before marker k+1 belongs
to test k. ``--top`` lists the K most expensive kernels of a bench trace summary and, for
each, the tests matching ``--oracle-tests`` (substrings of the node id) that dispatched it.
"""
import argparse
import csv
import re
import sys
from collections import Counter, defaultdict

MARKER = "trace_marker_kernel"


def short(name):
    """Kernel name without the argument list (template arguments kept)."""
    name = re.sub(r"^void ", "", name)
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def load_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                         int(r["Workgroup_Size_X"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    return rows


def split(rows, tests):
    per = defaultdict(Counter)
    cur = None
    for _, name, grid, wg, _ in rows:
        if MARKER in name:
            cur = grid // max(wg, 1)
            continue
        if cur is not None:
            per[cur][short(name)] += 1
    return {tests.get(k, "test#%d" % k): c for k, c in per.items()}


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("trace")
    p.add_argument("tests")
    p.add_argument("--top", default=None, help="kernel_stats.csv of a bench trace")
    p.add_argument("--k", type=int, default=20)
    p.add_argument("--oracle-tests", nargs="*", default=[],
                   help="substrings of the node ids of the tests that compare with the oracle directly")
    p.add_argument("--md", default=None)
    a = p.parse_args(argv)
    tests = {}
    with open(a.tests) as f:
        for line in f:
            k, nodeid = line.rstrip("\n").split("\t", 1)
            i = nodeid.find("tests/")
            tests[int(k)] = nodeid[i:] if i >= 0 else nodeid
    per = split(load_trace(a.trace), tests)
    out = ["# Kernels dispatched per GPU test", "",
           "From `%s` split at the `vn_trace_marker` launches (`tests/conftest.py`)." % a.trace, ""]
    for nodeid in [tests[k] for k in sorted(tests)]:
        c = per.get(nodeid, Counter())
        vn = sorted((n, m) for n, m in c.items() if n.startswith("vn::"))
        out.append("## %s" % nodeid)
        out.append("")
        out.append("%d vnav kernels (%d launches), %d other" % (
            len(vn), sum(m for _, m in vn), sum(m for n, m in c.items() if not n.startswith("vn::"))))
        out.append("")
        for n, m in vn:
            out.append("* `%s` x%d" % (n, m))
        out.append("")
    missing = []
    if a.top:
        with open(a.top) as f:
            top = [short(r["Name"]) for r in csv.DictReader(f)][:a.k]
        out += ["# Top %d kernels of `%s` and the direct-oracle tests that run them" % (a.k, a.top), "",
                "| kernel | direct-oracle tests |", "|---|---|"]
        for kname in top:
            hits = [t for t, c in per.items() if kname in c and any(s in t for s in a.oracle_tests)]
            if not hits:
                missing.append(kname)
            out.append("| `%s` | %s |" % (kname, "<br>".join("`%s`" % h.split("::", 1)[-1] for h in sorted(hits))
                                           or "**none**"))
        out.append("")
        out.append("%d of %d covered." % (len(top) - len(missing), len(top)))
    text = "\n".join(out) + "\n"
    if a.md:
        with open(a.md, "w") as f:
            f.write(text)
    else:
        sys.stdout.write(text)
    return 1 if missing else 0


if __name__ == "__main__":
    raise SystemExit(main())
