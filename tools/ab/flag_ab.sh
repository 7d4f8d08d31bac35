#!/bin/bash
# A/B of an environment switch read by the library (FLAG, e.g. VN_LSTM_WG_TRANSPOSED) on one
# box (BENCH_BASE=" " keeps the C5 leg in): rocprofv3 kernel traces of the training bench legs (LEG_ARGS) without and with FLAG=1,
# alternating twice; prints each run's ms per update and the kernel time of every update.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in off on; do
    d=$ROOT/gpurun_out/fab_${v}_$rep
    if [ $v = on ]; then export $FLAG=1; else unset $FLAG; fi
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o run \
       -- python3 $ROOT/bench.py ${BENCH_BASE:---no-c5} --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 2 \
       --train-warmup 1 ${LEG_ARGS:---no-train-ff --no-train-ref4} > $d.log 2>&1) || exit 1
    echo "$FLAG=$v rep $rep: $(grep -o '"ms_per_update": [0-9.]*' $d.log | tr '\n' ' ')"
    python3 - $d/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ups, cur = [], []
for r in rows:
    cur.append(r)
    if "rmsprop" in r["Kernel_Name"]:
        ups.append(cur)
        cur = []
print("   kernel ms per update:", " ".join("%.2f" % (sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in u) / 1e6) for u in ups))
PY
  done
done
unset $FLAG
