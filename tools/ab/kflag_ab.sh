#!/bin/bash
# Same-box A/B of an environment switch (FLAG) read by the library, per kernel: rocprofv3
# kernel stats of the bench's training legs (LEG_ARGS) with FLAG unset and FLAG=1, alternating
# REPS times (default 2); prints each run's ms per update and the average duration of every
# kernel whose name matches PAT (grep -E). BASE_ARGS (default --no-c5; set it empty for the
# C5 leg) precedes LEG_ARGS.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
PAT=${PAT:-conv1}
for rep in $(seq 1 ${REPS:-2}); do
  for v in off on; do
    d=$ROOT/gpurun_out/kf_${v}_$rep
    if [ $v = on ]; then export $FLAG=1; else unset $FLAG; fi
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
       -- python3 $ROOT/bench.py ${BASE_ARGS---no-c5} --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 3 \
       --train-warmup 1 ${LEG_ARGS:---no-train-ff --no-train-ref4 --no-short} > $d.log 2>&1) || exit 1
    echo "$FLAG=$v rep $rep: $(grep -o '"ms_per_update": [0-9.]*' $d.log | tr '\n' ' ')"
    python3 - $d/run_kernel_stats.csv "$PAT" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r["Name"]):
        print("   %9.1f us x %5d  %s" % (float(r["AverageNs"]) / 1e3, int(r["Calls"]), r["Name"][:100]))
PY
    rm -f $d/run_kernel_trace.csv
  done
done
unset $FLAG
