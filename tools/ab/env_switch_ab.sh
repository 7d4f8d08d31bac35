#!/bin/bash
# Same-box A/B of one library build under an environment switch: rocprofv3 kernel stats of the
# bench's training legs (LEG_ARGS) with SWITCH unset ("on") and SWITCH=1 ("off"), alternating
# ROUNDS times. Prints ms per update and the kernels matching KREGEX for each run.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
SW=${SWITCH:?environment switch}
for r in ${ROUNDS:-1}; do
  for v in on off; do
    d=$ROOT/gpurun_out/esab_$v$r
    if [ $v = on ]; then unset $SW; else export $SW=1; fi
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
       -- python3 $ROOT/bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps ${UPDATES:-2} --train-warmup 1 \
       ${LEG_ARGS:---no-train-ff --no-train-ref4} > $d.log 2>&1) || exit 1
    echo "$v$r: $(grep -o '"ms_per_update": [0-9.]*' $d.log | tr '\n' ' ')"
    grep -E "${KREGEX:-gemm_x6}" $d/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-100s %s calls avg %.1f us tot %.2f ms\n", substr($1,2,100), a[1], a[3]/1000, a[2]/1e6}'
  done
done
unset $SW
