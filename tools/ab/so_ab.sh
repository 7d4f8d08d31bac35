#!/bin/bash
# Per-kernel A/B of two library builds on one box: rocprofv3 kernel stats of the training
# bench legs (LEG_ARGS) with the in-tree libvnav.so ("new") and with tools/ab/$ALT ("alt").
# Prints the average duration of the kernels matching KREGEX for both.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
ALTS=${ALTS:-libvnav_b.so}
cp $L /tmp/new.so
for v in new $ALTS; do
  if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/$v $L; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/sab_$v -o run \
     -- python3 $ROOT/bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 2 --train-warmup 1 ${LEG_ARGS:---no-train-ff --no-train-ref4} > $ROOT/gpurun_out/sab_$v.log 2>&1) || { cp /tmp/new.so $L; exit 1; }
  echo "$v: $(grep -o '"ms_per_update": [0-9.]*' gpurun_out/sab_$v.log | tr '\n' ' ')"
  grep -E "${KREGEX:-conv1_wgrad}" gpurun_out/sab_$v/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-70s %s calls avg %.1f us\n", substr($1,1,70), a[1], a[3]/1000}'
done
cp /tmp/new.so $L
