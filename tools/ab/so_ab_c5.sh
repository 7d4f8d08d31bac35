#!/bin/bash
# so_ab.sh for the 300x400 (C5) training leg: rocprofv3 kernel stats with the in-tree
# libvnav.so ("new") and tools/ab/$ALTS ("alt"), alternating twice; prints ms per update and
# the average duration of the kernels matching KREGEX.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
ALTS=${ALTS:-libvnav_b.so}
cp $L /tmp/new.so
for rep in 1 2; do
  for v in new $ALTS; do
    if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/$v $L; fi
    d=$ROOT/gpurun_out/sab5_${v}_$rep
    (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run \
       -- python3 $ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 3 --train-warmup 1 \
       --no-train-ff --no-train-84 --no-train-ref --no-short > $d.log 2>&1) || { cp /tmp/new.so $L; exit 1; }
    echo "$v rep $rep: $(grep -o '"ms_per_update": [0-9.]*' $d.log | tr '\n' ' ')"
    grep -E "${KREGEX:-conv2_fwd}" $d/run_kernel_stats.csv | awk -F'",' '{split($2,a,","); printf "   %-70s %s calls avg %.1f us\n", substr($1,1,70), a[1], a[3]/1000}'
  done
done
cp /tmp/new.so $L
