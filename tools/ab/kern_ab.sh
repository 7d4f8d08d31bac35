#!/bin/bash
# Per-kernel A/B: rocprofv3 kernel stats of the training bench with the in-tree library and
# with tools/ab/libvnav_head.so on the same box; tools/ab/kern_diff.py compares them.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
cp $L /tmp/new.so
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-pmc ${KAB_ARGS:---no-train-ref}"
for v in new head; do
  if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/libvnav_head.so $L; fi
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/kab_$v -o run \
     -- python3 $ROOT/bench.py --no-c5 $ARGS > $ROOT/gpurun_out/kab_$v.log 2>&1) || exit 1
done
cp /tmp/new.so $L
python3 tools/ab/kern_diff.py gpurun_out/kab_head/run_kernel_stats.csv gpurun_out/kab_new/run_kernel_stats.csv
