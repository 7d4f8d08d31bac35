#!/bin/bash
# Kernel trace of the C5 bench leg (the top-20 list for the per-test kernel map) and its roofline.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
T=${TAG:-r04g}
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_c5$T -o run \
  -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff --no-train-ref \
  --train-steps 3 > $ROOT/gpurun_out/prof_c5$T.log 2>&1) || exit $?
TR=$(find gpurun_out/prof_c5$T -name '*kernel_trace.csv' | sort | tail -1)
python3 tools/kernel_roofline.py $TR 2 300 400 512 20 0.05 0.05 > gpurun_out/kernel_roofline_c5_$T.md || exit 1
head -3 gpurun_out/kernel_roofline_c5_$T.md
