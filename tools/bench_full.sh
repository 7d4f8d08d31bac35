#!/bin/bash
# The default bench line (all legs) and the rocprofv3 kernel summary of the same command.
# Usage on the GPU box: bash tools/bench_full.sh TAG -> gpurun_out/bench_TAG.log,
# gpurun_out/prof_TAG/run_kernel_stats.csv
set -o pipefail
ROOT=$GRAFT_REPO_ROOT
TAG=${1:?tag}
export TMPDIR=/tmp
cd $ROOT && timeout -k 10 500 python3 bench.py --no-c5 > gpurun_out/bench_$TAG.log 2>&1 || exit $?
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o run \
  -- python3 $ROOT/bench.py --no-c5 --no-pmc --no-cpu-baseline > $ROOT/gpurun_out/prof_$TAG.log 2>&1
