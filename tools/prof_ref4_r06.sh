#!/bin/bash
# Kernel trace of the 4-env (the logged run's batch) 174x174 LSTM + aux leg, then the
# per-update breakdown of one captured-graph update.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_ref4 -o run \
  -- python3 $ROOT/bench.py --no-c5 --steps 20 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff \
  --train-steps 1 --train-warmup 0 --no-short > $ROOT/gpurun_out/prof_ref4.log 2>&1 || exit 1
cd $ROOT && TR=$(find gpurun_out/prof_ref4 -name '*kernel_trace.csv' | sort | tail -1) && \
  python3 tools/update_breakdown.py $TR ${PICKS:-300,700} 40 > gpurun_out/breakdown_ref4.txt || exit 1
head -130 gpurun_out/breakdown_ref4.txt
