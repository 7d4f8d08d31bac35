#!/bin/bash
# Kernel trace of the 84x84 LSTM and 174x174 LSTM+aux training legs (bench.py), then the
# per-update breakdown (tools/update_breakdown.py) of one update of each leg.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
TAG=${TAG:-upd}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o run \
  -- python3 $ROOT/bench.py --no-c5 --steps 20 --warmup 2 --no-cpu-baseline --no-pmc --no-train-ff --no-train-ref4 \
  --train-steps 2 --train-warmup 1 ${EXTRA:-} > $ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 1
cd $ROOT && TR=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | sort | tail -1) && \
  python3 tools/update_breakdown.py $TR 3,6 45 > gpurun_out/breakdown_$TAG.txt || exit 1
tail -1 gpurun_out/prof_$TAG.log | cut -c1-400
