#!/bin/bash
# Kernel trace of one bench training leg (LEG_ARGS selects it; default the 84x84 LSTM leg) and
# the per-update breakdown of update PICK (tools/update_breakdown.py). TAG names the outputs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
TAG=${TAG:-leg}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o run \
  -- python3 $ROOT/bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps ${UPDATES:-3} --train-warmup 1 \
  ${LEG_ARGS:---no-train-ff --no-train-ref --no-train-ref4} > $ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 1
cd $ROOT && TR=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | sort | tail -1) && \
  python3 tools/update_breakdown.py $TR ${PICK:-3} ${TOPK:-45} > gpurun_out/breakdown_$TAG.txt || exit 1
grep -o '"ms_per_update": [0-9.]*' gpurun_out/prof_$TAG.log
head -${TOPK:-45} gpurun_out/breakdown_$TAG.txt
