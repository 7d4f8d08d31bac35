#!/bin/bash
# Kernel trace of the 174x174 LSTM + aux + UNREAL training leg (4096 envs) alone, its per-update
# breakdown, roofline table and kernel stats (the --top list of tools/test_kernel_map.py).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
export TMPDIR=/tmp
TAG=${TAG:-174}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_$TAG -o run \
  -- python3 $ROOT/bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --train-steps 3 --train-warmup 1 \
  --no-train-ff --no-train-84 --no-train-ref4 --no-short > $ROOT/gpurun_out/prof_$TAG.log 2>&1 || exit 1
cd $ROOT && TR=$(find gpurun_out/prof_$TAG -name '*kernel_trace.csv' | sort | tail -1) && \
  python3 tools/update_breakdown.py $TR 2 45 > gpurun_out/breakdown_$TAG.txt && \
  python3 tools/kernel_roofline.py $TR 2 174 174 4096 20 0.05 0.05 > gpurun_out/kernel_roofline_$TAG.md || exit 1
head -20 gpurun_out/breakdown_$TAG.txt
