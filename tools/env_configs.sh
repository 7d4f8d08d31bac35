#!/bin/bash
# vn_step at the SURVEY §8 configs on one GPU (env-only bench leg): C2 1 scene x 1024 envs,
# C3 4 scenes x 4096, C4's per-GPU shard 20 scenes x 4096, and 20 scenes x 32768 (C4's
# whole env count on one GPU).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for cfg in "1 1024" "4 4096" "20 4096" "20 32768"; do
  set -- $cfg
  timeout -k 10 200 python3 bench.py --no-c5 --train-steps 0 --no-cpu-baseline --scenes $1 --envs $2 --steps 1000 --warmup 300 > gpurun_out/envcfg_$1_$2.log 2>&1 || exit 1
  echo "scenes $1 envs $2 $(grep -o '"value": [0-9.]*' gpurun_out/envcfg_$1_$2.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/envcfg_$1_$2.log) $(grep -o '"frac": [0-9.]*' gpurun_out/envcfg_$1_$2.log | head -1) $(grep -o '"traffic": [0-9.]*' gpurun_out/envcfg_$1_$2.log) $(grep -o 'MB frame cache, [A-Za-z-]*' gpurun_out/envcfg_$1_$2.log)"
done
