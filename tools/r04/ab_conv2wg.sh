#!/bin/bash
# C5 conv2 weight gradient: x6 bands of one dZ2 row (default) vs the f32 kernel (VN_CONV2WG_F32).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_parity_dgrad_gpu.py \
  tests/test_goal_runs_gpu.py tests/test_prod_oracle_gpu.py -k "300 or c5" > gpurun_out/pytest_ab_conv2wg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ab_conv2wg.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  if [ $v = 0 ]; then export VN_CONV2WG_F32=1; else unset VN_CONV2WG_F32; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff \
    --no-train-ref --train-steps 3 > gpurun_out/ab_conv2wg_$v.log 2>&1 || exit $?
  echo "x6=$v $(grep -o '"train_c5_300x400": {[^}]*' gpurun_out/ab_conv2wg_$v.log | grep -o '"ms_per_update": [0-9.]*')"
done
