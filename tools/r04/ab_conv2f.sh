#!/bin/bash
# A/B of C5's conv2 forward: the banded x6 kernel (the default since this A/B; it ran under a
# VN_CONV2F_BAND switch then) vs the generic product (VN_CONV2F_GENERIC), with the C5 parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 240 --timeout-method thread \
  "tests/test_goal_runs_gpu.py" "tests/test_prod_oracle_gpu.py" -k "c5 or 300" > gpurun_out/pytest_ab_conv2f.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ab_conv2f.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  if [ $v = 0 ]; then export VN_CONV2F_GENERIC=1; else unset VN_CONV2F_GENERIC; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff \
    --no-train-ref --train-steps 3 > gpurun_out/ab_conv2f_$v.log 2>&1 || exit $?
  echo "band=$v $(grep -o '"train_c5_300x400": {[^}]*' gpurun_out/ab_conv2f_$v.log | grep -o '"ms_per_update": [0-9.]*')"
done
