#!/bin/bash
# Round-4 check of the banded conv3 weight gradient at 300x400: parity tests, then a kernel trace
# of the C5 bench leg.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -q --timeout 240 --timeout-method thread tests/test_parity_dgrad_gpu.py \
  tests/test_goal_runs_gpu.py tests/test_prod_oracle_gpu.py tests/test_aux_gpu.py > gpurun_out/pytest_c5wg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_c5wg.log; [ $rc -eq 0 ] || exit $rc
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_c5wg -o run \
  -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff --no-train-ref \
  --train-steps 3 > $ROOT/gpurun_out/prof_c5wg.log 2>&1) || exit $?
grep -o '"train_c5_300x400": {[^}]*' gpurun_out/prof_c5wg.log | head -c 400; echo
