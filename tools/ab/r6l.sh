#!/bin/bash
# conv3's forward (256-row tiles now the default): the per-slot-offset gather against the generic
# one (VN_CONV3F_GATHER), the pre-split weights against the in-kernel split (VN_CONV3F_NOPRESPLIT),
# same box, 174² leg; then the conv3 / goal-run / policy parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_goal_runs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6l.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6l.log; [ $rc -eq 0 ] || exit $rc
L="--no-train-ff --no-train-84 --no-train-ref4 --no-short"
for F in VN_CONV3F_GATHER VN_CONV3F_NOPRESPLIT VN_CONV3F_T128; do
  FLAG=$F PAT="NhwcIm2col.*EpiBiasAct|split3" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_prod_oracle_gpu.py tests/test_policy_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6l2.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6l2.log; exit $rc
