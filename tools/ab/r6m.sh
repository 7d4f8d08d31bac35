#!/bin/bash
# conv3's forward: the per-slot-offset gather (default) against the generic one
# (VN_CONV3F_GATHER) and 256-row tiles (default) against 128 (VN_CONV3F_T128), 174² and C5 legs,
# after the conv3 / goal-run parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_goal_runs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6m.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6m.log; [ $rc -eq 0 ] || exit $rc
L="--no-train-ff --no-train-84 --no-train-ref4 --no-short"
for F in VN_CONV3F_GATHER VN_CONV3F_T128; do
  FLAG=$F PAT="NhwcIm2col.*EpiBiasAct" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
done
for F in VN_CONV3F_GATHER VN_CONV3F_T128; do
  FLAG=$F PAT="NhwcIm2col.*EpiBiasAct" REPS=1 BASE_ARGS="" LEG_ARGS="$L --no-train-174" bash tools/ab/kflag_ab.sh || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_prod_oracle_gpu.py tests/test_policy_gpu.py tests/test_aux_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6m2.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6m2.log; exit $rc
