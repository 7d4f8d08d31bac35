#!/bin/bash
# conv3's forward: the gather with per-slot offsets kept across the K loop (default) against the
# generic gather (VN_CONV3F_GATHER), and 256 x 64 tiles (VN_CONV3F_T256), same box, 174² leg;
# then the conv3 parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
L="--no-train-ff --no-train-84 --no-train-ref4 --no-short"
FLAG=VN_CONV3F_GATHER PAT="NhwcIm2colGoal.*EpiBiasAct" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
FLAG=VN_CONV3F_T256 PAT="NhwcIm2colGoal.*EpiBiasAct" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
timeout -k 10 400 python -u -m pytest tests/test_prod_oracle_gpu.py tests/test_policy_gpu.py tests/test_goal_runs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6k.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6k.log; exit $rc
