#!/bin/bash
# conv3's forward with its weights pre-split once per call (default) against the split in every
# workgroup (VN_CONV3F_NOPRESPLIT), both on the per-slot-offset gather; 174² and C5 legs, after
# the conv3 / goal-run parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_goal_runs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6q.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6q.log; [ $rc -eq 0 ] || exit $rc
L="--no-train-ff --no-train-84 --no-train-ref4 --no-short"
P="NhwcIm2col.*EpiBiasAct|split3"
FLAG=VN_CONV3F_NOPRESPLIT PAT="$P" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
FLAG=VN_CONV3F_NOPRESPLIT PAT="$P" REPS=1 BASE_ARGS="" LEG_ARGS="$L --no-train-174" bash tools/ab/kflag_ab.sh || exit 1
