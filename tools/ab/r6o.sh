#!/bin/bash
# aux_backward2_kernel with the next item's dP prefetched into registers (default) against the
# staging-time loads (VN_AUXB_NOPF), 174² and C5 legs, after the aux parity tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 400 python -u -m pytest tests/test_aux_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6o.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6o.log; [ $rc -eq 0 ] || exit $rc
L="--no-train-ff --no-train-84 --no-train-ref4 --no-short"
FLAG=VN_AUXB_NOPF PAT="aux_backward2" REPS=2 LEG_ARGS="$L" bash tools/ab/kflag_ab.sh || exit 1
FLAG=VN_AUXB_NOPF PAT="aux_backward2" REPS=1 BASE_ARGS="" LEG_ARGS="$L --no-train-174" bash tools/ab/kflag_ab.sh || exit 1
