#!/bin/bash
# The LSTM cell fused into the gates product's epilogue (default) against the product +
# lstm_cell_kernel (VN_LSTM_CELL_UNFUSED), 84² and 174² legs, after the LSTM / oracle tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 500 python -u -m pytest tests/test_lstm_gpu.py tests/test_prod_oracle_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6u.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6u.log; [ $rc -eq 0 ] || exit $rc
FLAG=VN_LSTM_CELL_UNFUSED PAT="GateRows|EpiBias2>|lstm_cell_kernel" REPS=2 bash tools/ab/kflag_ab.sh || exit 1
