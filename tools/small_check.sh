#!/bin/bash
# Small-batch iteration: the A/B parity tests, the trainer tests, then the 4-env breakdown.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_parity_dgrad_gpu.py tests/test_trainer_gpu.py tests/test_prod_oracle_gpu.py tests/test_lstm_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_small.log 2>&1; rc=$?; tail -3 gpurun_out/t_small.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_ref4.sh | head -22
