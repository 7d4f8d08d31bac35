#!/bin/bash
# Iteration check for the 174x174 training kernels: the ring / generic conv2 forward parity
# tests, the production-size oracle tests, the conv2 forward A/B, and a rocprofv3 kernel
# summary of the bench's 174x174 LSTM + aux leg (2 timed updates). TAG names the outputs.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
R=$PWD
TAG=${TAG:-it}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_dgrad_gpu.py tests/test_prod_oracle_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1; rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab/conv2f_ab.py 4096 10 > gpurun_out/ab_$TAG.log 2>&1; rc=$?; tail -1 gpurun_out/ab_$TAG.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/p174_$TAG -o run --output-format csv -- python3 $R/bench.py --no-c5 --steps 10 --warmup 2 --no-cpu-baseline --no-pmc ${LEG_ARGS:---no-train-ff --no-train-84 --no-train-ref4} --train-steps 2 > $R/gpurun_out/p174_$TAG.log 2>&1; rc=$?; [ $rc -eq 0 ] || exit $rc
cd $R && python3 tools/kstats.py gpurun_out/p174_$TAG/run_kernel_stats.csv 2>/dev/null | head -30 || head -25 gpurun_out/p174_$TAG/run_kernel_stats.csv | cut -c1-160
grep -o '"train_174_lstm_aux": {[^}]*}' gpurun_out/p174_$TAG.log | grep -o '"ms_per_update": [0-9.]*'
