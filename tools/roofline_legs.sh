#!/bin/bash
# GPU box: kernel traces of the 84x84 LSTM and 174x174 LSTM + aux training legs, their
# per-update breakdowns (tools/prof_leg.sh) and roofline tables (tools/kernel_roofline.py),
# then the 4-env leg's breakdown (tools/prof_ref4.sh). TAG names the outputs.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
T=${TAG:-r03}
TAG=l84$T bash tools/prof_leg.sh > /dev/null || exit 1
TAG=l174$T LEG_ARGS="--no-train-ff --no-train-84 --no-train-ref4" UPDATES=2 PICK=2 bash tools/prof_leg.sh > /dev/null || exit 1
TR84=$(find gpurun_out/prof_l84$T -name '*kernel_trace.csv' | sort | tail -1)
TR174=$(find gpurun_out/prof_l174$T -name '*kernel_trace.csv' | sort | tail -1)
python3 tools/kernel_roofline.py $TR84 3 84 84 4096 20 0.05 0.05 > gpurun_out/kernel_roofline_84_lstm_$T.md || exit 1
python3 tools/kernel_roofline.py $TR174 2 174 174 4096 20 0.05 0.05 > gpurun_out/kernel_roofline_174_lstm_aux_$T.md || exit 1
bash tools/prof_ref4.sh > /dev/null || exit 1
cp gpurun_out/breakdown_ref4.txt gpurun_out/breakdown_ref4_$T.txt
head -3 gpurun_out/breakdown_l84$T.txt gpurun_out/breakdown_l174$T.txt gpurun_out/breakdown_ref4_$T.txt
cat gpurun_out/kernel_roofline_84_lstm_$T.md gpurun_out/kernel_roofline_174_lstm_aux_$T.md
