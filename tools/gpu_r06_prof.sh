#!/bin/bash
# Round-6 profiles of the final build, each step under its own limit, stopping at the first
# failure: (1) rocprofv3 kernel stats of the env-only bench (the headline kernel's average for
# the roofline cross-check), (2) kernel traces + per-update breakdowns + roofline tables of the
# 84² LSTM, 174² LSTM + aux + UNREAL and C5 legs, (3) the 4-env leg's breakdown (graph updates,
# without and with the replay sources). Outputs under gpurun_out/, TAG-suffixed.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
T=${TAG:-r06}
OUT=$ROOT/gpurun_out
echo "== env kernel stats"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_env_$T -o run \
  -- python3 $ROOT/bench.py --no-c5 --train-steps 0 --no-pmc --no-cpu-baseline > $OUT/prof_env_$T.log 2>&1) || exit 1
tail -1 $OUT/prof_env_$T.log | cut -c1-300
echo "== 84 leg"
TAG=l84$T bash tools/prof_leg.sh > /dev/null || exit 1
echo "== 174 leg"
TAG=l174$T LEG_ARGS="--no-train-ff --no-train-84 --no-train-ref4 --no-short" UPDATES=2 PICK=2 bash tools/prof_leg.sh > /dev/null || exit 1
TR84=$(find gpurun_out/prof_l84$T -name '*kernel_trace.csv' | sort | tail -1)
TR174=$(find gpurun_out/prof_l174$T -name '*kernel_trace.csv' | sort | tail -1)
python3 tools/kernel_roofline.py $TR84 3 84 84 4096 20 0.05 0.05 > gpurun_out/kernel_roofline_84_lstm_$T.md || exit 1
python3 tools/kernel_roofline.py $TR174 2 174 174 4096 20 0.05 0.05 > gpurun_out/kernel_roofline_174_$T.md || exit 1
echo "== c5 leg"
TAG=c5$T bash tools/prof_c5.sh > /dev/null || exit 1
mv gpurun_out/kernel_roofline_c5$T.md gpurun_out/kernel_roofline_c5_$T.md 2>/dev/null
echo "== 4-env leg"
bash tools/prof_ref4_r06.sh > /dev/null || exit 1
cp gpurun_out/breakdown_ref4.txt gpurun_out/breakdown_ref4_$T.txt
head -4 gpurun_out/breakdown_l84$T.txt gpurun_out/breakdown_l174$T.txt gpurun_out/breakdown_c5$T.txt gpurun_out/breakdown_ref4_$T.txt
# the traces have been reduced to the breakdowns and tables above; gpurun returns <= 64 MiB
find gpurun_out -name '*kernel_trace.csv' -delete
echo "== done"
