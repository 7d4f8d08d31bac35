#!/bin/bash
# Round-4 closing measurements: the goal-run tests (wide cases included), kernel traces +
# roofline tables of the 84x84 / 174x174 / 4-env legs (tools/roofline_legs.sh) and of the C5
# leg, then the C5 leg's PMC table (tools/pmc_leg.sh).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
T=${TAG:-r04f}
if [ "${SKIP_LEGS:-0}" != "1" ]; then
  timeout -k 10 400 python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_goal_runs_gpu.py \
    > gpurun_out/pytest_goalruns_$T.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_goalruns_$T.log; [ $rc -eq 0 ] || exit $rc
  TAG=$T bash tools/roofline_legs.sh > gpurun_out/roofline_legs_$T.log 2>&1 || exit $?
  echo "== legs done"
else
  bash tools/prof_ref4.sh > /dev/null || exit 1
  cp gpurun_out/breakdown_ref4.txt gpurun_out/breakdown_ref4_$T.txt
  echo "== ref4 done"
fi
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/prof_c5$T -o run \
  -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc --no-train-84 --no-train-ff --no-train-ref \
  --train-steps 3 > $ROOT/gpurun_out/prof_c5$T.log 2>&1) || exit $?
TR=$(find gpurun_out/prof_c5$T -name '*kernel_trace.csv' | sort | tail -1)
python3 tools/kernel_roofline.py $TR 2 300 400 512 20 0.05 0.05 > gpurun_out/kernel_roofline_c5_$T.md || exit 1
echo "== c5 done"
LEG=c5 TAG=c5$T bash tools/pmc_leg.sh > gpurun_out/pmc_c5_$T.log 2>&1 || exit $?
echo "== done"
