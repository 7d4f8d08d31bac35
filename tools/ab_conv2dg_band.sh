#!/bin/bash
# A/B of conv2's input gradient at 174x174: the whole-map kernel (default) against the banded
# kernel with BY = 8 / 14 (VN_CONV2DG_BAND): parity tests under each, then the 174 leg's
# update time, interleaved twice. The VN_CONV2DG_BAND dispatch existed for this run only (no gain,
# profiles/r05/ab_c2dg/; removed): the script records how it was measured.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
OUT=gpurun_out/ab_c2dg
mkdir -p $OUT
for by in 8 14; do
  VN_CONV2DG_BAND=$by timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_policy_gpu.py::test_autograd_policy_174_vs_torch_oracle tests/test_goal_runs_gpu.py \
    > $OUT/pytest_band$by.log 2>&1 || { tail -20 $OUT/pytest_band$by.log; exit 1; }
  tail -1 $OUT/pytest_band$by.log
done
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-train-ff --no-train-84 --no-train-ref4 --no-c5 --no-short"
for rep in 1 2; do
  for by in 0 8 14; do
    if [ $by = 0 ]; then
      timeout -k 10 300 python bench.py $ARGS > $OUT/bench_$by.$rep.log 2>&1 || exit 1
    else
      VN_CONV2DG_BAND=$by timeout -k 10 300 python bench.py $ARGS > $OUT/bench_$by.$rep.log 2>&1 || exit 1
    fi
    python3 -c "
import json,sys
d=json.loads([l for l in open('$OUT/bench_$by.$rep.log') if l.startswith('{')][-1])
print('band=$by', {k: round(v['ms_per_update'], 2) for k, v in d.items() if isinstance(v, dict) and 'ms_per_update' in v})"
  done
done
