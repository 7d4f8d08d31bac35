#!/bin/bash
# A/B of conv_merge's input-gradient product tiles (64x64 default vs 128x128, VN_CM_DGRAD_128):
# the 84 / 174 / C5 legs, interleaved twice; parity tests under the switch first. The switch existed
# for this run only (128x128 kept for FCIN >= 1024; profiles/r05/ab_cm/).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
OUT=gpurun_out/ab_cm
mkdir -p $OUT
VN_CM_DGRAD_128=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_policy_gpu.py tests/test_aux_gpu.py > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-train-ff --no-train-ref4 --no-short"
for rep in 1 2; do
  for cfg in 64 128; do
    if [ $cfg = 128 ]; then E="VN_CM_DGRAD_128=1"; else E=""; fi
    env $E timeout -k 10 400 python bench.py $ARGS > $OUT/bench_$cfg.$rep.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$cfg.$rep.log') if l.startswith('{')][-1])
print('tile=$cfg', {k: round(v['ms_per_update'], 2) for k, v in d.items() if isinstance(v, dict) and 'ms_per_update' in v})"
  done
done
