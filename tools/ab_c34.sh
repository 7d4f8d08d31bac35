#!/bin/bash
# A/B of conv34_small_kernel's pixels per workgroup (VN_C34_ROWS = 2 / 4 / 8) at the logged
# run's 4-env batch: the small-kernel parity test under each, then the ref4 leg, interleaved twice.
# The VN_C34_ROWS switch existed for these runs only (2 kept as kC34Rows; profiles/r05/ab_c34/).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
OUT=gpurun_out/ab_c34
mkdir -p $OUT
for r in ${PRS:-2 8}; do
  VN_C34_ROWS=$r timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_parity_dgrad_gpu.py::test_conv34_small_matches_generic_products \
    tests/test_prod_oracle_gpu.py::test_logged_run_shape_trainer_update_vs_fp64_oracle > $OUT/pytest_$r.log 2>&1 \
    || { tail -20 $OUT/pytest_$r.log; exit 1; }
  tail -1 $OUT/pytest_$r.log
done
ARGS="--no-cpu-baseline --no-pmc --no-train-ff --no-train-84 --no-train-174 --no-c5 --no-short"
for rep in 1 2; do
  for r in ${BRS:-4 2 8}; do
    VN_C34_ROWS=$r timeout -k 10 300 python bench.py $ARGS > $OUT/bench_$r.$rep.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$r.$rep.log') if l.startswith('{')][-1])
r=d['train_174_lstm_aux_4env']
print('rows=$r', round(r['ms_per_update'], 4), 'eager', round(r['eager_ms_per_update'], 4))"
  done
done
