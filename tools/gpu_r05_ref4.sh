#!/bin/bash
# Round 5: the small-batch kernel's parity test, the 4-env leg breakdown, then the logged-run
# replay on the thor-cached-auxiliary trainer as registered (tools/replicate_log.py --experiment).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_dgrad_gpu.py tests/test_trainer_gpu.py tests/test_prod_oracle_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ref4.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_ref4.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_ref4.sh > /dev/null || exit 1
head -12 gpurun_out/breakdown_ref4.txt
if [ "${REPLAY:-1}" = "1" ]; then
  timeout -k 10 900 python -u tools/replicate_log.py ${UPDATES:-12500} gpurun_out/replicate_log_curve.csv --experiment > gpurun_out/replicate_log.log 2>&1
  rc=$?; tail -3 gpurun_out/replicate_log.log; exit $rc
fi
