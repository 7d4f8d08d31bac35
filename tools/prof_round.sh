#!/bin/bash
# Round profile: full bench line, then rocprofv3 --kernel-trace --stats summaries of the
# env-only bench (same vn_step command as the bench's env leg) and of the training legs.
# TAG names the outputs under gpurun_out/.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=$ROOT/gpurun_out
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python3 bench.py --no-c5 ${BENCH_ARGS:-} > $OUT/bench_$TAG.log 2>&1
rc=$?; tail -1 $OUT/bench_$TAG.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_env_$TAG -o run \
  -- python3 $ROOT/bench.py --no-c5 --train-steps 0 --no-pmc --no-cpu-baseline > $OUT/prof_env_$TAG.log 2>&1
rc=$?; [ $rc -eq 0 ] || exit $rc
if [ "${TRAIN_PROF:-1}" = "1" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_train_$TAG -o run \
    -- python3 $ROOT/bench.py --no-c5 --steps 10 --warmup 2 --no-pmc --no-cpu-baseline ${TRAIN_ARGS:-} > $OUT/prof_train_$TAG.log 2>&1
  rc=$?; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
