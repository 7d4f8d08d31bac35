#!/bin/bash
# Iteration run on the GPU box: selected GPU tests (TESTS), then a bench with BENCH_ARGS and
# the rocprofv3 kernel summary of the same bench command (TAG names the outputs).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
TAG=${TAG:-iter}
OUT=gpurun_out
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 300 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 400 python3 bench.py --no-c5 $BENCH_ARGS > $OUT/bench_$TAG.log 2>&1
  rc=$?; tail -1 $OUT/bench_$TAG.log | cut -c1-3000; [ $rc -eq 0 ] || exit $rc
  if [ "${PROF:-1}" = "1" ]; then
    cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_$TAG -o run \
      -- python3 $ROOT/bench.py --no-c5 $BENCH_ARGS > $ROOT/$OUT/prof_$TAG.log 2>&1
    rc=$?; [ $rc -eq 0 ] || exit $rc
  fi
fi
echo "== done"
