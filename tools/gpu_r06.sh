#!/bin/bash
# Round-6 GPU run: (1) the tests named in NEW (verbose), (2) the whole -m gpu suite and smoke
# unless SKIP_TESTS=1, (3) the default bench unless SKIP_BENCH=1 (BENCH_ARGS), (4) a rocprofv3
# kernel trace of the bench with LEG_ARGS when set. Each step has its own limit; the chain
# stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r06}
mkdir -p $OUT
if [ -n "${NEW:-}" ]; then
  echo "== pytest $NEW"
  timeout -k 10 600 python -u -m pytest $NEW -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_new_$TAG.log 2>&1
  rc=$?; tail -15 $OUT/pytest_new_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "== pytest -m gpu tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1
  rc=$?; tail -4 $OUT/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
  echo "== smoke"
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  echo "== bench ${BENCH_ARGS:-}"
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench_$TAG.log 2>&1
  rc=$?; tail -1 $OUT/bench_$TAG.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${LEG_ARGS:-}" ]; then
  echo "== rocprofv3 $LEG_ARGS"
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/$OUT/prof_$TAG -o run \
    -- python3 $ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pmc $LEG_ARGS > $ROOT/$OUT/prof_$TAG.log 2>&1
  rc=$?; cd $ROOT; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
