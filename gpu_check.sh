#!/bin/bash
# GPU-box run: parity tests, smoke, bench, rocprof kernel trace. Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != "1" ]; then
echo "== pytest -m gpu" && timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke" && timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== bench" && timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?; tail -3 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
if [ "${SKIP_PROF:-0}" != "1" ]; then
echo "== rocprofv3" && ROOT=$PWD && (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT/prof -o run --output-format csv -- python3 $ROOT/bench.py --no-c5 --steps 100 --warmup 10 --no-cpu-baseline --no-pmc --train-steps 3 --train-warmup 1 > $ROOT/$OUT/bench_prof.log 2>&1); rc=$?; tail -2 $OUT/bench_prof.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
