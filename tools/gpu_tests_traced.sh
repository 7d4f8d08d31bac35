#!/bin/bash
# GPU box: (1) the tests named in NEW (verbose, all run), (2) the whole -m gpu suite under a
# rocprofv3 kernel trace with per-test markers, split per test by tools/test_kernel_map.py.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
OUT=gpurun_out
TAG=${TAG:-r03}
mkdir -p $OUT
if [ -n "${NEW:-}" ]; then
  timeout -k 10 500 python -u -m pytest $NEW -m gpu -v -s --timeout 240 --timeout-method thread > $OUT/pytest_new_$TAG.log 2>&1
  rc=$?; tail -15 $OUT/pytest_new_$TAG.log
  # test failures (1) go on to the traced suite; a crash / timeout stops here
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ "${TRACE:-1}" = "1" ]; then
  rm -f $OUT/tests_$TAG.tsv
  (cd /tmp && VN_TRACE_TESTS=$ROOT/$OUT/tests_$TAG.tsv timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv \
     -d /tmp/trace_$TAG -o run -- python3 -u -m pytest $ROOT/tests -m gpu -q --timeout 240 --timeout-method thread \
     -p no:cacheprovider > $ROOT/$OUT/pytest_gpu_traced_$TAG.log 2>&1)
  rc=$?; tail -5 $OUT/pytest_gpu_traced_$TAG.log
  f=$(find /tmp/trace_$TAG -name "*kernel_trace.csv" | head -1)
  if [ -n "$f" ]; then
    # (profiles/ does not travel to the box: without a TOP file the map lists kernels per test only;
    # the top-kernel coverage table is built here from the returned trace)
    TOPARG=""; [ -n "${TOP:-}" ] && [ -f "$TOP" ] && TOPARG="--top $TOP"
    python3 tools/test_kernel_map.py "$f" $OUT/tests_$TAG.tsv $TOPARG --k 20 \
      --oracle-tests ${ORACLE_TESTS:-test_prod_oracle_gpu vs_fp64_oracle vs_oracle} --md $OUT/test_kernels_$TAG.md; echo "map rc=$?"
    gzip -c "$f" > $OUT/kernel_trace_tests_$TAG.csv.gz
  fi
  [ $rc -eq 0 ] || exit $rc
fi
echo "== done"
