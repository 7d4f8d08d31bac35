#!/bin/bash
# SQ counters of the training kernels (one rocprofv3 --pmc pass per counter group, no
# tracing): issue-stall / wait / active split, MFMA busy cycles, LDS bank conflicts.
# Usage on the GPU box: bash tools/pmc_kernels.sh REGEX  -> gpurun_out/pmc_k*/ CSVs
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out
REGEX="${1:-conv1_fwd_kernel}"
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-train-ff ${PMC_BENCH_ARGS:---no-train-ref} --train-steps 1 --train-warmup 0"
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU"; do
  i=$((i + 1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" --output-format csv \
      -d $OUT/pmc_k$i -o run -- python3 $ROOT/bench.py --no-c5 $ARGS > $OUT/pmc_k$i.log 2>&1) || exit $?
  echo "pass $i done"
done
