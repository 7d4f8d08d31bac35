#!/bin/bash
# rocprofv3 --pmc passes (one per ';'-separated counter set, no tracing) over the training
# bench for the kernels matching REGEX. Usage on the GPU box:
#   PMC_SETS="A B;C D" bash tools/pmc_sets.sh REGEX  -> gpurun_out/pmcs_k*/ CSVs; summary: tools/pmc_sets_summary.py
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out
REGEX="${1:?kernel regex}"
ARGS="--steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-train-ff ${PMC_BENCH_ARGS:---no-train-ref} --train-steps 1 --train-warmup 0"
IFS=';' read -ra SETS <<< "${PMC_SETS:?counter sets}"
i=0
for SET in "${SETS[@]}"; do
  i=$((i + 1))
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" --output-format csv \
      -d $OUT/pmcs_k$i -o run -- python3 $ROOT/bench.py --no-c5 $ARGS > $OUT/pmcs_k$i.log 2>&1) || exit $?
  echo "pass $i done: $SET"
done
