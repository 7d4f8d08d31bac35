#!/bin/bash
# rocprofv3 --pmc passes (one per ';'-separated counter set, no tracing) for the kernels
# matching REGEX over an arbitrary python command (e.g. tools/ab/conv2f_ab.py). Usage on the
# GPU box: PMC_SETS="A B;C D" bash tools/pmc_cmd.sh REGEX script.py [args]
#   -> gpurun_out/pmcs_k*/ CSVs; summary: python tools/pmc_sets_summary.py
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out
REGEX="${1:?kernel regex}"
shift
SCRIPT="$ROOT/$1"
shift
IFS=';' read -ra SETS <<< "${PMC_SETS:?counter sets}"
i=0
for SET in "${SETS[@]}"; do
  i=$((i + 1))
  rm -rf $OUT/pmcs_k$i
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex "$REGEX" --output-format csv \
      -d $OUT/pmcs_k$i -o run -- python3 $SCRIPT "$@" > $OUT/pmcs_k$i.log 2>&1) || exit $?
  echo "pass $i done: $SET"
done
python3 $ROOT/tools/pmc_sets_summary.py $OUT
