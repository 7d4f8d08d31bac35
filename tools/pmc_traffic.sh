#!/bin/bash
# HBM traffic of the vn_step kernel from rocprofv3 PMC counters, one counter per pass
# (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE (KB) per dispatch of env_kernel
# at the bench configuration. Writes gpurun_out/pmc_{fetch,write}/ CSVs; summarise with
# tools/pmc_summary.py. Run on the GPU box: bash tools/pmc_traffic.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out
mkdir -p $OUT
ARGS="--steps 30 --warmup 5 --no-cpu-baseline --train-steps 0"
for C in FETCH_SIZE WRITE_SIZE; do
  name=$(echo $C | tr 'A-Z' 'a-z' | cut -d_ -f1)
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex env_kernel --output-format csv \
      -d $OUT/pmc_$name -o run -- python3 $ROOT/bench.py --no-c5 $ARGS > $OUT/pmc_$name.log 2>&1) || exit $?
  echo "pass $C done"
done
