#!/bin/bash
# SQ counters per training kernel of one bench leg: three rocprofv3 --pmc passes (no tracing,
# <= 8 SQ / 2 GRBM counters each) over `bench.py --pmc-leg LEG` (one warmup + one marked update),
# then tools/pmc_leg_table.py. Usage on the GPU box: LEG=c5 TAG=x bash tools/pmc_leg.sh
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/pmcleg_${TAG:-x}
LEG=${LEG:-174}
mkdir -p $OUT
i=0
for SET in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU"; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $SET --output-format csv -d $OUT/k$i -o run \
      -- python3 $ROOT/bench.py --pmc-leg $LEG > $OUT/k$i.log 2>&1) || exit $?
  echo "pass $i done"
done
python3 $ROOT/tools/pmc_leg_table.py $OUT > $OUT/table.md && cat $OUT/table.md
