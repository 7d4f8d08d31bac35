#!/bin/bash
# Round-6 PMC tables (tools/pmc_leg.sh: three counter passes over exactly one marked update) of the
# 174², C5 and 4-env legs, then the logged-run replay (tools/replicate_log.py --experiment
# thor-cached-auxiliary). Each step under its own limit; stops at the first failure.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
export TMPDIR=/tmp
T=${TAG:-r06}
for L in ${PMC_LEGS:-174 c5 ref4}; do
  echo "== pmc leg $L"
  LEG=$L TAG=${L}_$T timeout -k 10 700 bash tools/pmc_leg.sh > gpurun_out/pmc_leg_${L}_$T.log 2>&1 || { tail -5 gpurun_out/pmc_leg_${L}_$T.log; exit 1; }
  cp gpurun_out/pmcleg_${L}_$T/table.md gpurun_out/pmc_leg_${L}_$T.md
  head -12 gpurun_out/pmc_leg_${L}_$T.md
done
if [ "${REPLICATE:-1}" = "1" ]; then
  echo "== replicate log"
  timeout -k 10 600 python3 tools/replicate_log.py 12500 gpurun_out/replicate_log_curve_$T.csv --experiment > gpurun_out/replicate_log_$T.log 2>&1 || { tail -5 gpurun_out/replicate_log_$T.log; exit 1; }
  tail -8 gpurun_out/replicate_log_$T.log
fi
echo "== done"
