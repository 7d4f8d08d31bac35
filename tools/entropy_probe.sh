#!/bin/bash
# Late-entropy investigation: the logged run's replay (tools/replicate_log.py,
# 12,500 updates of 4 envs x 20) with another seed and with smaller entropy coefficients, as
# parallel processes on one GPU (each is launch-bound at 4 envs). Outputs under gpurun_out/entropy.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
OUT=gpurun_out/entropy
mkdir -p $OUT
U=${UPDATES:-12500}
pids=()
for v in "ec0.01_s1:--seed 1" "ec0.001_s0:--entropy-coef 0.001" "ec0_s0:--entropy-coef 0" "ec0.01_s0_noaux:--aux-weight 0"; do
  tag=${v%%:*}; a=${v#*:}
  timeout -k 10 900 python -u tools/replicate_log.py $U $OUT/$tag.csv $a > $OUT/$tag.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
tail -n 3 $OUT/*.log
exit $rc
