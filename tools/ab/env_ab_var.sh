#!/bin/bash
# A/B of an environment-variable switch on the training legs: VAR=value vs unset, alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
REF="--no-train-ref"; [ "${TRAIN_REF:-0}" = "1" ] && REF=""
for r in ${ROUNDS:-1 2}; do
  for v in on off; do
    if [ $v = on ]; then E="$VAR"; else E="VN_UNUSED=0"; fi
    env $E timeout -k 10 300 python3 bench.py --no-c5 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc $REF > gpurun_out/vab_$v$r.log 2>&1 || exit 1
    echo "$v $r $(grep -o '"ms_per_update": [0-9.]*' gpurun_out/vab_$v$r.log | tr '\n' ' ')"
  done
done
