#!/bin/bash
# vn_step copy-loop variants (VN_COPY_VARIANT, see vn_env.hip copy_two_frames), alternating rounds.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-0 1 2 3 4 5 6}; do
    VN_COPY_VARIANT=$v timeout -k 10 120 python3 bench.py --no-c5 --train-steps 0 --no-cpu-baseline --no-pmc --steps 1000 > gpurun_out/cv_$v$r.log 2>&1 || exit 1
    echo "cv $v r$r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/cv_$v$r.log) $(grep -o '"frac": [0-9.]*' gpurun_out/cv_$v$r.log | head -1)"
  done
done
