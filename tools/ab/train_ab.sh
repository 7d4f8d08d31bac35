#!/bin/bash
# A/B of the training legs: bench (84x84 LSTM + feed-forward legs; TRAIN_REF=1 adds the
# 174x174 leg) with the in-tree library and with tools/ab/libvnav_head.so, alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
cp $L /tmp/new.so
REF="--no-train-ref"; [ "${TRAIN_REF:-0}" = "1" ] && REF=""
for r in ${ROUNDS:-1 2}; do
  for v in new head; do
    if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/libvnav_head.so $L; fi
    timeout -k 10 300 python3 bench.py --no-c5 --steps 20 --warmup 5 --no-cpu-baseline --no-pmc $REF > gpurun_out/trab_$v$r.log 2>&1 || exit 1
    echo "$v $r $(grep -o '"ms_per_update": [0-9.]*' gpurun_out/trab_$v$r.log | tr '\n' ' ')"
  done
done
cp /tmp/new.so $L
