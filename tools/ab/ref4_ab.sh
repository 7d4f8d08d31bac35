#!/bin/bash
# A/B of two library builds on the logged run's batch (174x174, 4 envs x 20, hipGraph): the
# 4-env bench leg with the in-tree libvnav.so ("new") and tools/ab/$ALT, alternating REPS times;
# prints the leg's ms per update (and the replayed-batch form's when the line carries it).
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
ALT=${ALT:-libvnav_pre.so}
cp $L /tmp/new.so
for rep in $(seq ${REPS:-3}); do
  for v in new $ALT; do
    if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/$v $L; fi
    timeout -k 10 300 python3 bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-train-ff \
      --no-train-84 --no-train-174 --no-short > gpurun_out/r4ab_${v}_$rep.log 2>&1 || { cp /tmp/new.so $L; exit 1; }
    python3 - gpurun_out/r4ab_${v}_$rep.log $v $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
leg = d["train_174_lstm_aux_4env"]
extra = {k: v for k, v in leg.items() if "replay" in k and isinstance(v, (int, float))}
print(sys.argv[2], "rep", sys.argv[3], "ms_per_update %.4f" % leg["ms_per_update"], extra)
PY
  done
done
cp /tmp/new.so $L
