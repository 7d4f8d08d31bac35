#!/bin/bash
# Same-box A/B of the replayed aux pass merged into the replayed UNREAL pass (VN_REPLAY_MERGED=1)
# against the separate passes (the default): the bench's 4-env leg (replay_sources: captured graph and
# eager), no profiler, alternating REPS times.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
for rep in $(seq 1 ${REPS:-3}); do
  for v in merged separate; do
    if [ $v = merged ]; then export VN_REPLAY_MERGED=1; else unset VN_REPLAY_MERGED; fi
    timeout -k 10 300 python3 bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-train-84 \
      --no-train-ff --no-train-174 --no-short --train-steps 1 --train-warmup 0 > gpurun_out/replay_ab_$v.log 2>&1 || exit 1
    python3 - gpurun_out/replay_ab_$v.log $v $rep <<'PY'
import json, sys
p = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
r = p["train_174_lstm_aux_4env"]["replay_sources"]
print("%-9s rep %s: replay graph %.3f ms, eager %.3f ms" % (sys.argv[2], sys.argv[3], r["ms_per_update"], r["eager_ms_per_update"]))
PY
  done
done
unset VN_REPLAY_MERGED
