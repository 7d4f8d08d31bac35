#!/bin/bash
# The replayed aux pass on a second side stream (default) against the main stream
# (VN_AUX_REPLAY_MAIN=1): the bench's 4-env leg with thor-cached-auxiliary's replay sources
# (captured graph and eager), no profiler, alternating; after the replay tests.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
timeout -k 10 500 python -u -m pytest tests/test_replay_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r6s.log 2>&1; rc=$?; tail -3 gpurun_out/t_r6s.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in side main; do
    if [ $v = main ]; then export VN_AUX_REPLAY_MAIN=1; else unset VN_AUX_REPLAY_MAIN; fi
    timeout -k 10 300 python3 bench.py --no-c5 --steps 5 --warmup 1 --no-cpu-baseline --no-pmc --no-train-84 \
      --no-train-ff --no-train-174 --no-short --train-steps 1 --train-warmup 0 > gpurun_out/r6s_$v.log 2>&1 || exit 1
    python3 - gpurun_out/r6s_$v.log $v $rep <<'PY'
import json, sys
p = json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
r = p["train_174_lstm_aux_4env"]
print("%-5s rep %s: 4-env %.3f ms; replay graph %.3f ms, eager %.3f ms" % (sys.argv[2], sys.argv[3], r["ms_per_update"],
      r["replay_sources"]["ms_per_update"], r["replay_sources"]["eager_ms_per_update"]))
PY
  done
done
unset VN_AUX_REPLAY_MAIN
