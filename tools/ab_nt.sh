#!/bin/bash
# A/B of nontemporal stores for conv1's X1 (VN_NT_X1) and conv2's dX1 (VN_NT_DX1): the 84x84
# and 174x174 training legs under each setting, interleaved twice. The two switches existed for
# this run only (both slower, profiles/r05/ab_nt/; removed): the script records how it was measured.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-/root/repo}
cd $ROOT
OUT=gpurun_out/ab_nt
mkdir -p $OUT
ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-pmc --no-train-ff --no-train-ref4 --no-c5 --no-short"
for rep in 1 2; do
  for cfg in none dx1 x1 both; do
    case $cfg in
      none) E="" ;; dx1) E="VN_NT_DX1=1" ;; x1) E="VN_NT_X1=1" ;; both) E="VN_NT_DX1=1 VN_NT_X1=1" ;;
    esac
    env $E timeout -k 10 300 python bench.py $ARGS > $OUT/bench_$cfg.$rep.log 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/bench_$cfg.$rep.log') if l.startswith('{')][-1])
print('$cfg', {k: round(v['ms_per_update'], 2) for k, v in d.items() if isinstance(v, dict) and 'ms_per_update' in v})"
  done
done
