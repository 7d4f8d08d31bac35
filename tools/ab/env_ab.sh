#!/bin/bash
# A/B of the env step kernel: bench env leg with the in-tree library and with
# tools/ab/libvnav_head.so, alternating, 3 rounds each.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
cp $L /tmp/new.so
for r in 1 2 3; do
  for v in new head; do
    if [ $v = new ]; then cp /tmp/new.so $L; else cp tools/ab/libvnav_head.so $L; fi
    timeout -k 10 120 python3 bench.py --no-c5 --train-steps 0 --no-cpu-baseline --no-pmc --steps 400 > gpurun_out/envab_$v$r.log 2>&1 || exit 1
    echo "$v $r $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/envab_$v$r.log) $(grep -o '"value": [0-9.]*' gpurun_out/envab_$v$r.log | head -1)"
  done
done
cp /tmp/new.so $L
