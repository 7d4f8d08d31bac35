#!/bin/bash
# A/B: train_hash.py with the in-tree library (new) twice, then with tools/ab/libvnav_head.so.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
L=a2cat-vn-pytorch_amd/vnav/_lib/libvnav.so
U=${U:-200}
timeout -k 10 200 python3 -u tools/ab/train_hash.py $U > gpurun_out/ab_new1.log 2>&1 &&
true &&
cp tools/ab/libvnav_head.so $L &&
timeout -k 10 200 python3 -u tools/ab/train_hash.py $U > gpurun_out/ab_head.log 2>&1 &&
paste gpurun_out/ab_new1.log gpurun_out/ab_head.log
