#!/bin/bash
# N=2 rehearsal of bench.py --no-c5 on ONE GPU (both ranks share cuda:0): gloo backend, short legs.
# Checks the multi-process path end to end (barrier, max-over-ranks timing, the trainer's
# gradient all-reduce and parameter broadcast) where no second GPU exists.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p gpurun_out
export CUDA_VISIBLE_DEVICES=0
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --no-c5 --gpus 2 --steps 200 --warmup 20 --envs 1024 --train-steps 2 --train-warmup 1 \
  --no-train-ff --dist-backend ${BACKEND:-gloo} > gpurun_out/dist2_${BACKEND:-gloo}.log 2>&1
rc=$?; grep '^{' gpurun_out/dist2_${BACKEND:-gloo}.log | cut -c1-600; tail -3 gpurun_out/dist2_${BACKEND:-gloo}.log | cut -c1-300; exit $rc
