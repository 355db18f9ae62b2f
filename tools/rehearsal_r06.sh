#!/bin/bash
# Multi-rank rehearsal of the sync-DP path on one card (gloo over device tensors, every rank on cuda:0):
# ResNet-50 at 224 px (the stage-2..4 linear-halo weight gradients and the stage-1 halo kernels run), 2 and 4 ranks,
# and BERT, 2 ranks.  Each step has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rehearsal
export DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  tools/ddp_rehearsal.py --model resnet --batch 8 --image 224 > gpurun_out/rehearsal/resnet_2r.log 2>&1 &&
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29542 \
  tools/ddp_rehearsal.py --model resnet --batch 8 --image 224 > gpurun_out/rehearsal/resnet_4r.log 2>&1 &&
timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29543 \
  tools/ddp_rehearsal.py --model bert > gpurun_out/rehearsal/bert_2r.log 2>&1
