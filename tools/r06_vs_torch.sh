#!/bin/bash
# Final tree against stock PyTorch-ROCm on the same box (tools/torch_baseline.py: MIOpen / hipBLASLt / HF BERT, bf16
# autocast) at the round-2 comparison batches and at the headline batches, plus the kernel-vs-library microbenchmarks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/vs_torch
mkdir -p $O
timeout -k 10 600 python tools/bench_kernels.py --json $O/kbench.json > $O/kbench.log 2>&1 &&
timeout -k 10 600 python tools/torch_baseline.py --model resnet50 --batch 256 > $O/torch_resnet_b256.log 2>&1 &&
timeout -k 10 300 python bench.py --batch 256 > $O/dtg_resnet_b256.log 2>&1 &&
timeout -k 10 600 python tools/torch_baseline.py --model bert --batch 64 > $O/torch_bert_b64.log 2>&1 &&
timeout -k 10 300 python bench.py --model bert --batch 64 > $O/dtg_bert_b64.log 2>&1 &&
timeout -k 10 600 python tools/torch_baseline.py --model bert --batch 256 > $O/torch_bert_b256.log 2>&1 &&
timeout -k 10 900 python tools/torch_baseline.py --model resnet50 --batch 1024 > $O/torch_resnet_b1024.log 2>&1
