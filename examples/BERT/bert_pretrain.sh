#!/bin/bash
# BERT-base pre-training (MLM + NSP), synchronous all-reduce DP on N GPUs (BASELINE config 5).
N=${1:-8}
cd "$(dirname "$0")/../.."
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --model bert --gpus "$N" --steps 50 --warmup 10
