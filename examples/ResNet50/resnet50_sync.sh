#!/bin/bash
# ResNet-50 synchronous all-reduce data parallelism on N GPUs of this node (BASELINE config 3).
N=${1:-8}
cd "$(dirname "$0")/../.."
python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus "$N" --steps 50 --warmup 10
