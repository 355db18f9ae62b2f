#!/bin/bash
# Final-tree runs of BASELINE configs 2 (MNIST CNN, bench.py --model mnist, batch 512 / 4096) and 4 (ResNet-50 async
# parameter server: 1 PS + 2 workers on one card, then bench.py --mode async_ps on one rank)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/configs
mkdir -p $O
timeout -k 10 300 python bench.py --model mnist > $O/mnist_b512.log 2>&1 &&
timeout -k 10 300 python bench.py --model mnist --batch 4096 > $O/mnist_b4096.log 2>&1 &&
timeout -k 10 300 bash tools/async_ps_rehearsal.sh 2 > $O/async_ps_rehearsal.log 2>&1
