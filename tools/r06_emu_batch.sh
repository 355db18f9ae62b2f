#!/bin/bash
# Final-tree N>1 emulation (8 ranks, 100 / 50 GB/s bus bandwidth, busy+traffic) for both models, then per-GPU batch
# sweeps of both steps.  Each run has its own time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/emu_batch
mkdir -p $O
bash tools/comm_emu_sweep.sh resnet 100 "none busy+traffic" "64" --steps 20 --warmup 5 > $O/emu_resnet_100.txt 2>&1 &&
bash tools/comm_emu_sweep.sh resnet 50 "busy+traffic" "64" --steps 20 --warmup 5 > $O/emu_resnet_50.txt 2>&1 &&
bash tools/comm_emu_sweep.sh bert 100 "none busy+traffic" "64" --steps 20 --warmup 5 > $O/emu_bert_100.txt 2>&1 &&
bash tools/comm_emu_sweep.sh bert 50 "busy+traffic" "64" --steps 20 --warmup 5 > $O/emu_bert_50.txt 2>&1 &&
for b in 512 768 1024 1280; do timeout -k 10 300 python bench.py --batch $b > $O/resnet_b$b.log 2>&1 || exit $?; done &&
for b in 128 256 384 512; do timeout -k 10 300 python bench.py --model bert --batch $b > $O/bert_b$b.log 2>&1 || exit $?; done
