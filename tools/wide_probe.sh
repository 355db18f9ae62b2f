#!/bin/bash
# 128x256 8-wave tile for BERT's wide short-K GEMMs: test, then in-step A/B of the two uses
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wide
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -m gpu -k "wide or colsum or gelu" > gpurun_out/wide/test.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 1000 bash tools/ab_bench.sh 3 "DTG_AB_WIDE=0" "DTG_AB_WIDE=1" "DTG_AB_WIDE=2" "DTG_AB_WIDE=3" -- --model bert --steps 20 --warmup 5
