#!/bin/bash
# BERT FFN1 bias gradient: side-stream column sums vs the main-stream dgrad epilogue
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/b1side
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py tests/test_ddp_gpu.py -m gpu > gpurun_out/b1side/test.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_SET=models.bert_fused._B1_SIDE=0" "DTG_AB_SET=models.bert_fused._B1_SIDE=1" -- --model bert --steps 20 --warmup 5
