#!/bin/bash
# Full GPU test suite + smoke, then the BERT step ablation (interleaved A/B).  Each step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ck2
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ck2/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/ck2/smoke.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 2 \
  "" "DTG_WGRAD_STREAM=0" "DTG_AB_SET=models.bert_fused._ATTN=0" "DTG_AB_SET=models.bert_fused._FUSED_DBIAS=0" \
  -- --model bert --steps 20 --warmup 5 && cp gpurun_out/ab.log gpurun_out/ck2/ablation_bert.log
