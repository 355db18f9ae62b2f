#!/bin/bash
# LayerNorm forward with 4-element lane chunks: tests, in-step BERT A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ln4
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -m gpu > gpurun_out/ln4/test.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_LN_FWD4=0" "DTG_AB_LN_FWD4=1" -- --model bert --steps 20 --warmup 5
