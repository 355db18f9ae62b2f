#!/bin/bash
# K = 256 streaming expand GEMM: tests, then an in-step A/B (plus the strided-conv weight-gradient split target)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/expand256
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused_gpu.py -m gpu > gpurun_out/expand256/test.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_EXPAND256=0" "DTG_AB_EXPAND256=1" "DTG_RESNET_CWSPLIT_WGS=128" -- --steps 20 --warmup 5
