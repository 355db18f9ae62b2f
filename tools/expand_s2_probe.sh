#!/bin/bash
# stride-2 projection on the gathered expand kernel: tests, isolated strided-conv timings, in-step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/expand_s2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_bn_fused_gpu.py -m gpu > gpurun_out/expand_s2/test.log 2>&1 &&
timeout -k 10 300 python tools/conv_tile_ab.py --strided --rounds 3 --codes 0 > gpurun_out/expand_s2/conv_s2.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_EXPAND_S2=0" "DTG_AB_EXPAND_S2=1" -- --steps 20 --warmup 5
