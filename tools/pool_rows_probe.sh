#!/bin/bash
# row-walking stem max-pool forward: tests, then the in-step A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pool_rows
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_resnet_gpu.py -m gpu > gpurun_out/pool_rows/test.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_POOL_ROWS=0" "DTG_AB_POOL_ROWS=1" -- --steps 20 --warmup 5
