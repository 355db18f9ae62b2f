#!/bin/bash
# per-kernel times of the two stem max-pool forward kernels in the ResNet step (kernel trace, 2 runs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pool_rows
DTG_AB_POOL_ROWS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pool_rows/p0 -o run --output-format csv -- python3 tools/bench_cfg.py --steps 5 --warmup 3 > gpurun_out/pool_rows/p0.log 2>&1 &&
DTG_AB_POOL_ROWS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pool_rows/p1 -o run --output-format csv -- python3 tools/bench_cfg.py --steps 5 --warmup 3 > gpurun_out/pool_rows/p1.log 2>&1
