#!/bin/bash
# BN-epilogue GEMM tiles at the ResNet-50 b1024 1x1 shapes: every forced configuration (0 = the heuristic)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bn_cfg
for c in 0 1 2 3 4 5 6; do
  timeout -k 10 200 python tools/bn_gemm_ab.py --batch 1024 --cfg $c > gpurun_out/bn_cfg/cfg$c.log 2>&1 || exit $?
done
