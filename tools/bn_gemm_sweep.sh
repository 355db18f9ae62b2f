#!/bin/bash
# tools/bn_gemm_ab.py under every forced BN-GEMM tile configuration, one process each
#   tools/bn_gemm_sweep.sh [batch=512]
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
b=${1:-512}
for c in 0 1 2 3 4 5 6; do
  timeout -k 5 150 python tools/bn_gemm_ab.py --cfg $c --batch $b > gpurun_out/bn_gemm_cfg${c}_b$b.txt 2>&1
done
