#!/bin/bash
# tools/bn_gemm_ab.py under every forced BN-GEMM tile configuration, one process each
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in 0 1 2 3 4 5 6; do
  DTG_BN_GEMM_CFG=$c timeout -k 5 150 python tools/bn_gemm_ab.py > gpurun_out/bn_gemm_cfg$c${DTG_BN_AB_BATCH:+_b$DTG_BN_AB_BATCH}.txt 2>&1
done
