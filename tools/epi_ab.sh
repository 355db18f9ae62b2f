#!/bin/bash
# Standalone timings of the BN-epilogue GEMM / conv kernels on the ResNet-50 shapes (tools/op_bench.py)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in "gemm_bn3 802816 256 64" "gemm_bn3 50176 1024 256" "gemm_bn3 200704 512 128" "gemm_bn3 12544 2048 512" \
         "gemm_bn2 50176 256 1024" "gemm_bn2 802816 64 256" "gemm_bn2 200704 128 512" \
         "conv_dgrad_bn 256 14 256 256 3 1" "conv_dgrad_bn 256 56 64 64 3 1" "conv_dgrad_bn 256 28 128 128 3 1" \
         "conv_dgrad 256 14 256 256 3 1" "conv_dgrad 256 56 64 64 3 1"; do
  timeout -k 5 60 python tools/op_bench.py $c 2>&1 | grep -v amdgpu.ids
done
