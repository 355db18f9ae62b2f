#!/bin/bash
# Build the GEMM lab on the GPU box (gpurun does not carry extension-less binaries) and run it on the
# given shapes ("M N K" each), every run under its own time limit.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/include tools/gemm_lab/lab.hip -o /tmp/lab
for s in "$@"; do timeout -k 5 90 /tmp/lab $s; done
