#!/bin/bash
# Fused attention at the BERT-base step shape (B 256, S 128, 12 heads): timing with and without dropout, and one
# PMC pass (instruction mix + busy cycles) over the microbenchmark.  Each step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/attn_probe
timeout -k 10 120 python tools/bench_attention.py --B 256 --p 0.0 > gpurun_out/attn_probe/p0.log 2>&1 &&
timeout -k 10 120 python tools/bench_attention.py --B 256 --p 0.1 > gpurun_out/attn_probe/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d gpurun_out/attn_probe/pmc -o run --output-format csv -- python3 tools/bench_attention.py --B 256 --p 0.1 > gpurun_out/attn_probe/pmc.log 2>&1
