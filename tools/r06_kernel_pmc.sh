#!/bin/bash
# PMC passes over the ResNet and BERT steps for the round-6 kernels (expand K=256 / stride-2 gather, row-walking
# stem pool, linear-halo wgrad, transposed attention forward): instruction mix, LDS bank conflicts, busy / wait cycles.
# One counter group per rocprofv3 run, each under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/kpmc
mkdir -p $O
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $pass -d $O/resnet_p$i -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $O/resnet_p$i.log 2>&1 || exit $?
  timeout -s KILL 300 rocprofv3 --pmc $pass -d $O/bert_p$i -o run --output-format csv -- python3 bench.py --model bert --steps 2 --warmup 1 > $O/bert_p$i.log 2>&1 || exit $?
done
