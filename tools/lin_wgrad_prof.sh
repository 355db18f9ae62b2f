#!/bin/bash
# kernel-trace stats and two PMC passes of the linear-halo 3x3 weight gradient (tools/conv_wgrad_ab.py --only lin),
# plus the in-step-setting implicit GEMM (split target 256) for comparison.  Usage: tools/lin_wgrad_prof.sh [H]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
H=${1:-28}
OUT=$R/gpurun_out/linprof_$H
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/tools/conv_wgrad_ab.py --shapes $H --target 256 > $OUT/ab256.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/conv_wgrad_ab.py --shapes $H --only lin --iters 3 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/conv_wgrad_ab.py --shapes $H --only lin --iters 3 > $OUT/p2.log 2>&1 || exit $?
