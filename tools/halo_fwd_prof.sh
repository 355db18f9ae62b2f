#!/bin/bash
# isolated time + one PMC pass of the stage-1 halo forward conv (tools/halo_fwd_bench.py)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/hfw
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 python3 $R/tools/halo_fwd_bench.py > $OUT/iso.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/halo_fwd_bench.py --iters 3 > $OUT/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/halo_fwd_bench.py --iters 3 > $OUT/p2.log 2>&1 || exit $?
