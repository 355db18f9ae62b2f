#!/bin/bash
# PMC passes (SQ / L2 / SQ waits) over tools/op_bench.py gemm for each "cfg M N K" case, each under its own
# limit.  Usage: tools/gemm_pmc.sh "98 32768 3072 768" ["0 8192 8192 8192" ...]  -> gpurun_out/gpmc/<case>/p{1,2,3}
# PASSES="1 3" selects passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ITERS=${ITERS:-10}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
P2="TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum TCC_EA0_RDREQ_sum"
P3="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for c in "$@"; do
  set -- $c
  cfg=$1; shift
  name="cfg${cfg}_$1x$2x$3"
  for i in ${PASSES:-1 2}; do
    eval "pass=\$P$i"
    GEMM_CFG=$cfg timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/gpmc/$name/p$i -o run --output-format csv -- \
      python3 tools/op_bench.py gemm "$@" > gpurun_out/gpmc_${name}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $i of $c rc=$rc"; tail -5 gpurun_out/gpmc_${name}_p$i.log; exit $rc; fi
  done
done
