#!/bin/bash
# PMC passes of tools/gemm_pmc_lib.py (dtg vs hipBLASLt, BERT FFN shapes), each pass its own process and limit:
#   tools/gemm_pmc_lib.sh -> gpurun_out/gpl/<case>_p<i>, then tools/gemm_pmc_lib.py summary gpurun_out/gpl/*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for c in ffn1 ffn2; do
  for i in 1 2; do
    eval "pass=\$P$i"
    timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/gpl/${c}_p$i -o run --output-format csv -- \
      python3 tools/gemm_pmc_lib.py run $c > gpurun_out/gpl_${c}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $i of $c rc=$rc"; tail -5 gpurun_out/gpl_${c}_p$i.log; exit $rc; fi
  done
done
