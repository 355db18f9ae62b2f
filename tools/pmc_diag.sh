#!/bin/bash
# Two PMC passes (issue/MFMA/LDS and TA/L2) over tools/op_bench.py cases, one rocprofv3 run each:
#   tools/pmc_diag.sh "<op args>" ...  -> gpurun_out/pmc_diag/<case>/{p1,p2}/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ITERS=${ITERS:-10}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES"
P2="TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for c in "$@"; do
  name=$(echo "$c" | tr ' ' '_')
  i=0
  for pass in "$P1" "$P2"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/pmc_diag/$name/p$i -o run --output-format csv -- \
      python3 tools/op_bench.py $c > gpurun_out/pmc_diag_${name}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $i of $c rc=$rc"; tail -5 gpurun_out/pmc_diag_${name}_p$i.log; exit $rc; fi
  done
done
