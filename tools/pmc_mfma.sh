#!/bin/bash
# MFMA-utilisation PMC pass (one rocprofv3 run per op) over tools/op_bench.py cases:
#   tools/pmc_mfma.sh "<op args>" ...  -> gpurun_out/pmc_mfma/<case>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ITERS=${ITERS:-10}
P="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for c in "$@"; do
  name=$(echo "$c" | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_mfma/$name -o run --output-format csv -- \
    python3 tools/op_bench.py $c > gpurun_out/pmc_mfma_${name}.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc of $c rc=$rc"; tail -5 gpurun_out/pmc_mfma_${name}.log; exit $rc; fi
done
