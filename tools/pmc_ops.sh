#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, each under its own time limit) over tools/op_bench.py
# cases.  Usage: tools/pmc_ops.sh "<op args>" ["<op args>" ...]   -> gpurun_out/pmc/<case>/<pass>/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp ITERS=${ITERS:-10}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="FETCH_SIZE"
P3="WRITE_SIZE"
P4="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
for c in "$@"; do
  name=$(echo "$c" | tr ' ' '_')
  timeout -k 10 120 python tools/op_bench.py $c || exit $?
  i=0
  for pass in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i + 1))
    timeout -s KILL 90 rocprofv3 --pmc $pass -d gpurun_out/pmc/$name/p$i -o run --output-format csv -- \
      python3 tools/op_bench.py $c > gpurun_out/pmc_${name}_p$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc pass $i of $c rc=$rc"; tail -5 gpurun_out/pmc_${name}_p$i.log; exit $rc; fi
  done
done
