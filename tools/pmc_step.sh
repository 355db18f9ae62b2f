#!/bin/bash
# Whole-step PMC passes over bench.py (one counter group per rocprofv3 run, each under its own time limit);
# summarised by tools/pmc_step.py.  Usage: tools/pmc_step.sh [bench.py args...]  -> gpurun_out/pmc_step/p*/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for pass in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $pass -d gpurun_out/pmc_step/p$i -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 "$@" > gpurun_out/pmc_step_p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pmc pass $i rc=$rc"; tail -5 gpurun_out/pmc_step_p$i.log; exit $rc; fi
done
