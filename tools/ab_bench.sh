#!/bin/bash
# Interleaved A/B of bench.py under different environments, on one box (cdna_hip_programming.md §5.4 rule 24):
#   tools/ab_bench.sh ROUNDS "ENV_A" "ENV_B" [...] -- [bench.py flags]
# e.g. tools/ab_bench.sh 2 "" "DTG_WGRAD8=1" -- --steps 20 --warmup 5
# Each run has its own time limit; the first failing run ends the script with its status.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
rounds=$1; shift
envs=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
[ $# -gt 0 ] && shift
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
  for e in "${envs[@]}"; do
    out=$(env $e timeout -k 10 300 python ${AB_SCRIPT:-bench.py} "$@" 2>gpurun_out/ab_err.log)
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$e] rc=$rc"; tail -20 gpurun_out/ab_err.log; exit $rc; fi
    v=$(echo "$out" | python -c "import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d.get('allreduce_probe',''))")
    echo "round $r [${e:-default}] $v" | tee -a gpurun_out/ab.log
  done
done
