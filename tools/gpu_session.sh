#!/bin/bash
# One GPU-box session: tests, benchmark, profile.  Every GPU step has its own time limit; a
# crash/fault/timeout (exit >= 124 or signal) stops the session so nothing else touches the GPU.
# Usage: tools/gpu_session.sh [steps...]   steps: test test_tf bench bench_bert prof prof_bert kbench smoke ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ $# -eq 0 ]; then set -- test bench prof; fi

run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "fatal rc=$rc in $name: stopping session"
    exit $rc
  fi
  return 0
}

for s in "$@"; do
  case $s in
    test) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    test_tf) run pytest_tf 600 python -m pytest tests/test_transformer_gpu.py -m gpu -q ;;
    bench_bert) run bench_bert 600 python bench.py --model bert --steps 20 --warmup 5 ;;
    prof_bert) run prof_bert 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- \
            python3 bench.py --model bert --steps 5 --warmup 3 ;;
    smoke) run smoke 300 python __graft_entry__.py smoke ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench_pg) DTG_DDP_FORCE=1 run bench_pg 600 python bench.py --steps 20 --warmup 5 ;;
    bench_pg_main) DTG_DDP_FORCE=1 DTG_WGRAD_STREAM=0 run bench_pg_main 600 python bench.py --steps 20 --warmup 5 ;;
    prof_pg) DTG_DDP_FORCE=1 run prof_pg 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pg -o run --output-format csv -- \
            python3 bench.py --steps 4 --warmup 3 ;;
    test_launch) run pytest_launch 400 python -u -m pytest tests/test_launch_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    bench_emu) DTG_DDP_FORCE=1 DTG_COMM_EMULATE=${EMU:-100} run bench_emu 600 python bench.py --steps 20 --warmup 5 ;;
    prof_emu) DTG_DDP_FORCE=1 DTG_COMM_EMULATE=${EMU:-100} run prof_emu 900 rocprofv3 --kernel-trace -d gpurun_out/prof_emu -o run \
            --output-format csv -- python3 bench.py --steps 6 --warmup 3 ;;
    test_resnet) run pytest_resnet 900 python -u -m pytest tests/test_resnet_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread ;;
    kbench) run kbench 600 python tools/bench_kernels.py --json gpurun_out/kbench.json ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
            python3 bench.py --steps 5 --warmup 3 ;;
    *) run "$(echo "$s" | tr -c 'A-Za-z0-9_.-' '_' | cut -c1-80)" 900 bash -c "$s < /dev/null" ;;
  esac
done
