#!/bin/bash
# Round-6 final evidence from the committed tree, one box: GPU suite, smoke, ResNet-50 and BERT benches (3 each),
# kernel traces of both steps, whole-step PMC passes of both.  Every GPU step has its own time limit; the first
# failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
step() { echo "=== $1 $(date +%T)"; }
step pytest && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
step smoke && timeout -k 10 300 python __graft_entry__.py smoke > $O/smoke.log 2>&1 &&
step bench && for i in 1 2 3; do timeout -k 10 300 python bench.py > $O/bench_$i.log 2>&1 || exit $?; done &&
step bench_bert && for i in 1 2 3; do timeout -k 10 300 python bench.py --model bert > $O/bench_bert_$i.log 2>&1 || exit $?; done &&
step prof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 > $O/prof.log 2>&1 &&
step prof_bert && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_bert -o run --output-format csv -- python3 bench.py --model bert --steps 5 --warmup 3 > $O/prof_bert.log 2>&1 &&
step pmc_resnet && bash tools/pmc_step.sh > $O/pmc_resnet.log 2>&1 && mv gpurun_out/pmc_step $O/pmc_resnet &&
step pmc_bert && bash tools/pmc_step.sh --model bert > $O/pmc_bert.log 2>&1 && mv gpurun_out/pmc_step $O/pmc_bert &&
step done
