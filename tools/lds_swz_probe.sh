#!/bin/bash
# 64-row MC swizzle fix: full GPU suite, attention microbenchmark, LDS bank-conflict counters, then in-step A/B of
# both models against the previous commit built in a worktree (.ab_old, tools/ab_tree.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/lds_swz
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python tools/bench_attention.py --B 256 --p 0.1 > $O/attn_new.log 2>&1 &&
timeout -k 10 120 python .ab_old/tools/bench_attention.py --B 256 --p 0.1 > $O/attn_old.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_new -o run --output-format csv -- python3 tools/bench_attention.py --B 256 --p 0.1 > $O/pmc_new.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/pmc_old -o run --output-format csv -- python3 .ab_old/tools/bench_attention.py --B 256 --p 0.1 > $O/pmc_old.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/ab_tree.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_TREE=.ab_old" "DTG_AB_TREE=." -- --model bert --steps 20 --warmup 5 && cp gpurun_out/ab.log $O/ab_bert.log &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/ab_tree.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_TREE=.ab_old" "DTG_AB_TREE=." -- --steps 20 --warmup 5 && cp gpurun_out/ab.log $O/ab_resnet.log
