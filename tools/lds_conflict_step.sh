#!/bin/bash
# LDS bank-conflict cycles per kernel class over both training steps (one PMC pass each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ldsc
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/resnet -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 > $O/resnet.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE -d $O/bert -o run --output-format csv -- python3 bench.py --model bert --steps 2 --warmup 1 > $O/bert.log 2>&1
