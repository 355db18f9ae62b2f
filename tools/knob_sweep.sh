#!/bin/bash
# A/B of the env knobs of dtg's kernel heuristics on the full bench step (one bench run per knob)
#   tools/knob_sweep.sh resnet|bert
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
model=${1:-resnet}
run() { echo "== $*"; env "$@" timeout -k 5 120 python bench.py --model $model --steps 10 --warmup 3 2>/dev/null | grep -o '"value": [0-9.]*'; }
if [ "$model" = resnet ]; then
  run X=0
  run DTG_CONV_STAGES=1
  run DTG_CONV_STAGES=2
  run DTG_CONV_STAGES=3
  run DTG_GEMM_RP=0
  run DTG_WGRAD_BLOCKS=512
  run DTG_WGRAD_BLOCKS=2048
  run DTG_BN_BITS=0
  run X=0
elif [ "$model" = bert_wgrad ]; then  # weight-gradient placement / split-K knobs of the BERT step
  model=bert
  run X=0
  run DTG_WGRAD_STREAM=0
  run DTG_GEMM_SPLIT_WGS=256
  run DTG_GEMM_SPLIT_WGS=1024
  run DTG_SIDE_PRIO=0
  run DTG_WGRAD_STREAM=0 DTG_GEMM_SPLIT_WGS=256
  run X=0
else
  run X=0
  run DTG_LN_BWD_BLOCKS=1024
  run DTG_LN_BWD_BLOCKS=2048
  run DTG_LN_BWD_BLOCKS=256
  run DTG_GEMM_RP=0
  run X=0
fi
