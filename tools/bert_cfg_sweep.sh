#!/bin/bash
# Every forced GEMM tile configuration on the BERT-base b256 step shapes, with the model's epilogues
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bert_cfg
C=0,1,14,15,25,26,27,28,29,30,31
timeout -k 10 300 python tools/gemm_ab.py --cfgs $C --rounds 3 --layout nt --epi gelu --shapes 32768x3072x768 > gpurun_out/bert_cfg/ffn1_gelu.log 2>&1 &&
timeout -k 10 300 python tools/gemm_ab.py --cfgs $C --rounds 3 --layout nt --epi bias --shapes 32768x2304x768,32768x768x768,32768x768x3072 > gpurun_out/bert_cfg/fwd_bias.log 2>&1 &&
timeout -k 10 300 python tools/gemm_ab.py --cfgs $C --rounds 3 --layout nn --epi dgelu --shapes 32768x3072x768 > gpurun_out/bert_cfg/ffn2_dgrad.log 2>&1 &&
timeout -k 10 300 python tools/gemm_ab.py --cfgs $C --rounds 3 --layout nn --shapes 32768x768x3072,32768x768x2304,32768x768x768 > gpurun_out/bert_cfg/dgrad.log 2>&1
