#!/bin/bash
# Fine re-check of the side-stream split-K targets after the round-6 kernels (ResNet 1x1 wgrads, BERT wgrads)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/split_fine
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "" "DTG_RESNET_WSPLIT_WGS=192" "DTG_RESNET_WSPLIT_WGS=384" "DTG_RESNET_WSPLIT_WGS=512" -- --steps 20 --warmup 5 && cp gpurun_out/ab.log gpurun_out/split_fine/resnet.log &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/bench_cfg.py timeout -k 10 900 bash tools/ab_bench.sh 3 "" "DTG_AB_SET=models.bert_fused._WSPLIT_WGS=384" "DTG_AB_SET=models.bert_fused._WSPLIT_WGS=768" -- --model bert --steps 20 --warmup 5 && cp gpurun_out/ab.log gpurun_out/split_fine/bert.log
