#!/bin/bash
# Round-6 ablation of the ResNet-50 step (bench.py defaults, b1024): each design choice switched off alone against
# the default, interleaved on one box (tools/ab_bench.sh), then the multi-rank DP rehearsal on one card.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
AB_SCRIPT=tools/bench_cfg.py timeout -k 10 1500 bash tools/ab_bench.sh 2 \
  "" \
  "DTG_WGRAD_STREAM=0" \
  "DTG_AB_LIN_WGRAD=0" \
  "DTG_AB_HALO=0" \
  "DTG_AB_HALO_DGRAD=0" \
  "DTG_AB_HALO_WGRAD=0" \
  "DTG_AB_STEM_STREAM=0" \
  "DTG_AB_SET=models.resnet_fused._DXW=0" \
  "DTG_AB_SET=models.resnet_fused._FUSE=0" \
  "DTG_AB_SET=models.resnet_fused._STEM=0" \
  -- --steps 20 --warmup 5 && cp gpurun_out/ab.log gpurun_out/ablation_resnet.log &&
bash tools/rehearsal_r06.sh
