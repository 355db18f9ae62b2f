#!/bin/bash
# BN streaming-pass grid / unroll sweep (tools/bn_bench.py), one run per setting
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "DTG_BN_EWG=8192" "DTG_BN_EWG=16384" "DTG_BN_EWG=32768" "DTG_BN_EWG=16384 DTG_BN_RU=2" "DTG_BN_EWG=65536 DTG_BN_RU=2"; do
  name=$(echo "$cfg" | tr ' =' '_-')
  env $cfg timeout -k 5 200 python tools/bn_bench.py > gpurun_out/bn_$name.txt 2>&1
done
