#!/bin/bash
# Kernel traces of the ResNet step without a process group and on the forced one-rank DDP path (the N>1 code path)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ddp_ovh
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 > $O/plain.log 2>&1 &&
DTG_DDP_FORCE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29581 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ddp -o run --output-format csv -- python3 bench.py --steps 5 --warmup 3 > $O/ddp.log 2>&1
