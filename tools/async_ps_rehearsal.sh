#!/bin/bash
# One-card rehearsal of the ResNet-50 async parameter-server GPU path (BASELINE.json config 4):
# 1 PS + N workers, all on cuda:0, point-to-point over gloo with host staging
# (DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda).  On a node the same script runs over RCCL with one GPU
# per process (examples/ResNet50/run_async.sh).  Exits non-zero if any process fails.
#   tools/async_ps_rehearsal.sh [workers=2] [extra flags for resnet50_async_ps.py]
set -u
N=${1:-2}; shift || true
cd "$(dirname "$0")/../examples/ResNet50"
export DTG_BACKEND=gloo DTG_GLOO_DEVICE=cuda
PORT=$((23000 + RANDOM % 2000))
pids=()
timeout -k 10 240 python -u resnet50_async_ps.py --job_name ps --task_index 0 --workers "$N" --base_port $PORT "$@" &
pids+=($!)
for i in $(seq 0 $((N - 1))); do
  timeout -k 10 240 python -u resnet50_async_ps.py --job_name worker --task_index "$i" --workers "$N" --base_port $PORT "$@" &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "async_ps_rehearsal rc=$rc"
exit $rc
