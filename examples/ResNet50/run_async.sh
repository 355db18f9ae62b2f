#!/bin/bash
# 1 PS + N workers, one process per MI355X (PS on GPU 0, worker i on GPU i+1).  Extra flags are forwarded.
# Waits for every process and exits non-zero if any of them failed.
cd "$(dirname "$0")"
N=${WORKERS:-7}
pids=()
HIP_VISIBLE_DEVICES=0 python resnet50_async_ps.py --job_name ps --task_index 0 --workers "$N" "$@" &
pids+=($!)
for i in $(seq 0 $((N - 1))); do
  HIP_VISIBLE_DEVICES=$((i + 1)) python resnet50_async_ps.py --job_name worker --task_index "$i" --workers "$N" "$@" &
  pids+=($!)
done
status=0
for p in "${pids[@]}"; do
  wait "$p" || status=1
done
exit $status
