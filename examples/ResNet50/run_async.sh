#!/bin/bash
# 1 PS + N workers, one process per MI355X: rank r (PS = 0, worker i = i + 1) uses GPU r, and every process
# sees every GPU, so RCCL's point-to-point transfers can take the direct xGMI link of each PS<->worker pair
# (a process pinned with HIP_VISIBLE_DEVICES to one device cannot see its peers).  Extra flags are forwarded.
# Waits for every process and exits non-zero if any of them failed.
cd "$(dirname "$0")"
N=${WORKERS:-7}
pids=()
python resnet50_async_ps.py --job_name ps --task_index 0 --workers "$N" "$@" &
pids+=($!)
for i in $(seq 0 $((N - 1))); do
  python resnet50_async_ps.py --job_name worker --task_index "$i" --workers "$N" "$@" &
  pids+=($!)
done
status=0
for p in "${pids[@]}"; do
  wait "$p" || status=1
done
exit $status
