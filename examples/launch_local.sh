#!/bin/bash
# Local-cluster launcher shared by the examples' run scripts.
#
#   launch_local.sh [--gpu] SCRIPT NUM_PS NUM_WORKERS [flags forwarded to every task ...]
#
# Starts NUM_PS parameter-server tasks and NUM_WORKERS worker tasks of SCRIPT on this host
# (`--job_name ps|worker --task_index i`, the ClusterSpec-style CLI of every example), waits for
# all of them and exits non-zero if any task failed.  The PS tasks exit by themselves once every
# worker has reported done, so nothing has to be killed by hand.
# --gpu: one MI355X per worker process (HIP_VISIBLE_DEVICES=<worker index>); PS tasks see no GPU.
gpu=0
if [ "$1" = "--gpu" ]; then
  gpu=1
  shift
fi
script=$1
nps=$2
nworkers=$3
shift 3

pids=()
spawn() {  # spawn JOB INDEX DEVICES [flags...]
  local job=$1 idx=$2 devs=$3
  shift 3
  if [ "$gpu" = 1 ]; then
    HIP_VISIBLE_DEVICES=$devs python "$script" --job_name "$job" --task_index "$idx" "$@" &
  else
    python "$script" --job_name "$job" --task_index "$idx" "$@" &
  fi
  pids+=($!)
}

for ((i = 0; i < nps; i++)); do spawn ps "$i" -1 "$@"; done
for ((i = 0; i < nworkers; i++)); do spawn worker "$i" "$i" "$@"; done

status=0
for p in "${pids[@]}"; do
  wait "$p" || status=1
done
exit $status
