#!/bin/bash
# Synchronous SGD (SyncReplicasOptimizer, PS accumulators): 1 PS + 2 workers.
# Extra flags are forwarded, e.g. ./run.sh --observe_sleep 0 --cluster '{"ps":[...],"worker":[...]}'
# The parameter server exits by itself once every worker has finished (no pkill needed).
cd "$(dirname "$0")"
python ssgd.py --job_name "ps" --task_index 0 "$@" &
python ssgd.py --job_name "worker" --task_index 0 "$@" &
python ssgd.py --job_name "worker" --task_index 1 "$@" &
wait
