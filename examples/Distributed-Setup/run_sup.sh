#!/bin/bash
# 1 PS + 1 worker, Supervisor with checkpoints in ./logdir.
# Extra flags are forwarded, e.g. ./run.sh --observe_sleep 0 --cluster '{"ps":[...],"worker":[...]}'
# The parameter server exits by itself once every worker has finished (no pkill needed).
cd "$(dirname "$0")"
python dist_setup_sup.py --job_name "ps" --task_index 0 "$@" &
python dist_setup_sup.py --job_name "worker" --task_index 0 "$@" &
wait
