#!/bin/bash
# 1 PS + 2 workers on localhost (same launcher shape as the reference's run.sh files).
cd "$(dirname "$0")"
python AEASGD.py --job_name "ps" --task_index 0 "$@" &
python AEASGD.py --job_name "worker" --task_index 0 "$@" &
python AEASGD.py --job_name "worker" --task_index 1 "$@" &
wait
