#!/bin/bash
# One process per MI355X: the PS sees no GPU, worker i sees only GPU i (HIP_VISIBLE_DEVICES).
# Extra flags are forwarded.  The PS exits by itself once both workers have finished.
cd "$(dirname "$0")"
HIP_VISIBLE_DEVICES=-1 python dist_mult_gpu_sing_mach.py --job_name "ps" --task_index 0 "$@" &
HIP_VISIBLE_DEVICES=0 python dist_mult_gpu_sing_mach.py --job_name "worker" --task_index 0 "$@" &
HIP_VISIBLE_DEVICES=1 python dist_mult_gpu_sing_mach.py --job_name "worker" --task_index 1 "$@" &
wait
