#!/bin/bash
# Process-per-GPU asynchronous DP: the PS sees no GPU, worker i sees only MI355X i.
# Flags are forwarded to every task (e.g. --cluster '{"ps":[...],"worker":[...]}'); see ../launch_local.sh.
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here" && exec bash ../launch_local.sh --gpu dist_mult_gpu_sing_mach.py 1 2 "$@"
