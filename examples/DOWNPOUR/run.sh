#!/bin/bash
# DOWNPOUR (local Adagrad, summed T-step window, global Adagrad): 1 PS + 2 workers.
# Flags are forwarded to every task (e.g. --cluster '{"ps":[...],"worker":[...]}'); see ../launch_local.sh.
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here" && exec bash ../launch_local.sh DOWNPOUR.py 1 2 "$@"
