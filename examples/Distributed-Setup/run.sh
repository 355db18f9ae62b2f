#!/bin/bash
# PS hello world with MonitoredTrainingSession: 1 PS + 1 worker.
# Flags are forwarded to every task (e.g. --cluster '{"ps":[...],"worker":[...]}'); see ../launch_local.sh.
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here" && exec bash ../launch_local.sh dist_setup.py 1 1 "$@"
