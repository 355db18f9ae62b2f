#!/bin/bash
# Synchronous SGD through SyncReplicasOptimizer: 1 PS + 2 workers.
# Flags are forwarded to every task (e.g. --cluster '{"ps":[...],"worker":[...]}'); see ../launch_local.sh.
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here" && exec bash ../launch_local.sh ssgd.py 1 2 "$@"
