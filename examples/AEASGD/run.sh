#!/bin/bash
# AEASGD / AEAMSGD (elastic averaging): 1 PS + 2 workers on localhost.
# Flags are forwarded to every task (e.g. --cluster '{"ps":[...],"worker":[...]}'); see ../launch_local.sh.
here="$(cd "$(dirname "$0")" && pwd)"
cd "$here" && exec bash ../launch_local.sh AEASGD.py 1 2 "$@"
