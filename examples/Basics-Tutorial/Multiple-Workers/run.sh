#!/bin/bash
# PS + two workers sharing one PS variable; extra flags (e.g. --cluster) are forwarded.
cd "$(dirname "$0")"
python Parameter-Server.py "$@" &
python Local-then-Global-Variables-Worker1.py "$@" &
python Local-then-Global-Variables-Worker2.py "$@" &
wait
