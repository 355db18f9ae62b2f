#!/bin/bash
# PS + two workers sharing one PS variable; extra flags (e.g. --cluster) are forwarded.
# Each process is waited for by PID, so a failing task fails the script (exit code of the first failure).
cd "$(dirname "$0")"
python Parameter-Server.py "$@" & ps=$!
python Local-then-Global-Variables-Worker1.py "$@" & w1=$!
python Local-then-Global-Variables-Worker2.py "$@" & w2=$!
rc=0
for pid in $w1 $w2 $ps; do
  wait "$pid"
  s=$?
  if [ "$s" -ne 0 ] && [ "$rc" -eq 0 ]; then rc=$s; fi
done
exit $rc
