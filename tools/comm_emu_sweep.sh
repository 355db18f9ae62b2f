#!/bin/bash
# One-card N>1 evidence under the pessimistic collective emulation (verdict r4, next-round item 3): bench.py with a
# one-rank RCCL group (DTG_DDP_FORCE=1) and DTG_COMM_EMULATE=<busbw>,<ranks>,<wgs>,<latency us>,<modes> for each
# mode set x workgroup count, one line per run: model, modes, wgs, img/s (or seq/s), ms/step, compute-only ms,
# exposed comm ms (bench.py's own split: the same step re-timed with the collectives off).
#   tools/comm_emu_sweep.sh <model> <busbw GB/s> "<modes...>" "<wgs...>" [bench.py flags]
# e.g. tools/comm_emu_sweep.sh resnet 100 "none busy busy+traffic" "32 64 128" --steps 20 --warmup 5
# Every run has its own time limit; the first failing run ends the script with its status.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
model=$1; bw=$2; modes=$3; wgss=$4; shift 4
mkdir -p gpurun_out
for m in $modes; do
  for w in $wgss; do
    mm=$m; [ "$m" = "none" ] && mm=""
    out=$(DTG_DDP_FORCE=1 DTG_COMM_EMULATE="$bw,8,$w,10,$mm" MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 \
          timeout -k 10 300 python bench.py --model "$model" "$@" 2>gpurun_out/emu_err.log)
    rc=$?
    if [ $rc -ne 0 ]; then echo "[$m $w] rc=$rc"; tail -20 gpurun_out/emu_err.log; exit $rc; fi
    echo "$out" | python -c "
import json, sys
d = json.loads([l for l in sys.stdin if l.startswith('{')][-1])
p = d.get('allreduce_probe', {})
print('$model', '${m}', $w, d['value'], d['ms_per_step'], p.get('compute_only_ms_per_step'), p.get('exposed_comm_ms_per_step'), flush=True)"
  done
done
