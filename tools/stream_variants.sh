#!/bin/bash
# One-rank RCCL process group (DTG_DDP_FORCE=1) on one GPU: ResNet-50 b512 bench + a short kernel trace per
# stream-layout variant, to see which HIP streams share a hardware queue (Queue_Id per dispatch).
#   tools/stream_variants.sh "name:VAR=1 VAR2=x" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  echo "=== $name: $envs"
  env $envs DTG_DDP_FORCE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/sv_$name.log 2>&1 || { echo "bench rc=$?"; exit 1; }
  grep '^{' gpurun_out/sv_$name.log | python3 -c "import json,sys; j=json.loads(sys.stdin.read()); print('$name', j['value'], j['ms_per_step'])"
  env $envs DTG_DDP_FORCE=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/sv_$name -o run --output-format csv -- \
      python3 bench.py --steps 2 --warmup 2 > gpurun_out/sv_${name}_prof.log 2>&1 || { echo "prof rc=$?"; exit 1; }
done
