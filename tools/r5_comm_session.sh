#!/bin/bash
# Round-5 one-card N>1 evidence session (verdict r4 item 3), run on a GPU box from the repo root:
#   1. ResNet-50 b1024 and BERT b256 under the emulated 8-rank collective at 100 GB/s bus bandwidth, the
#      round-4 (sleeping, no traffic) form vs the pessimistic forms (busy-poll; busy-poll + ring HBM traffic),
#      32 / 64 / 128 workgroups (tools/comm_emu_sweep.sh);
#   2. a kernel trace of the ResNet step with one-rank out-of-place all-gathers on the process group's stream
#      (DTG_COMM_QUEUE_PROBE=1) next to the pessimistic emulation, for tools/queue_trace.py.
# Every GPU step has its own time limit and the steps are chained: the first failure ends the script.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r5_comm
mkdir -p "$out"
tools/comm_emu_sweep.sh resnet 100 "none busy busy+traffic" "32 64 128" --steps 15 --warmup 4 > "$out/sweep_resnet.txt"
tools/comm_emu_sweep.sh bert 100 "none busy+traffic" "32 128" --steps 15 --warmup 4 > "$out/sweep_bert.txt"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
DTG_DDP_FORCE=1 DTG_COMM_EMULATE="100,8,64,10,busy+traffic" DTG_COMM_QUEUE_PROBE=1 MASTER_ADDR=127.0.0.1 \
  MASTER_PORT=29581 timeout -k 10 300 rocprofv3 --kernel-trace -d "$out/qt" -o qt --output-format csv -- \
  python3 bench.py --steps 8 --warmup 3 > "$out/qt_bench.log" 2>&1
trace=$(find "$out/qt" -name "*kernel_trace.csv" | head -1)
python tools/queue_trace.py "$trace" --skip 3 --out "$out/queues_probe.md"
rm -f "$trace"
