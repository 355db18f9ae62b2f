set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s4
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
i=1
for pass in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $pass -d gpurun_out/s4/p$i -o run --output-format csv -- python3 tools/stem_fwd_ab.py --batch 256 --rounds 1 > gpurun_out/s4/p$i.log 2>&1 || exit $?
  i=$((i+1))
done
