set -e
cd $GRAFT_REPO_ROOT
for hw in "56 64 64" "28 128 128" "14 256 256" "7 512 512"; do
  set -- $hw
  for op in conv_fwd conv_fwd_bn conv_dgrad conv_dgrad_bn conv_wgrad; do
    timeout -k 5 60 python tools/op_bench.py $op 256 $1 $2 $3 3 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/convsweep.txt
