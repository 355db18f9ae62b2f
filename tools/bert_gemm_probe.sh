set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/gemm_ab.py --cfgs 0 --layout nt --shapes 32768x3072x768,32768x768x3072,32768x2304x768,32768x768x768 > gpurun_out/gab_nt.log 2>&1 &&
timeout -k 10 300 python tools/gemm_ab.py --cfgs 0 --layout nn --shapes 32768x3072x768,32768x768x3072,32768x768x2304,32768x768x768 > gpurun_out/gab_nn.log 2>&1 &&
timeout -k 10 300 python tools/gemm_ab.py --cfgs 0 --layout tn --shapes 768x3072x32768,3072x768x32768,768x768x32768,2304x768x32768 > gpurun_out/gab_tn.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python3 bench.py --model bert --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1
