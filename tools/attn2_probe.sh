set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/attn2
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -m gpu > gpurun_out/attn2/test.log 2>&1 &&
timeout -k 10 120 python tools/bench_attention.py --B 256 --p 0.0 > gpurun_out/attn2/p0.log 2>&1 &&
timeout -k 10 120 python tools/bench_attention.py --B 256 --p 0.1 > gpurun_out/attn2/p1.log 2>&1 &&
rm -f gpurun_out/ab.log && AB_SCRIPT=tools/ab_tree.py timeout -k 10 900 bash tools/ab_bench.sh 3 "DTG_AB_TREE=.ab_old" "DTG_AB_TREE=." -- --model bert --steps 20 --warmup 5
