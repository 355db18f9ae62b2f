cd "$GRAFT_REPO_ROOT"
for shp in "8192 768 3072" "8192 3072 768" "8192 2304 768" "8192 768 768"; do
  for c in 0 1 2 3 12 13 15 16 17 25 26 27 99; do
    echo -n "cfg $c: "; DTG_GEMM_CFG=$c ITERS=50 timeout -k 5 60 python tools/op_bench.py gemm $shp 2>/dev/null | grep "TF/s" || exit 1
  done
done
