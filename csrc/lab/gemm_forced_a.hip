// Forced GEMM tile configurations (gemm_force_cfg): the table tools/gemm_sweep.py and
// tools/gemm_ab.py measure the heuristic in gemm.hip against.  Split over three translation units
// (gemm_forced*.hip) so the instantiations compile in parallel.
#include "dtg/gemm_launch.cuh"
#include "lab.h"

namespace dtg {

bool gemm_launch_forced_a(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt) {
#define DTG_CFG_CASE(n, ...)                                                                          \
  case n:                                                                                            \
    launch_exact<__VA_ARGS__>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt); \
    return true;
  switch (cfg) {
    DTG_CFG_CASE(1, Cfg<128, 128, 1>)
    DTG_CFG_CASE(2, Cfg<128, 128, 2>)
    DTG_CFG_CASE(3, Cfg<128, 128, 3>)
    DTG_CFG_CASE(4, Cfg<128, 128, 4>)
    DTG_CFG_CASE(5, Cfg<256, 64, 2>)
    DTG_CFG_CASE(6, Cfg<256, 64, 3>)
    DTG_CFG_CASE(7, Cfg<256, 64, 4>)
    DTG_CFG_CASE(8, Cfg<256, 128, 3, 8>)
    DTG_CFG_CASE(9, Cfg<256, 128, 2, 8>)
    default: return false;
  }
#undef DTG_CFG_CASE
}

}  // namespace dtg
