// Forced GEMM tile configurations (gemm_force_cfg): the table tools/gemm_sweep.py and
// tools/gemm_ab.py measure the heuristic in gemm.hip against.  Split over three translation units
// (gemm_forced*.hip) so the instantiations compile in parallel.
#include "dtg/gemm_launch.cuh"
#include "lab.h"

namespace dtg {

bool gemm_launch_forced_c(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt) {
#define DTG_CFG_CASE(n, ...)                                                                          \
  case n:                                                                                            \
    launch_exact<__VA_ARGS__>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt); \
    return true;
  switch (cfg) {
    DTG_CFG_CASE(19, Cfg<64, 256, 3, 4, 32>)
    DTG_CFG_CASE(20, Cfg<256, 64, 3, 4, 32>)
    DTG_CFG_CASE(21, Cfg<64, 256, 2, 4, 32>)
    DTG_CFG_CASE(22, Cfg<256, 64, 2, 4, 32>)
    DTG_CFG_CASE(23, Cfg<128, 128, 5, 4, 32>)
    DTG_CFG_CASE(24, Cfg<64, 256, 4, 4, 32>)
    DTG_CFG_CASE(25, Cfg<128, 128, 1, 4, 64, true>)
    DTG_CFG_CASE(26, Cfg<64, 256, 1, 4, 64, true>)
    DTG_CFG_CASE(27, Cfg<256, 64, 1, 4, 64, true>)
    DTG_CFG_CASE(28, Cfg<256, 128, 1, 8>)
    DTG_CFG_CASE(29, Cfg<128, 256, 1, 8>)
    DTG_CFG_CASE(30, Cfg<256, 128, 1, 8, 64, true>)
    DTG_CFG_CASE(31, Cfg<128, 256, 1, 8, 64, true>)
    default: return false;
  }
#undef DTG_CFG_CASE
}

}  // namespace dtg
