// Forced GEMM tile configurations (gemm_force_cfg): the table tools/gemm_sweep.py and
// tools/gemm_ab.py measure the heuristic in gemm.hip against.  Split over three translation units
// (gemm_forced*.hip) so the instantiations compile in parallel.
#include "dtg/gemm_launch.cuh"
#include "lab.h"

namespace dtg {

bool gemm_launch_forced_b(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt) {
#define DTG_CFG_CASE(n, ...)                                                                          \
  case n:                                                                                            \
    launch_exact<__VA_ARGS__>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt); \
    return true;
  switch (cfg) {
    DTG_CFG_CASE(10, Cfg<128, 256, 2, 8>)
    DTG_CFG_CASE(11, Cfg<128, 256, 3, 8>)
    DTG_CFG_CASE(12, Cfg<64, 256, 2>)
    DTG_CFG_CASE(13, Cfg<64, 256, 3>)
    DTG_CFG_CASE(14, Cfg<256, 64, 1>)
    DTG_CFG_CASE(15, Cfg<64, 256, 1>)
    DTG_CFG_CASE(16, Cfg<128, 128, 2, 4, 32>)
    DTG_CFG_CASE(17, Cfg<128, 128, 3, 4, 32>)
    DTG_CFG_CASE(18, Cfg<128, 128, 4, 4, 32>)
    default: return false;
  }
#undef DTG_CFG_CASE
}

}  // namespace dtg
