// One GEMM through a forced tile configuration (lab extension): the entry point of tools/gemm_ab.py,
// gemm_sweep.py, epi_gemm_ab.py and op_bench.py, which time the production heuristic (gemm.hip) against the
// kernels and tiles it does not pick.  Same operand conventions and split-K rounding as gemm_bf16.
#include "dtg/gemm_launch.cuh"
#include "lab.h"

namespace dtg {

bool gemm_lab_cfg(int cfg, const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, void* C,
                  long long ldc, int c_bf16, int M, int N, int K, float alpha, float beta, const float* bias, int act,
                  int split_k, float* ws, hipStream_t st, void* aux, int aux_mode) {
  if (M <= 0 || N <= 0) return true;
  if (split_k < 1) split_k = 1;
  int kps = (K + split_k - 1) / split_k;
  kps = (kps + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  split_k = (K + kps - 1) / kps;
  if (split_k < 1) split_k = 1;
  Epi e{C, ldc, c_bf16, alpha, beta, bias, act, aux, aux_mode};
  if (cfg >= 96 && cfg <= 98) return split_k == 1 && gemm8p_bf16(A, lda, a_kc, B, ldb, b_kc, e, M, N, K, st, 98 - cfg);
  if (cfg == 99) {
    gemm8_bf16(A, lda, a_kc, B, ldb, b_kc, e, M, N, K, split_k, kps, ws, st);
    return true;
  }
  return gemm_launch_forced(cfg, a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, GemmBatch());
}

}  // namespace dtg
