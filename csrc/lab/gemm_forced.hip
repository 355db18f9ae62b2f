// Forced GEMM tile configurations (gemm_force_cfg): the table tools/gemm_sweep.py and
// tools/gemm_ab.py measure the heuristic in gemm.hip against.  Split over three translation units
// (gemm_forced*.hip) so the instantiations compile in parallel.
#include "dtg/gemm_launch.cuh"
#include "lab.h"

namespace dtg {

bool gemm_launch_forced_a(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt);
bool gemm_launch_forced_b(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt);
bool gemm_launch_forced_c(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt);

bool gemm_launch_forced(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B,
                         long long ldb, int M, int N, int K, int split_k, int kps, const Epi& e, float* ws,
                         hipStream_t st, const GemmBatch& bt) {
  return gemm_launch_forced_a(cfg, a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt) ||
         gemm_launch_forced_b(cfg, a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt) ||
         gemm_launch_forced_c(cfg, a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
}

}  // namespace dtg
