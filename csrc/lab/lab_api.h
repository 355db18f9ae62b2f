// Host API of the lab extension (csrc/lab), includable from the g++-compiled bindings.
#pragma once
#include "dtg/kernels.h"

namespace dtg {
// one GEMM through a forced configuration (gemm_lab.hip): 96-98 the persistent 8-phase kernel (98 plain, 97 / 96
// ablations), 99 the 8-phase kernel, others the gemm_forced table; false if the configuration does not apply
bool gemm_lab_cfg(int cfg, const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, void* C,
                  long long ldc, int c_bf16, int M, int N, int K, float alpha, float beta, const float* bias, int act,
                  int split_k, float* ws, hipStream_t st, void* aux, int aux_mode);

}  // namespace dtg
