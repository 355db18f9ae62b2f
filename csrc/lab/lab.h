// Declarations of the lab-only kernels (tools-only extension dtg._lab; never linked into _C).  They reuse the
// production templates (dtg/gemm_launch.cuh) and, at load time, production symbols of _C (gemm_splitk_reduce):
// dtg.ops._native.lab() promotes _C's symbols to global scope before importing _lab.
#pragma once
#include "dtg/kernels.h"
#include "dtg/gemm_epi.cuh"
#include "lab_api.h"

namespace dtg {

// 256x256 8-wave 8-phase GEMM (gemm8.hip); same operand conventions as gemm_bf16, no batching.  Lost to the
// production 128x128 single-stage tiles on every flagship shape (profiles/r02_gemm, r04_gemm_lab).
void gemm8_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, const Epi& e,
                int M, int N, int K, int split_k, int kps, float* ws, hipStream_t st);
// persistent 256x256 8-phase GEMM (gemm8.hip gemm8p_kernel): bf16 out, K-contiguous A, epilogues plain / bias /
// bias+GELU with GELU' saved / x aux; false when the problem or epilogue does not fit (abl: timing ablations)
bool gemm8p_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, const Epi& e,
                 int M, int N, int K, hipStream_t st, int abl = 0);
// forced tile configurations (gemm_forced*.hip): the table tools/gemm_sweep.py / gemm_ab.py measure the
// production heuristic against
bool gemm_launch_forced(int cfg, int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb,
                        int M, int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st,
                        const GemmBatch& bt);
}  // namespace dtg
