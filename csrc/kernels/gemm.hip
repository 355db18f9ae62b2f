// Dense bf16 GEMM on MFMA (see dtg/mfma_gemm.cuh for the core):
//   C = act( alpha * op(A) * op(B) + beta * C + bias )
// A is [M,K] (a_kc=1, lda = row stride) or stored K-major [K,M] (a_kc=0);
// B is [N,K] (b_kc=1: nn.Linear weight layout) or [K,N] (b_kc=0).
// Output fp32 or bf16.  split_k > 1 writes fp32 partial slabs to a workspace and a second pass
// reduces them and applies the epilogue (deterministic; no atomics) -- used for weight-gradient
// GEMMs whose K (= batch*H*W) is huge and whose output is a few tiles.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include <type_traits>

namespace dtg {
using namespace gemm;

struct Epi {
  void* C;
  long long ldc;
  int c_bf16;
  float alpha, beta;
  const float* bias;  // per column (N), may be null
  int act;            // 0 none, 1 relu, 2 gelu(tanh)
};

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) {
    const float u = 0.7978845608028654f * (v + 0.044715f * v * v * v);
    return 0.5f * v * (1.f + tanhf(u));
  }
  return v;
}

__device__ __forceinline__ void epi_store(const Epi& e, int M, int N, int m, int n, float v) {
  if (m >= M || n >= N) return;
  v *= e.alpha;
  const long long off = (long long)m * e.ldc + n;
  if (e.beta != 0.f) v += e.beta * (e.c_bf16 ? bf2f(((const bf16_t*)e.C)[off]) : ((const float*)e.C)[off]);
  if (e.bias) v += e.bias[n];
  v = apply_act(v, e.act);
  if (e.c_bf16) ((bf16_t*)e.C)[off] = f2bf(v);
  else ((float*)e.C)[off] = v;
}

template <bool AKC, bool BKC, class SA, class SB>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(SA sa, SB sb, int M, int N, int K, int tiles_n, int split_k,
                                                     int k_per_split, Epi e, float* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  const int ntiles = gridDim.x;  // (tiles_m * tiles_n) per split
  const int t = xcd_remap(blockIdx.x, ntiles);
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int bm0 = tm * BM, bn0 = tn * BN;
  const int split = blockIdx.y;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop<AKC, BKC>(sa, sb, smem, bm0, bn0, kbeg, kend, acc);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  if (split_k > 1) {
    float* slab = ws + (long long)split * M * N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = bm0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
          const int n = bn0 + wn * 64 + j * 16 + (lane & 15);
          if (m < M && n < N) slab[(long long)m * N + n] = acc[i][j][r];
        }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = bm0 + wm * 64 + i * 16 + (lane >> 4) * 4 + r;
        const int n = bn0 + wn * 64 + j * 16 + (lane & 15);
        epi_store(e, M, N, m, n, acc[i][j][r]);
      }
}

__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int split_k, int M, int N,
                                                            Epi e) {
  const long long total = (long long)M * N;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < split_k; ++k) s += ws[(long long)k * total + i];
    epi_store(e, M, N, (int)(i / N), (int)(i % N), s);
  }
}

long long gemm_workspace_floats(int M, int N, int K, int split_k) {
  return split_k > 1 ? (long long)split_k * M * N : 0;
}

int gemm_pick_split(int M, int N, int K) {
  const long long tiles = (long long)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int s = 1;
  // aim for >= ~512 workgroups (2 per CU over 256 CUs) while keeping >= 512 K per split
  while (tiles * s < 512 && (long long)K / (s * 2) >= 512 && s < 64) s *= 2;
  return s;
}

void gemm_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, void* C,
               long long ldc, int c_bf16, int M, int N, int K, float alpha, float beta, const float* bias, int act,
               int split_k, float* ws, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  if (split_k < 1) split_k = 1;
  int kps = (K + split_k - 1) / split_k;
  kps = (kps + BK - 1) / BK * BK;
  split_k = (K + kps - 1) / kps;
  if (split_k < 1) split_k = 1;
  Epi e{C, ldc, c_bf16, alpha, beta, bias, act};
  dim3 grid(tiles_m * tiles_n, split_k);
  const size_t lds = 0;
#define DTG_GEMM_LAUNCH(AK, BK_)                                                                              \
  do {                                                                                                        \
    using SA = std::conditional_t<AK, DenseKC, DenseMC>;                                                      \
    using SB = std::conditional_t<BK_, DenseKC, DenseMC>;                                                     \
    SA sa{A, lda, M, K};                                                                                      \
    SB sb{B, ldb, N, K};                                                                                      \
    hipLaunchKernelGGL((gemm_kernel<AK, BK_, SA, SB>), grid, dim3(NT), lds, st, sa, sb, M, N, K, tiles_n,    \
                       split_k, kps, e, ws);                                                                  \
  } while (0)
  if (a_kc && b_kc) DTG_GEMM_LAUNCH(true, true);
  else if (a_kc && !b_kc) DTG_GEMM_LAUNCH(true, false);
  else if (!a_kc && b_kc) DTG_GEMM_LAUNCH(false, true);
  else DTG_GEMM_LAUNCH(false, false);
#undef DTG_GEMM_LAUNCH
  if (split_k > 1) {
    const long long total = (long long)M * N;
    splitk_reduce_kernel<<<grid_for(total, 256, 2048), 256, 0, st>>>(ws, split_k, M, N, e);
  }
}

}  // namespace dtg
