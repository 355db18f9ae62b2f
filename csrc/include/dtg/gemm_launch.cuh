// MFMA GEMM kernel template and its launchers, shared by gemm.hip (heuristic dispatch) and
// gemm_forced.hip (the forced-configuration table of tools/gemm_sweep.py), so the two compile in parallel.
#pragma once
#include <type_traits>
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"
#include "dtg/bn_epi.cuh"

namespace dtg {
using namespace gemm;

template <class CF, bool AKC, bool BKC, class SA, class SB, int BNMODE = 0, bool FAST = false, bool BNPF = false>
__global__ void __launch_bounds__(CF::NTH, CF::NW == 4 ? 2 : 1) gemm_kernel(SA sa, SB sb, int M, int N, int K, int tiles_n, int split_k,
                                                     int k_per_split, Epi e, float* __restrict__ ws, GemmBatch bt,
                                                     BnEpi bn) {
  __shared__ __attribute__((aligned(16))) char smem_raw[CF::LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  if (bt.count > 1) {  // batched problem z: offset the operands (element strides)
    const int zb = blockIdx.z / bt.nh, zh = blockIdx.z % bt.nh;
    sa.p += zb * bt.sa_b + zh * bt.sa_h;
    sb.p += zb * bt.sb_b + zh * bt.sb_h;
    const long long co = zb * bt.sc_b + zh * bt.sc_h;
    e.C = (char*)e.C + co * (e.c_bf16 ? 2 : 4);
    if (e.aux) e.aux = (char*)e.aux + co * 2;
  }
  const int ntiles = gridDim.x;  // tiles per split
  // XCD-aware over the whole (tile, split) grid: the hardware deals linear workgroup ids round-robin
  // to the 8 XCDs, so remapping blockIdx.x alone would scatter the tiles of one K-split (which share
  // their A/B K-slabs) over all 8 L2s.  Remapped, consecutive (split, tile) work ids -- all tiles of a
  // split -- land on one XCD and re-read the slabs from its L2.
  int t, split;
  if (gridDim.y > 1) {
    const int w = xcd_remap(blockIdx.x + blockIdx.y * ntiles, ntiles * gridDim.y);
    split = w / ntiles;
    t = w - split * ntiles;
  } else {
    t = xcd_remap(blockIdx.x, ntiles);
    split = 0;
  }
  const int tm = t / tiles_n, tn = t % tiles_n;
  const int bm0 = tm * CF::BM, bn0 = tn * CF::BN;
  const int kbeg = split * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop<CF, AKC, BKC>(sa, sb, smem, bm0, bn0, kbeg, kend, acc);
  if constexpr (BNMODE != 0) {  // (no split-K, no batching: gemm_bf16_bn)
    // one tile per workgroup, the column statistics live only in the epilogue.  (Several M tiles per
    // workgroup, statistics carried across their main loops, ran ResNet-50 3-4 % slower: the gemm bn3
    // kernels 4.8 -> 6.2 ms per step, profiles/r02_bn_tiles and profiles/r02_bn_revert.)
    epilogue_bn<CF, BNMODE, RowId, BNPF>(smem, acc, bm0, bn0, M, N, e, bn, t, RowId());
    return;
  }
  if (split_k > 1) {
    float* slab = ws + (long long)split * M * N;
    const bool vec = (N & 3) == 0;
    epilogue_staged<CF>(smem, acc, bm0, bn0, M, N, [&](int m, int n, float (&v)[8]) {
      float* p = slab + (long long)m * N + n;
      if (vec && n + 8 <= N) store8_f32(p, v);
      else
        for (int k = 0; k < 8 && n + k < N; ++k) p[k] = v[k];
    });
    return;
  }
  if constexpr (FAST) {  // bf16, aligned (fast_epi() checked): no per-group / per-element switches
    constexpr bool FULL = !SA::kGuard && !SB::kGuard;
    if (!e.bias && e.act == 0 && e.aux_mode == 0) {
      auto op = [&](int m, int n, float (&v)[8]) { epi_store8_fast(e, m, n, v); };
      epilogue_staged<CF, decltype(op), FULL>(smem, acc, bm0, bn0, M, N, op);
    } else {
      // a thread's 8-column group is the same in every pass of epilogue_staged: its bias is loaded once
      static_assert(CF::NTH % (CF::BN / 8) == 0, "fixed column group per thread");
      float pb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int nb = bn0 + (int)(threadIdx.x % (CF::BN / 8)) * 8;
      if (e.bias && nb < N) load8_f32(e.bias + nb, pb);
      auto op = [&](int m, int n, float (&v)[8]) { epi_store8_fast_act<true>(e, m, n, v, pb); };
      epilogue_staged<CF, decltype(op), FULL>(smem, acc, bm0, bn0, M, N, op);
    }
  } else {
    epilogue_staged<CF>(smem, acc, bm0, bn0, M, N, [&](int m, int n, float (&v)[8]) { epi_store8(e, N, m, n, v); });
  }
}

// epilogue specialisation: bf16 output (and aux), 16-B aligned 8-column groups
inline bool fast_epi(const Epi& e, int N) {
  return e.c_bf16 && (e.ldc % 8) == 0 && (N % 8) == 0 && ((uintptr_t)e.C % 16) == 0 &&
         ((uintptr_t)e.bias % 16) == 0 && ((uintptr_t)e.aux % 16) == 0;
}

template <class CF, bool AK, bool BK_, bool GUARD>
inline void launch(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K, int split_k,
                   int kps, const Epi& e, float* ws, hipStream_t st, const GemmBatch& bt) {
  using SA = std::conditional_t<AK, DenseKC<GUARD>, DenseMC<GUARD>>;
  using SB = std::conditional_t<BK_, DenseKC<GUARD>, DenseMC<GUARD>>;
  SA sa{A, lda, M, K};
  SB sb{B, ldb, N, K};
  const int tiles_m = (M + CF::BM - 1) / CF::BM, tiles_n = (N + CF::BN - 1) / CF::BN;
  dim3 grid(tiles_m * tiles_n, split_k, bt.count);
  if constexpr (AK) {  // (K-contiguous A = forward / dgrad GEMMs; weight gradients go through split-K)
    if (split_k == 1 && fast_epi(e, N) && (bt.count == 1 || ((bt.sc_b | bt.sc_h) & 7) == 0)) {
      hipLaunchKernelGGL((gemm_kernel<CF, AK, BK_, SA, SB, 0, true>), grid, dim3(CF::NTH), 0, st, sa, sb, M, N, K,
                         tiles_n, split_k, kps, e, ws, bt, BnEpi()); DTG_LAUNCH_CHECK();
      if (split_k > 1) gemm_splitk_reduce(ws, split_k, M, N, e, st);
      return;
    }
  }
  hipLaunchKernelGGL((gemm_kernel<CF, AK, BK_, SA, SB>), grid, dim3(CF::NTH), 0, st, sa, sb, M, N, K, tiles_n, split_k,
                       kps, e, ws, bt, BnEpi()); DTG_LAUNCH_CHECK();
  if (split_k > 1) gemm_splitk_reduce(ws, split_k, M, N, e, st);
}

template <class CF, bool GUARD>
inline void launch_layout(int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M,
                          int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st,
                          const GemmBatch& bt) {
  if (a_kc && b_kc) launch<CF, true, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  else if (a_kc) launch<CF, true, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  else if (b_kc) launch<CF, false, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  else launch<CF, false, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
}

template <class CF>
inline void launch_exact(int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M,
                         int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st,
                         const GemmBatch& bt) {
  const bool full = (M % CF::BM == 0) && (N % CF::BN == 0) && (K % BK == 0);
  if (full) launch_layout<CF, false>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  else launch_layout<CF, true>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
}

}  // namespace dtg
