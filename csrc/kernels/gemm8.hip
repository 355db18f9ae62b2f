// 256x256 bf16 GEMM, 8 waves, 8-phase staggered schedule (cdna_hip_programming.md §5 "The 256² 8-phase
// template", T3+T4+T5), for the large GEMMs of ResNet-50 (1x1 convs at batch 256) and BERT.
//
// Wave w = (wr = w>>2, wc = w&3) owns the 128x64 output block rows [128 wr, +128), cols [64 wc, +64)
// = acc[8][4] (16x16 MFMA tiles).  A K-tile (BK = 64) is split into four LDS "halves", each 128 rows x
// 64 k = 16 KB, arranged so that every phase reads exactly one A half and one B half:
//     A_h = rows {128 wr + 64 h + [0, 64)}  (the h-th 64-row quarter of both wave-row slabs)
//     B_h = cols {64 wc + 32 h + [0, 32)}   (the h-th 32-col half of every wave's column block)
// Phases per K-tile compute one (mq, nq) quadrant (64x32 per wave, 16 MFMA) in the order
//     P0 (0,0): ds_read A_0, B_0     P1 (1,0): ds_read A_1     P2 (1,1): ds_read B_1     P3 (0,1): -
// (A_0's fragments stay in registers until P3), so every half of buffer u&1 is read in exactly one
// phase (A_0, B_0 @P0, A_1 @P1, B_1 @P2) and is re-staged (LDS-DMA, 2 glds per thread per half) for
// a later tile at least two phases after that read:
//     tile u issues  P0: A_1(u+1)  P1: B_1(u+1)  P2: A_0(u+2)  P3: B_0(u+2)
// giving every half >= 3 phases of DMA flight.  Each phase = { ds_read; glds; s_barrier; lgkmcnt(0);
// setprio 1; 16 MFMA; setprio 0; counted vmcnt; s_barrier }.  Waves 4-7 run one barrier behind
// waves 0-3 (one extra s_barrier up front), so on every SIMD one wave is in its MFMA section while
// the other is in its load section.  With that stagger a DMA is visible to every reader two phases
// after the issuing waves' vmcnt, and a half can be overwritten two phases after its last read: the
// waits at the end of P0 / P2 / P3 retire exactly the halves read two phases later and leave the
// three newest halves (vmcnt 6) in flight; the tail counts are exact.
// All LDS is one __shared__ array (a second LDS object can make hipcc drain vmcnt each step).
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"
#include <type_traits>

namespace dtg {
using namespace gemm;

namespace g8 {

constexpr int BM = 256, BN = 256, NTH = 512, HALF = 16384, BUF = 4 * HALF;  // A0 A1 B0 B1 per buffer
constexpr int LDS = 2 * BUF;                                                  // 128 KB

// Stage half h of a KC operand: LDS [128 rows][64 k] (frag_kc layout), LDS row lr -> operand row
//   A: rc0 + 128 (lr / 64) + 64 h + lr % 64         B: rc0 + 64 (lr / 32) + 32 h + lr % 32
template <bool IS_A, class Src>
__device__ __forceinline__ void stage_half_kc(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = (wave * 2 + i) * 8;
    const int lr = r0 + (lane >> 3);
    const int row = IS_A ? rc0 + 128 * (lr >> 6) + 64 * h + (lr & 63) : rc0 + 64 * (lr >> 5) + 32 * h + (lr & 31);
    const int cl = lane & 7, c = cl ^ (lr & 7);
    __builtin_amdgcn_global_load_lds(src.chunk(row, k0 + c * 8), (lds_void*)(t + r0 * 128), 16, 0, 0);
  }
}

// Stage half h of an MC operand: LDS [64 k][128 cols] (frag_mc<128> layout), LDS col lc -> operand col
// with the same mapping as above
template <bool IS_A, class Src>
__device__ __forceinline__ void stage_half_mc(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
  constexpr int CH = 16, KPI = 4;  // 16 chunks per 256-B k-row, 4 k-rows per wave-instruction
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kr0 = (wave * 2 + i) * KPI;
    const int kr = kr0 + lane / CH;
    const int cl = lane % CH, c = cl ^ mc_swz<CH>(kr);
    const int lc = c * 8;  // first of the 8 columns of this chunk (a chunk never straddles a run)
    const int col = IS_A ? rc0 + 128 * (lc >> 6) + 64 * h + (lc & 63) : rc0 + 64 * (lc >> 5) + 32 * h + (lc & 31);
    __builtin_amdgcn_global_load_lds(src.chunk(k0 + kr, col), (lds_void*)(t + kr0 * 256), 16, 0, 0);
  }
}

template <bool KC, bool IS_A, class Src>
__device__ __forceinline__ void stage_half(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
  if constexpr (KC) stage_half_kc<IS_A>(src, t, rc0, h, k0, wave, lane);
  else stage_half_mc<IS_A>(src, t, rc0, h, k0, wave, lane);
}

template <bool KC>
__device__ __forceinline__ v8bf hfrag(const lds_char* t, int r0, int ks, int lane) {
  if constexpr (KC) return frag_kc(t, r0, ks, lane);
  else return frag_mc<128>(t, r0, ks, lane);
}

}  // namespace g8

template <bool AKC, bool BKC, class SA, class SB>
__global__ void __launch_bounds__(512, 1) gemm8_kernel(SA sa, SB sb, int M, int N, int K, int tiles_n, int split_k,
                                                       int k_per_split, Epi e, float* __restrict__ ws) {
  using namespace g8;
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BN;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half slots: buffer u&1, A_h at h*HALF, B_h at (2+h)*HALF
  auto A_h = [&](int u, int h) { return smem + (u & 1) * BUF + h * HALF; };
  auto B_h = [&](int u, int h) { return smem + (u & 1) * BUF + (2 + h) * HALF; };
  auto stA = [&](int u, int h) { g8::stage_half<AKC, true>(sa, A_h(u, h), bm0, h, kbeg + u * BK, wave, lane); };
  auto stB = [&](int u, int h) { g8::stage_half<BKC, false>(sb, B_h(u, h), bn0, h, kbeg + u * BK, wave, lane); };

  if (nk > 0) {
    // prologue: tile 0 plus the two tile-1 halves steady state issues two phases before tile 0
    // starts; retire A_0, B_0, A_1 of tile 0 (needed by P0/P1), keep 3 halves in flight
    stA(0, 0);
    stB(0, 0);
    stA(0, 1);
    stB(0, 1);
    if (nk > 1) {
      stA(1, 0);
      stB(1, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // raw barrier: __syncthreads would drain the in-flight DMA
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 run one barrier behind

    // A_0 fragments stay in registers from P0 to P3 (a0), A_1 from P1 to P2 (a1), so every half is
    // read from LDS in exactly one phase and can be re-staged early (>= 3 phases of DMA flight)
    v8bf a0[4][2], a1[4][2], b[2][2];
    for (int u = 0; u < nk; ++u) {
      const bool n1 = u + 1 < nk, n2 = u + 2 < nk;
      // ---- P0: quadrant (0,0): read A_0, B_0; issue A_1(u+1); retire B_1(u)
      {
        const lds_char* ta = A_h(u, 0);
        const lds_char* tb = B_h(u, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a0[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::hfrag<BKC>(tb, wc * 32 + j * 16, ks, lane);
        if (n1) stA(u + 1, 1);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i][ks], b[j][ks], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      // ---- P1: quadrant (1,0): read A_1; issue B_1(u+1)
      {
        const lds_char* ta = A_h(u, 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a1[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
        if (n1) stB(u + 1, 1);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i][ks], b[j][ks], acc[4 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
      }
      // ---- P2: quadrant (1,1): read B_1; issue A_0(u+2); retire A_0(u+1), B_0(u+1)
      {
        const lds_char* tb = B_h(u, 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::hfrag<BKC>(tb, wc * 32 + j * 16, ks, lane);
        if (n2) stA(u + 2, 0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[4 + i][2 + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i][ks], b[j][ks], acc[4 + i][2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      // ---- P3: quadrant (0,1): registers only (a0, B_1); issue B_0(u+2); retire A_1(u+1)
      {
        if (n2) stB(u + 2, 0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i][ks], b[j][ks], acc[i][2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: 8 passes of 32 rows through LDS (fp32, padded rows), 16-B stores
  constexpr int LD = BN + 4, R = 32;
  lds_float* stg = reinterpret_cast<lds_float*>(smem);
  const bool slab = split_k > 1;
  float* slab_p = ws + (long long)blockIdx.y * M * N;
#pragma unroll
  for (int pass = 0; pass < BM / R; ++pass) {  // fully unrolled: acc is indexed with constants only
    if (wr == pass / 4) {
      const int ib = (pass % 4) * 2;  // the two 16-row m-tiles of this pass
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(ii * 16 + (lane >> 4) * 4 + r) * LD + wc * 64 + j * 16 + (lane & 15)] = acc[ib + ii][j][r];
    }
    __syncthreads();
    constexpr int CPR = BN / 8;
    for (int idx = tid; idx < R * CPR; idx += NTH) {
      const int rr = idx / CPR, cg = idx % CPR;
      const int m = bm0 + pass * R + rr, n = bn0 + cg * 8;
      if (m < M && n < N) {
        float v[8];
        const lds_float* s = stg + rr * LD + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = s[k];
        if (slab) {
          float* p = slab_p + (long long)m * N + n;
          if ((N & 3) == 0 && n + 8 <= N) store8_f32(p, v);
          else
            for (int k = 0; k < 8 && n + k < N; ++k) p[k] = v[k];
        } else {
          epi_store8(e, N, m, n, v);
        }
      }
    }
    __syncthreads();
  }
}

// ---- host ----------------------------------------------------------------------------------------
template <bool AK, bool BK_, bool GUARD>
static void launch8(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K, int split_k,
                    int kps, const Epi& e, float* ws, hipStream_t st) {
  using SA = std::conditional_t<AK, DenseKC<GUARD>, DenseMC<GUARD>>;
  using SB = std::conditional_t<BK_, DenseKC<GUARD>, DenseMC<GUARD>>;
  SA sa{A, lda, M, K};
  SB sb{B, ldb, N, K};
  const int tiles_m = (M + g8::BM - 1) / g8::BM, tiles_n = (N + g8::BN - 1) / g8::BN;
  dim3 grid(tiles_m * tiles_n, split_k);
  hipLaunchKernelGGL((gemm8_kernel<AK, BK_, SA, SB>), grid, dim3(g8::NTH), 0, st, sa, sb, M, N, K, tiles_n, split_k,
                     kps, e, ws); DTG_LAUNCH_CHECK();
}

template <bool GUARD>
static void launch8_layout(int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M,
                           int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st) {
  if (a_kc && b_kc) launch8<true, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else if (a_kc) launch8<true, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else if (b_kc) launch8<false, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else launch8<false, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
}

void gemm8_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, const Epi& e,
                int M, int N, int K, int split_k, int kps, float* ws, hipStream_t st) {
  const bool full = (M % g8::BM == 0) && (N % g8::BN == 0) && (K % BK == 0);
  if (full) launch8_layout<false>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else launch8_layout<true>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  if (split_k > 1) gemm_splitk_reduce(ws, split_k, M, N, e, st);
}

}  // namespace dtg
