// Dense bf16 GEMM on MFMA (see dtg/mfma_gemm.cuh for the core):
//   C = act( alpha * op(A) * op(B) + beta * C + bias )
// A is [M,K] (a_kc=1, lda = row stride) or stored K-major [K,M] (a_kc=0);
// B is [N,K] (b_kc=1: nn.Linear weight layout) or [K,N] (b_kc=0).
// Output fp32 or bf16, written through an LDS-staged epilogue as 16-byte vectors.
// split_k > 1 writes fp32 partial slabs to a workspace and a second pass reduces them and applies
// the epilogue (deterministic; no atomics) -- used for weight-gradient GEMMs whose K
// (= batch*H*W) is huge and whose output is a handful of tiles.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/gemm_launch.cuh"
#include <stdlib.h>
#include <type_traits>

namespace dtg {
using namespace gemm;


// Split-K reduction: a thread owns 8 consecutive outputs and sums their split_k partials; the
// split loop is unrolled by 4 so 4 x 32 B of loads are in flight per thread (the reduce is a pure
// stream: split_k * M * N * 4 bytes in, the epilogue's bytes out).
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const float* __restrict__ ws, int split_k, int M, int N,
                                                            Epi e) {
  const int cgs = (N + 7) / 8;
  const long long total = (long long)M * cgs;
  const long long plane = (long long)M * N;
  const bool vec = (N & 7) == 0;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int m = (int)(i / cgs), n = (int)(i % cgs) * 8;
    const long long off = (long long)m * N + n;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (vec) {
      int k = 0;
      for (; k + 4 <= split_k; k += 4) {
        float v0[8], v1[8], v2[8], v3[8];
        load8_f32(ws + (k + 0) * plane + off, v0);
        load8_f32(ws + (k + 1) * plane + off, v1);
        load8_f32(ws + (k + 2) * plane + off, v2);
        load8_f32(ws + (k + 3) * plane + off, v3);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += (v0[j] + v1[j]) + (v2[j] + v3[j]);
      }
      for (; k < split_k; ++k) {
        float v[8];
        load8_f32(ws + k * plane + off, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] += v[j];
      }
    } else {
      for (int k = 0; k < split_k; ++k)
        for (int j = 0; j < 8 && n + j < N; ++j) s[j] += ws[k * plane + off + j];
    }
    epi_store8(e, N, m, n, s);
  }
}

// Large split counts (conv wgrad over N*H*W can split 64-256 ways): a block owns 256 consecutive
// outputs (32 lanes x 8 floats) and its 8 lane-groups stride over the splits; partial sums meet in
// LDS.  Needs (M*N) % 8 == 0, N % 8 == 0.
__global__ void __launch_bounds__(256) splitk_reduce_par_kernel(const float* __restrict__ ws, int split_k, int M,
                                                                int N, Epi e) {
  __shared__ float red[8][256 + 8];
  const long long plane = (long long)M * N;
  const long long base = (long long)blockIdx.x * 256;
  const int lane = threadIdx.x & 31, grp = threadIdx.x >> 5;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (base + lane * 8 < plane) {
    for (int k = grp; k < split_k; k += 8) {
      float v[8];
      load8_f32(ws + k * plane + base + lane * 8, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += v[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) red[grp][lane * 8 + j] = s[j];
  __syncthreads();
  if (grp == 0 && base + lane * 8 < plane) {
#pragma unroll
    for (int g = 1; g < 8; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += red[g][lane * 8 + j];
    const long long i = base + lane * 8;
    epi_store8(e, N, (int)(i / N), (int)(i % N), s);
  }
}

long long gemm_workspace_floats(int M, int N, int K, int split_k) {
  return split_k > 1 ? (long long)split_k * M * N : 0;
}

static bool skinny(int N) { return N <= 64; }

static bool short_m(int M, int N) { return M <= 64 && N >= 128; }

int gemm_pick_split(int M, int N, int K, int a_kc, int target_wgs) {
  const int BMv = skinny(N) ? 256 : (short_m(M, N) ? 64 : 128), BNv = skinny(N) ? 64 : (short_m(M, N) ? 256 : 128);
  const long long tiles = (long long)((M + BMv - 1) / BMv) * ((N + BNv - 1) / BNv);
  // forward / data-gradient GEMMs (K-contiguous A) with >= 128 tiles: the fp32 partial round trip
  // costs more than the idle CUs do (BERT 8192x768x3072: 47 us unsplit, 56 us split 2;
  // profiles/r01_rp/sweep_bert.log)
  if (a_kc && tiles >= 128) {
    // ... except a long reduction over a short grid (BERT's MLM decoder dgrad 5120x768x30528: 240
    // tiles, 834 us unsplit on the 8-phase kernel, 286 us split 2 -- profiles/r02_gemm): split until the
    // grid is ~1.5 workgroups per CU while each split keeps >= 4096 of K
    int s = 1;
    if (K >= 8192)
      while (tiles * s < 384 && (long long)K / (s * 2) >= 4096) s *= 2;
    return s;
  }
  int s = 1;
  // aim for >= ~512 workgroups (or the caller's target) while keeping >= 1024 K (16 K-steps) per split
  const long long target = target_wgs > 0 ? target_wgs : 512;
  while (tiles * s < target && (long long)K / (s * 2) >= 1024 && s < 256) s *= 2;
  return s;
}

template <int BM_, int BN_>
static void launch_cfg(int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M,
                       int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st,
                       const GemmBatch& bt) {
  // full tiles -> no bounds checks in the address computation
  const bool full = (M % BM_ == 0) && (N % BN_ == 0) && (K % BK == 0);
  // short K per block -> single-stage ring (half the LDS, 2x the resident workgroups)
  const bool short_k = kps <= 2 * BK;
  if (full) {
    if (short_k) launch_layout<Cfg<BM_, BN_, 1>, false>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
    else launch_layout<Cfg<BM_, BN_, 2>, false>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  } else {
    if (short_k) launch_layout<Cfg<BM_, BN_, 1>, true>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
    else launch_layout<Cfg<BM_, BN_, 2>, true>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  }
}

// (The 256x256 8-wave 8-phase kernel and the forced-configuration table that measured every tile against this
// heuristic -- BERT's MLM decoder 30528x768x5120 wgrad 419 vs 289 us, 5120x768x30528 dgrad 834 vs 286 us split 2,
// profiles/r02_gemm -- live in the tools-only lab extension, csrc/lab.)

// Register pipelining pays when each workgroup has a long K loop and the problem is compute-heavy
// enough that latency, not occupancy (3 instead of 4 workgroups per CU), limits it: long K (>= 2048),
// or K >= 768 at >= 300 flop per operand byte (BERT's 8192-token GEMMs: 5-12 % faster; ResNet's
// 50176x256x1024 at 204 flop/B is 8 % slower with it).
static bool use_rp(int M, int N, int kps) {
  // ... but only while the grid is short: with more than ~2 rounds of 128x128 tiles (> 2048 at 4 per CU)
  // the fourth resident workgroup the plain single stage keeps is worth more than in-block pipelining
  // (BERT-base at 32768 tokens: 32768x3072x768 990 vs 896 TF/s, 32768x2304x768 979 vs 922; at
  // 1536 tiles the two tie or RP wins -- tools/gemm_ab.py, profiles/r02_gemm)
  if ((long long)((M + 127) / 128) * ((N + 127) / 128) > 2048) return false;
  if (kps >= 2048) return true;
  const double flop = 2.0 * M * N * kps, bytes = 2.0 * ((double)M * kps + (double)N * kps + (double)M * N);
  return kps >= 768 && flop / bytes >= 300.0;
}

void gemm_splitk_reduce(const float* ws, int split_k, int M, int N, const Epi& e, hipStream_t st) {
  if (N % 8 == 0 && split_k > 16) {
    const long long plane = (long long)M * N;
    splitk_reduce_par_kernel<<<(unsigned)((plane + 255) / 256), 256, 0, st>>>(ws, split_k, M, N, e); DTG_LAUNCH_CHECK();
  } else {
    const long long total = (long long)M * ((N + 7) / 8);
    splitk_reduce_kernel<<<grid_for(total, 256, 1 << 16), 256, 0, st>>>(ws, split_k, M, N, e); DTG_LAUNCH_CHECK();
  }
}

void gemm_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, void* C,
               long long ldc, int c_bf16, int M, int N, int K, float alpha, float beta, const float* bias, int act,
               int split_k, float* ws, hipStream_t st, const GemmBatch& bt, void* aux, int aux_mode) {
  if (M <= 0 || N <= 0) return;
  if (bt.count > 1) split_k = 1;  // batched problems are small tiles: no split-K
  if (split_k < 1) split_k = 1;
  int kps = (K + split_k - 1) / split_k;
  kps = (kps + BK - 1) / BK * BK;
  if (kps < BK) kps = BK;
  split_k = (K + kps - 1) / kps;
  if (split_k < 1) split_k = 1;
  Epi e{C, ldc, c_bf16, alpha, beta, bias, act, aux, aux_mode};
  if (split_k > 1 || !a_kc) {
    // weight gradients (MN-contiguous A, split-K over the token/pixel dimension): the single-stage
    // 128x128 ring beat every other tile and the 2-stage ring on all of them, BERT's 768x3072x8192
    // by 1.4x (profiles/r01_tiles/sweep_wgrad.json); its register-pipelined variant (next K-step's DMA
    // issued under this step's MFMAs) is another 5-8 % on all wgrad shapes but one (sweep_rp.json)
    // (round 4, measured in the ResNet-50 b1024 step and alone at 128 workgroups, tools/gemm_ab.py --layout tn,
    // profiles/r04_wgrad: a 2-4 slot LDS-DMA ring 6-18 % slower alone and 4-9 % slower in the step; the
    // 256x128 8-wave tile 28 % faster alone at equal workgroups but neutral in the step; 256x256 gemm8 tiles
    // -0.5 %: the side-stream weight gradients cost the step HBM bandwidth, not CU time)
    launch_exact<Cfg<128, 128, 1, 4, 64, true>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
    return;
  }
  if (short_m(M, N)) {  // 64-row outputs: no half-empty 128-row tiles
    launch_cfg<64, 256>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
    return;
  }
  // (the 128x256 8-wave single stage for wide outputs over a short reduction -- BERT's FFN1 forward / FFN2
  // dgrad -- won 156 vs 165 us as a plain GEMM but lost with the real GELU / aux epilogues, 8.92k vs 9.05k
  // seq/s, profiles/r02_gemm: forced configuration 29 only)
  // Tile width follows N so the streamed activation operand A is read as few times as possible:
  // 256x64 for N <= 64, 64x256 for N >= 256 with K <= 256, else 128x128 (r01_tiles sweeps).  LDS ring depth: a single stage
  // (32-40 KB: ~4 workgroups per CU hide the HBM latency across blocks) unless the grid is short
  // (< 512 tiles) and K long enough (>= 2048) that in-block prefetch pays (profiles/r01_tiles).
  const long long tiles128 = (long long)((M + 127) / 128) * ((N + 127) / 128) * split_k * bt.count;
  if (use_rp(M, N, kps)) {  // the register-pipelined single stage (sweep_rp.json, sweep_bert.log)
    launch_exact<Cfg<128, 128, 1, 4, 64, true>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  } else if (tiles128 < 512 && kps >= 2048) {
    launch_exact<Cfg<128, 128, 2>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  } else if (skinny(N)) {
    launch_exact<Cfg<256, 64, 1>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  } else if (N >= 256 && M >= 64 && kps <= 256) {
    launch_exact<Cfg<64, 256, 1>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  } else {
    launch_exact<Cfg<128, 128, 1>>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st, bt);
  }
}

// ---- BN-statistics epilogue (gemm_bf16_bn) ---------------------------------------------------------
template <class CF, int MODE, bool GUARD, bool PF>
static void launch_bn(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                      const Epi& e, const BnEpi& bn, hipStream_t st) {
  using SB = std::conditional_t<MODE == 1, DenseKC<GUARD>, DenseMC<GUARD>>;
  SB sb{B, ldb, N, K};
  const int tiles_m = (M + CF::BM - 1) / CF::BM, tiles_n = (N + CF::BN - 1) / CF::BN;
  using SA = DenseKC<GUARD>;
  SA sa{A, lda, M, K};
  hipLaunchKernelGGL((gemm_kernel<CF, true, MODE == 1, SA, SB, MODE, false, PF>), dim3(tiles_m * tiles_n, 1, 1),
                     dim3(CF::NTH), 0, st, sa, sb, M, N, K, tiles_n, 1, K, e, (float*)nullptr, GemmBatch(), bn); DTG_LAUNCH_CHECK();
}


template <class CF, int MODE>
static void launch_bn_cfg(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                          const Epi& e, const BnEpi& bn, hipStream_t st) {
  const bool full = (M % CF::BM == 0) && (N % CF::BN == 0) && (K % BK == 0);
  // prefetching backward epilogue where the epilogue's streaming dominates: wide outputs or short
  // reductions (measured per shape, profiles/r02_epi_pf; see epilogue_bn)
  if constexpr (MODE >= 2 && MODE <= 4) {
    if (N >= 512 || K <= 128) {
      if (full) launch_bn<CF, MODE, false, true>(A, lda, B, ldb, M, N, K, e, bn, st);
      else launch_bn<CF, MODE, true, true>(A, lda, B, ldb, M, N, K, e, bn, st);
      return;
    }
  }
  if (full) launch_bn<CF, MODE, false, false>(A, lda, B, ldb, M, N, K, e, bn, st);
  else launch_bn<CF, MODE, true, false>(A, lda, B, ldb, M, N, K, e, bn, st);
}

// gemm_bn_force_cfg (tools/bn_gemm_ab.py) forces the BN-epilogue GEMM tile: 1 128x128, 2 64x256, 3 128x128
// register-pipelined, 4 256x64, 5 128x256 8 waves, 6 256x128 8 waves; 0 = the heuristic below (mode 1: the streaming
// expand kernel first, gemm_expand.hip, where it applies); -1 = the heuristic without the expand kernel; -2 / -3 =
// expand kernel variants 1 / 2 (non-temporal stores / 3 workgroups per CU)
static int g_bn_gemm_cfg = 0;
void gemm_bn_force_cfg(int cfg) { g_bn_gemm_cfg = cfg; }

template <int MODE>
static void gemm_bn_dispatch(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                             const Epi& e, const BnEpi& bn, hipStream_t st) {
  switch (g_bn_gemm_cfg) {
    case 1: return launch_bn_cfg<Cfg<128, 128, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    case 2: return launch_bn_cfg<Cfg<64, 256, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    case 3: return launch_bn_cfg<Cfg<128, 128, 1, 4, 64, true>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    case 4: return launch_bn_cfg<Cfg<256, 64, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    case 5: return launch_bn_cfg<Cfg<128, 256, 1, 8>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    case 6: return launch_bn_cfg<Cfg<256, 128, 1, 8>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    default: break;
  }
  // measured per ResNet-50 shape (tools/bn_gemm_ab.py, profiles/r03_bn_gemm_tiles): the forward 1x1 expand
  // GEMMs (K <= 128, N >= 256) on 128x128 tiles (-5..7 % vs 64x256); the backward epilogues (modes 2-4) on the
  // register-pipelined 128x128 tile from K >= 256 (-4..9 %), except the 64-channel outputs (256x64 stays)
  if (MODE == 1 && K <= 128 && N >= 256 && M >= 128) {
    launch_bn_cfg<Cfg<128, 128, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    return;
  }
  if (MODE >= 2 && MODE <= 4 && K >= 256 && N >= 128) {
    launch_bn_cfg<Cfg<128, 128, 1, 4, 64, true>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
    return;
  }
  // otherwise the same tile choice as gemm_bf16's heuristic
  if (use_rp(M, N, K)) launch_bn_cfg<Cfg<128, 128, 1, 4, 64, true>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
  else if ((long long)((M + 127) / 128) * ((N + 127) / 128) < 512 && K >= 2048)
    launch_bn_cfg<Cfg<128, 128, 2>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
  else if (skinny(N)) launch_bn_cfg<Cfg<256, 64, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
  else if (N >= 256 && M >= 64 && K <= 256) launch_bn_cfg<Cfg<64, 256, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
  else launch_bn_cfg<Cfg<128, 128, 1>, MODE>(A, lda, B, ldb, M, N, K, e, bn, st);
}

// gemm_expand.hip: persistent streaming GEMM + statistics for short-K, wide-N forward 1x1 convs
bool gemm_expand_bn(const bf16_t* A, long long lda, const bf16_t* W, long long ldw, bf16_t* C, long long ldc, int M,
                    int N, int K, float* part, hipStream_t st, int variant);

void gemm_bf16_bn(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, bf16_t* C, long long ldc, int M,
                  int N, int K, float beta, const BnEpi& bn, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  Epi e{C, ldc, 1, 1.f, bn.mode == 3 ? beta : 0.f, nullptr, 0};
  if (bn.mode == 1) {
    if ((g_bn_gemm_cfg == 0 || g_bn_gemm_cfg <= -2) &&
        gemm_expand_bn(A, lda, B, ldb, C, ldc, M, N, K, bn.part, st, g_bn_gemm_cfg == 0 ? 0 : -1 - g_bn_gemm_cfg))
      return;
    gemm_bn_dispatch<1>(A, lda, B, ldb, M, N, K, e, bn, st);
  }
  else if (bn.mode == 2) gemm_bn_dispatch<2>(A, lda, B, ldb, M, N, K, e, bn, st);
  else if (bn.x2) gemm_bn_dispatch<4>(A, lda, B, ldb, M, N, K, e, bn, st);
  else gemm_bn_dispatch<3>(A, lda, B, ldb, M, N, K, e, bn, st);
}

void gemm_bf16_colsum(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, bf16_t* C, long long ldc, int M,
                      int N, int K, const float* bias, int act, void* aux, int aux_mode, float* colsum, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  Epi e{C, ldc, 1, 1.f, 0.f, bias, act, aux, aux_mode};
  BnEpi bn;
  bn.part = colsum;
  bn.mode = 5;
  gemm_bn_dispatch<5>(A, lda, B, ldb, M, N, K, e, bn, st);
}

}  // namespace dtg
