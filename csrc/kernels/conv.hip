// Implicit-GEMM 2-D convolution, NHWC bf16, on the MFMA GEMM core (dtg/mfma_gemm.cuh).
// No im2col buffer: each lane's LDS-DMA source address IS the gather (the glds global address is
// per lane), so the "im2col" matrix only ever exists as 16-byte chunks in flight.
//
//   x  [N, H, W, C]     w [K, R, S, C]  (= a channels_last [K, C, R, S] parameter)    y [N, P, Q, K]
//
//   fwd    y[(n,p,q), k]      = sum_{(r,s,c)} x[n, p*st-pad+r, q*st-pad+s, c] * w[k, r, s, c]
//          A: gather of x (K-contiguous chunks of 8 channels)          B: w, dense K-contiguous
//   dgrad  dx[(n,h,w), c]     = sum_{(r,s,k)} dy[n, h+pad-r, w+pad-s, k] * w[k, r, s, c]     (stride 1)
//          A: gather of dy (K-contiguous)                              B: gather of w, MN-contiguous
//   wgrad  dw[k, (r,s,c)]     = sum_{(n,p,q)} dy[(n,p,q), k] * x[n, p*st-pad+r, q*st-pad+s, c]
//          A: dy, dense MN-contiguous                                  B: gather of x, MN-contiguous
//          split over (n,p,q) with fp32 slabs + a reduce pass that accumulates into the flat grad.
// Requirements (checked on the host): C % 64 == 0 and K % 64 == 0 (a 64-deep K-step then stays inside
// one filter tap, so the tap is uniform per step and only the row/channel part is per lane).
// Out-of-image taps read the zero page; row/column clamps keep every address inside its tensor.
#include <algorithm>

#include "dtg/common.h"
#include <stdlib.h>
#include "dtg/gemm_epi.cuh"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/bn_epi.cuh"

namespace dtg {
using namespace gemm;

// stride applies to both spatial dims except in the C8 forward and the wgrad, which also take a separate
// W stride (sw): the ResNet stem runs as a stride (2, 1) conv over pixel pairs (stem_pairs in
// models/resnet_fused.py)
struct ConvGeom {
  int N, H, W, C, K, R, S, P, Q, stride, pad, sw;
  FastDiv fPQ, fQ, fHW, fW, fC, fS, fK;
};

static ConvGeom make_geom(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int sw = 0) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.stride = stride; g.pad = pad;
  g.sw = sw > 0 ? sw : stride;
  g.P = (H + 2 * pad - R) / stride + 1;
  g.Q = (W + 2 * pad - S) / g.sw + 1;
  g.fPQ = FastDiv(g.P * g.Q); g.fQ = FastDiv(g.Q); g.fHW = FastDiv(H * W); g.fW = FastDiv(W);
  g.fC = FastDiv(C); g.fS = FastDiv(S); g.fK = FastDiv(K);
  return g;
}

// ---- fwd A: x gathered at the output positions of the tile rows (KC) ---------------------------
// C8: the input has exactly 8 (zero-padded) channels -- the ResNet stem, 3 -> 8 -- so one 16-B
// chunk is one pixel and a 64-deep K step spans 8 (r, s) taps; K runs over (r, s, c) padded to a
// multiple of 64 (taps rs >= R*S read the zero page; their weights are zero too).
template <int ROWS, bool C8 = false, int NW = 4>
struct FwdA {
  static constexpr int PW = ROWS / (8 * NW);  // 8-row pieces per wave (one wave-instruction each)
  const bf16_t* x;
  const ConvGeom* g;
  int nbase[PW], ih0[PW], iw0[PW];
  int cx;  // this lane's source chunk (0..7) -- constant: (lane & 7) ^ (row & 7) with row & 7 = lane >> 3
  __device__ __forceinline__ void init(const ConvGeom& G, const bf16_t* xp, int row0, int wave, int lane) {
    x = xp;
    g = &G;
    const int M = G.N * G.P * G.Q;
    cx = (lane & 7) ^ (lane >> 3);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      int m = row0 + (wave * PW + i) * 8 + (lane >> 3);
      m = m < M ? m : M - 1;
      uint32_t n, pq, p, q;
      G.fPQ.divmod((uint32_t)m, n, pq);
      G.fQ.divmod(pq, p, q);
      nbase[i] = (int)n * G.H;
      ih0[i] = (int)p * G.stride - G.pad;
      iw0[i] = (int)q * G.sw - G.pad;
    }
  }
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave) const {
    uint32_t rs, c0, r, s;
    bool rs_ok = true;
    if constexpr (C8) {
      rs = (uint32_t)(k0 >> 3) + cx;
      c0 = 0;
      rs_ok = rs < (uint32_t)(g->R * g->S);
      g->fS.divmod(rs_ok ? rs : 0, r, s);
    } else {
      g->fC.divmod((uint32_t)k0, rs, c0);
      g->fS.divmod(rs, r, s);
    }
    const int ch = C8 ? 0 : (int)c0 + cx * 8;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int ih = ih0[i] + (int)r, iw = iw0[i] + (int)s;
      const bool ok = rs_ok && (unsigned)ih < (unsigned)g->H && (unsigned)iw < (unsigned)g->W;
      const int ihc = ok ? ih : 0, iwc = ok ? iw : 0;
      const void* src = sel(ok, x + ((long long)(nbase[i] + ihc) * g->W + iwc) * g->C + ch);
      const int r0 = (wave * PW + i) * 8;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + r0 * 128), 16, 0, 0);
    }
  }
};

// ---- dgrad A: dy gathered at the input positions of the tile rows (KC), stride 1 ----------------
template <int ROWS, int NW = 4>
struct DgradA {
  static constexpr int PW = ROWS / (8 * NW);
  const bf16_t* dy;
  const ConvGeom* g;
  int nbase[PW], ph0[PW], qw0[PW];
  int cx;
  __device__ __forceinline__ void init(const ConvGeom& G, const bf16_t* dyp, int row0, int wave, int lane) {
    dy = dyp;
    g = &G;
    const int M = G.N * G.H * G.W;
    cx = (lane & 7) ^ (lane >> 3);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      int m = row0 + (wave * PW + i) * 8 + (lane >> 3);
      m = m < M ? m : M - 1;
      uint32_t n, hw, h, w;
      G.fHW.divmod((uint32_t)m, n, hw);
      G.fW.divmod(hw, h, w);
      nbase[i] = (int)n * G.P;
      ph0[i] = (int)h + G.pad;
      qw0[i] = (int)w + G.pad;
    }
  }
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave) const {
    uint32_t rs, k0c, r, s;
    g->fK.divmod((uint32_t)k0, rs, k0c);
    g->fS.divmod(rs, r, s);
    const int ch = (int)k0c + cx * 8;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int p = ph0[i] - (int)r, q = qw0[i] - (int)s;
      const bool ok = (unsigned)p < (unsigned)g->P && (unsigned)q < (unsigned)g->Q;
      const int pc = ok ? p : 0, qc = ok ? q : 0;
      const void* src = sel(ok, dy + ((long long)(nbase[i] + pc) * g->Q + qc) * g->K + ch);
      const int r0 = (wave * PW + i) * 8;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + r0 * 128), 16, 0, 0);
    }
  }
};

// ---- dgrad B: w as B[(r,s,k)][c] (MC: c contiguous) ---------------------------------------------
template <int ROWS, int NW = 4>
struct DgradB {
  static constexpr int CH = ROWS / 8, KPI = 64 / CH, PW = 64 / KPI / NW;
  const bf16_t* w;
  const ConvGeom* g;
  int col0;
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave, int lane) const {
    uint32_t rs, kb;
    g->fK.divmod((uint32_t)k0, rs, kb);
    const long long rsc = (long long)g->R * g->S * g->C;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int kr0 = (wave * PW + i) * KPI;
      const int kr = kr0 + lane / CH;
      const int c = (lane % CH) ^ mc_swz<CH>(kr);
      const int col = col0 + c * 8;
      const bool ok = col < g->C;
      const void* src = sel(ok, w + (long long)((int)kb + kr) * rsc + (long long)rs * g->C + (ok ? col : 0));
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + kr0 * ROWS * 2), 16, 0, 0);
    }
  }
};

// ---- wgrad B: x as B[(n,p,q)][(r,s,c)] (MC: c contiguous) ----------------------------------------
// A lane's columns (r, s, c) are the same at every K step (k0 advances by 64 rows and the MC swizzle
// depends on the row within the tile only), so they are decomposed once in init(); a K step
// decomposes only its rows m = k0 + kr into (n, p, q).
template <int ROWS, int NW = 4>
struct WgradB {
  static constexpr int CH = ROWS / 8, KPI = 64 / CH, PW = 64 / KPI / NW;
  const bf16_t* x;
  const ConvGeom* g;
  int M;
  int dr[PW], ds[PW], cc[PW];  // r - pad, s - pad, channel; a padded column gets dr far out of range
  __device__ __forceinline__ void init(const bf16_t* xp, const ConvGeom& G, int col0, int Mrows, int wave, int lane) {
    x = xp;
    g = &G;
    M = Mrows;
    const int ncols = G.R * G.S * G.C;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int kr = (wave * PW + i) * KPI + lane / CH;
      const int c = (lane % CH) ^ mc_swz<CH>(kr);
      const int col = col0 + c * 8;
      uint32_t rs, ch, r, s;
      G.fC.divmod((uint32_t)(col < ncols ? col : 0), rs, ch);
      G.fS.divmod(rs, r, s);
      dr[i] = col < ncols ? (int)r - G.pad : -(1 << 28);
      ds[i] = (int)s - G.pad;
      cc[i] = (int)ch;
    }
  }
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave, int lane) const {
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int kr0 = (wave * PW + i) * KPI;
      const int m = k0 + kr0 + lane / CH;
      uint32_t n, pq, p, q;
      g->fPQ.divmod((uint32_t)(m < M ? m : 0), n, pq);
      g->fQ.divmod(pq, p, q);
      const int ih = (int)p * g->stride + dr[i], iw = (int)q * g->sw + ds[i];
      const bool ok = m < M && (unsigned)ih < (unsigned)g->H && (unsigned)iw < (unsigned)g->W;
      const void* src = sel(ok, x + ((long long)((int)n * g->H + (ok ? ih : 0)) * g->W + (ok ? iw : 0)) * g->C + cc[i]);
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + kr0 * ROWS * 2), 16, 0, 0);
    }
  }
};

// ---- strided dgrad: one residue class (h % st, w % st) of dx per launch --------------------------
// For stride st the input row h = st*i + ph only receives the taps r = r0 + st*tr (r0 = (ph+pad) mod
// st), from dy row p = i + dh - tr (dh = (ph + pad - r0) / st).  Each residue class is therefore a
// dense stride-1 problem over (n, i, j) x (tr, ts, k) -- no MFMA work is spent on the zero taps the
// st^2-times-larger "dilated dy" formulation would multiply.
struct StrideClass {
  int ph, pw, r0, s0, nr, ns, Hc, Wc, dh, dw, tiles;
  FastDiv fHWc, fWc, fNS;
};
// all residue classes of one dgrad go out in ONE launch (blockIdx.y = class, heaviest first) so the
// small classes fill the CUs the big ones leave idle instead of each being a sub-wave launch
constexpr int kMaxClasses = 9;
struct StrideClasses {
  StrideClass c[kMaxClasses];
};

template <int ROWS, int NW = 4>
struct DgradSA {
  static constexpr int PW = ROWS / (8 * NW);
  const bf16_t* dy;
  const ConvGeom* g;
  const StrideClass* sc;
  int nbase[PW], pi[PW], qj[PW];
  int cx;
  __device__ __forceinline__ void init(const ConvGeom& G, const StrideClass& S, const bf16_t* dyp, int row0, int wave,
                                       int lane) {
    dy = dyp;
    g = &G;
    sc = &S;
    const int M = G.N * S.Hc * S.Wc;
    cx = (lane & 7) ^ (lane >> 3);
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      int m = row0 + (wave * PW + i) * 8 + (lane >> 3);
      m = m < M ? m : M - 1;
      uint32_t n, ij, ii, jj;
      S.fHWc.divmod((uint32_t)m, n, ij);
      S.fWc.divmod(ij, ii, jj);
      nbase[i] = (int)n * G.P;
      pi[i] = (int)ii + S.dh;
      qj[i] = (int)jj + S.dw;
    }
  }
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave) const {
    uint32_t t, k0c, tr, ts;
    g->fK.divmod((uint32_t)k0, t, k0c);
    sc->fNS.divmod(t, tr, ts);
    const int ch = (int)k0c + cx * 8;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int p = pi[i] - (int)tr, q = qj[i] - (int)ts;
      const bool ok = (unsigned)p < (unsigned)g->P && (unsigned)q < (unsigned)g->Q;
      const int pc = ok ? p : 0, qc = ok ? q : 0;
      const void* src = sel(ok, dy + ((long long)(nbase[i] + pc) * g->Q + qc) * g->K + ch);
      const int r0 = (wave * PW + i) * 8;
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + r0 * 128), 16, 0, 0);
    }
  }
};

template <int ROWS, int NW = 4>
struct DgradSB {
  static constexpr int CH = ROWS / 8, KPI = 64 / CH, PW = 64 / KPI / NW;
  const bf16_t* w;
  const ConvGeom* g;
  const StrideClass* sc;
  int col0;
  __device__ __forceinline__ void operator()(lds_char* tile, int k0, int wave, int lane) const {
    uint32_t t, kb, tr, ts;
    g->fK.divmod((uint32_t)k0, t, kb);
    sc->fNS.divmod(t, tr, ts);
    const int rs = (sc->r0 + g->stride * (int)tr) * g->S + sc->s0 + g->stride * (int)ts;
    const long long rsc = (long long)g->R * g->S * g->C;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const int kr0 = (wave * PW + i) * KPI;
      const int kr = kr0 + lane / CH;
      const int c = (lane % CH) ^ mc_swz<CH>(kr);
      const int col = col0 + c * 8;
      const bool ok = col < g->C;
      const void* src = sel(ok, w + (long long)((int)kb + kr) * rsc + (long long)rs * g->C + (ok ? col : 0));
      __builtin_amdgcn_global_load_lds(src, (lds_void*)(tile + kr0 * ROWS * 2), 16, 0, 0);
    }
  }
};

// ---------------------------------------------------------------------------------------------
template <class CF, int BNMODE = 0, bool C8 = false>
__global__ void __launch_bounds__(CF::NTH, CF::NW == 4 ? 2 : 1) conv_fwd_kernel(ConvGeom G, const bf16_t* __restrict__ x,
                                                         const bf16_t* __restrict__ w, Epi e, int tiles_n, BnEpi bn) {
  static_assert(CF::BK == 64, "conv loaders stage 64-deep K steps");
  __shared__ __attribute__((aligned(16))) char smem_raw[CF::LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * CF::BM, bn0 = (t % tiles_n) * CF::BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = G.N * G.P * G.Q, Kd = C8 ? (G.R * G.S * 8 + 63) / 64 * 64 : G.R * G.S * G.C;  // C8: w is [K][Kd]
  FwdA<CF::BM, C8, CF::NW> sa;
  sa.init(G, x, bm0, wave, lane);
  DenseKC<false> sb{w, (long long)Kd, G.K, Kd};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop_st<CF, true, true>([&](lds_char* tl, int k0) { sa(tl, k0, wave); },
                              [&](lds_char* tl, int k0) { stage_kc<CF::BN, DenseKC<false>, CF::NW>(sb, tl, bn0, k0, wave, lane); },
                              smem, 0, Kd, acc);
  if constexpr (BNMODE != 0) {
    epilogue_bn<CF, BNMODE>(smem, acc, bm0, bn0, M, G.K, e, bn, t, [](int m) { return m; });
    return;
  }
  epilogue_staged<CF>(smem, acc, bm0, bn0, M, G.K, [&](int m, int n, float (&v)[8]) { epi_store8_fast(e, m, n, v); });
}

// WT: w is the transposed weight wT[c][(r,s,k)] (K-contiguous, transposed once per step by the caller),
// so B is staged like the forward's weights (ds_read_b128) instead of through the MN-contiguous
// [(r,s,k)][c] image and hardware-transposed reads
template <class CF, int BNMODE = 0, bool WT = false>
__global__ void __launch_bounds__(CF::NTH, CF::NW == 4 ? 2 : 1) conv_dgrad_kernel(ConvGeom G, const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ w, Epi e, int tiles_n, BnEpi bn) {
  static_assert(CF::BK == 64, "conv loaders stage 64-deep K steps");
  __shared__ __attribute__((aligned(16))) char smem_raw[CF::LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * CF::BM, bn0 = (t % tiles_n) * CF::BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = G.N * G.H * G.W, Kd = G.R * G.S * G.K;
  DgradA<CF::BM, CF::NW> sa;
  sa.init(G, dy, bm0, wave, lane);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (WT) {
    DenseKC<true> sb{w, (long long)Kd, G.C, Kd};
    mainloop_st<CF, true, true>([&](lds_char* tl, int k0) { sa(tl, k0, wave); },
                                [&](lds_char* tl, int k0) { stage_kc<CF::BN, DenseKC<true>, CF::NW>(sb, tl, bn0, k0, wave, lane); },
                                smem, 0, Kd, acc);
  } else {
    DgradB<CF::BN, CF::NW> sb{w, &G, bn0};
    mainloop_st<CF, true, false>([&](lds_char* tl, int k0) { sa(tl, k0, wave); },
                                 [&](lds_char* tl, int k0) { sb(tl, k0, wave, lane); }, smem, 0, Kd, acc);
  }
  if constexpr (BNMODE != 0) {
    epilogue_bn<CF, BNMODE>(smem, acc, bm0, bn0, M, G.C, e, bn, t, [](int m) { return m; });
    return;
  }
  epilogue_staged<CF>(smem, acc, bm0, bn0, M, G.C, [&](int m, int n, float (&v)[8]) { epi_store8_fast(e, m, n, v); });
}

template <class CF>
__global__ void __launch_bounds__(CF::NTH, CF::NW == 4 ? 2 : 1) conv_wgrad_kernel(ConvGeom G, const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ x, float* __restrict__ ws,
                                                           int tiles_n, int k_per_split) {
  static_assert(CF::BK == 64, "conv loaders stage 64-deep K steps");
  __shared__ __attribute__((aligned(16))) char smem_raw[CF::LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  // (split, tile) remapped over the whole grid so a K-split's tiles share one XCD's L2 (see gemm_kernel)
  const int ntl = gridDim.x;
  const int wid = xcd_remap(blockIdx.x + blockIdx.y * ntl, ntl * gridDim.y);
  const int split = wid / ntl, t = wid - split * ntl;
  const int bm0 = (t / tiles_n) * CF::BM, bn0 = (t % tiles_n) * CF::BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = G.N * G.P * G.Q;              // reduction length
  const int Mo = G.K, No = G.R * G.S * G.C;   // output dw [K][RSC]
  const int kbeg = split * k_per_split, kend = min(M, kbeg + k_per_split);
  DenseMC<true> sa{dy, (long long)G.K, G.K, M};
  WgradB<CF::BN, CF::NW> sb;
  sb.init(x, G, bn0, M, wave, lane);
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop_st<CF, false, false>([&](lds_char* tl, int k0) { stage_mc<CF::BM, DenseMC<true>, CF::NW>(sa, tl, bm0, k0, wave, lane); },
                                [&](lds_char* tl, int k0) { sb(tl, k0, wave, lane); }, smem, kbeg, kend, acc);
  float* slab = ws + (long long)split * Mo * No;
  epilogue_staged<CF>(smem, acc, bm0, bn0, Mo, No, [&](int m, int n, float (&v)[8]) {
    store8_f32(slab + (long long)m * No + n, v);
  });
}

template <class CF, int BNMODE = 0>
__global__ void __launch_bounds__(CF::NTH, CF::NW == 4 ? 2 : 1) conv_dgrad_s_kernel(ConvGeom G, StrideClasses SC,
                                                             const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ w, Epi e, int tiles_n,
                                                             BnEpi bn) {
  static_assert(CF::BK == 64, "conv loaders stage 64-deep K steps");
  __shared__ __attribute__((aligned(16))) char smem_raw[CF::LDS_BYTES];
  lds_char* smem = (lds_char*)smem_raw;
  const StrideClass S = SC.c[blockIdx.y];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  if (t >= S.tiles) return;
  const int bm0 = (t / tiles_n) * CF::BM, bn0 = (t % tiles_n) * CF::BN;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int M = G.N * S.Hc * S.Wc, Kd = S.nr * S.ns * G.K;
  DgradSA<CF::BM, CF::NW> sa;
  sa.init(G, S, dy, bm0, wave, lane);
  DgradSB<CF::BN, CF::NW> sb{w, &G, &S, bn0};
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  mainloop_st<CF, true, false>([&](lds_char* tl, int k0) { sa(tl, k0, wave); },
                               [&](lds_char* tl, int k0) { sb(tl, k0, wave, lane); }, smem, 0, Kd, acc);
  auto rowmap = [&](int m) {
    uint32_t nn, ij, ii, jj;
    S.fHWc.divmod((uint32_t)m, nn, ij);
    S.fWc.divmod(ij, ii, jj);
    return ((int)nn * G.H + G.stride * (int)ii + S.ph) * G.W + G.stride * (int)jj + S.pw;
  };
  if constexpr (BNMODE != 0) {  // slot index spread over the residue classes too
    epilogue_bn<CF, BNMODE>(smem, acc, bm0, bn0, M, G.C, e, bn, t + (int)blockIdx.y * 7, rowmap);
    return;
  }
  epilogue_staged<CF>(smem, acc, bm0, bn0, M, G.C, [&](int m, int n, float (&v)[8]) { epi_store8_fast(e, rowmap(m), n, v); });
}

// ---------------------------------------------------------------------------------------------
static bool conv_skinny(int n) { return n <= 64; }

// LDS ring depth of the implicit-GEMM kernels: 1 (32-40 KB of LDS, ~4 workgroups per CU hide latency
// across blocks) or 2 (64-80 KB, 2 per CU, DMA of the next K-step under the current one).
// conv_set_stages() overrides it per pass (fwd, dgrad, wgrad) for A/B tools (tools/conv_sweep.sh).
// Default (measured, profiles/r01_tiles): one stage, except fwd/dgrad grids shorter than 512
// 128x128 tiles with a reduction of >= 2048 (the 7x7 / 512-channel layers), which keep the 2-deep ring.
static int g_conv_stages[4] = {-1, -1, -1, -1};  // fwd, dgrad, wgrad, 8-channel (stem) fwd
static int conv_stages(int which, long long M = 0, int N = 0, int Kred = 0) {
  if (g_conv_stages[which] > 0) return g_conv_stages[which];
  if (which == 2) return 1;
  const long long tiles = ((M + 127) / 128) * ((N + 127) / 128);
  return (tiles < 512 && Kred >= 2048) ? 2 : 1;
}
// schedule code: 1 = single LDS stage, 2 = two-stage ring, 3 = single stage, register-pipelined (Cfg RP)
void conv_set_stages(int which, int stages) {  // 0 restores the measured default
  if (which >= 0 && which < 4) g_conv_stages[which] = stages >= 1 && stages <= 3 ? stages : -1;
}

// Output tile forced per pass (fwd, dgrad) for A/B tools (conv_force_tile; tools/conv_tile_ab.py): 0 = the
// heuristics; 1 = 128x256, 8 waves, register-pipelined; 2 = 256x128, 8 waves, RP; 3 = 128x256, 8 waves, single
// stage.  Wider output tiles re-read the gathered input through L2 once per 256 output channels instead of 128.
static int g_conv_tile[2] = {0, 0};
void conv_force_tile(int which, int code) {
  if (which >= 0 && which < 2) g_conv_tile[which] = code;
}
template <class F>
static bool run_forced_tile(int which, F&& run) {
  switch (g_conv_tile[which]) {
    case 1: run(Cfg<128, 256, 1, 8, 64, true>()); return true;
    case 2: run(Cfg<256, 128, 1, 8, 64, true>()); return true;
    case 3: run(Cfg<128, 256, 1, 8>()); return true;
    default: return false;
  }
}

template <int BM, int BN, class F>
static void run_sched(int sched, F&& run) {
  if (sched == 1) run(Cfg<BM, BN, 1>());
  else if (sched == 2) run(Cfg<BM, BN, 2>());
  else run(Cfg<BM, BN, 1, 4, 64, true>());
}


int conv_supported(int C, int K, int R, int S, int stride, int pad, int which) {
  if (C == 8 && K % 64 == 0 && which != 1) return 1;  // stem: fwd (conv_fwd_c8) and wgrad
  if (C % 64 || K % 64) return 0;
  if (which == 1 && stride * stride > kMaxClasses) return 0;  // one launch holds <= 9 residue classes
  return 1;
}

void conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, int C, int K, int R, int S,
              int stride, int pad, hipStream_t st, const BnEpi& bn) {
  // 64 -> 64 3x3 / s1 / p1 with the BN statistics (ResNet-50 stage 1): the direct halo-tile conv (conv_halo.hip)
  if (bn.mode == 1 && R == 3 && S == 3 && stride == 1 && pad == 1 && g_conv_tile[0] == 0 && g_conv_stages[0] <= 0 &&
      conv3x3_halo_bn_ok(C, K, H, W) && conv3x3_halo_bn_fwd(x, w, y, N, H, W, bn.part, st))
    return;
  // 1x1 / s2 projection from 256 channels with the BN statistics (ResNet-50 stage 2): the streaming expand kernel
  // with a stride-2 row gather (gemm_expand.hip)
  if (bn.mode == 1 && R == 1 && S == 1 && stride == 2 && pad == 0 && g_conv_tile[0] == 0 && g_conv_stages[0] <= 0 &&
      conv1x1_s2_expand_bn(x, N, H, W, C, w, y, K, bn.part, st))
    return;
  ConvGeom G = make_geom(N, H, W, C, K, R, S, stride, pad);
  const int M = N * G.P * G.Q;
  Epi e{y, K, 1, 1.f, 0.f, nullptr, 0};
  auto run = [&](auto cf) {
    using CF = decltype(cf);
    const int tn = (K + CF::BN - 1) / CF::BN, tm = (M + CF::BM - 1) / CF::BM;
    if (bn.mode == 1) { conv_fwd_kernel<CF, 1><<<tm * tn, CF::NTH, 0, st>>>(G, x, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else { conv_fwd_kernel<CF><<<tm * tn, CF::NTH, 0, st>>>(G, x, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
  };
  if (run_forced_tile(0, run)) return;
  const int sc = conv_stages(0, M, K, R * S * C);
  if (conv_skinny(K)) run_sched<256, 64>(sc, run);
  else run_sched<128, 128>(sc, run);
}

// 8-channel input (the stem, zero padded 3 -> 8); w is [K][Kp], Kp = ceil64(R*S*8), (r, s, c) order
bool stem_conv_stream_bn(const bf16_t* x8, const bf16_t* w8, bf16_t* y, int N, int Hp, int Wp2, int P, int Q,
                         float* part, hipStream_t st);

void conv_fwd_c8(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, int K, int R, int S, int stride,
                 int pad, hipStream_t st, const BnEpi& bn, int stride_w) {
  ConvGeom G = make_geom(N, H, W, 8, K, R, S, stride, pad, stride_w);
  const int M = N * G.P * G.Q;
  // ResNet's pixel-pair stem (64 channels, 7 x 4 taps = K 256 padded, (2, 1) stride, padding already in x): the
  // streaming form (gemm_expand.hip)
  if (bn.mode == 1 && K == 64 && R == 7 && S == 4 && stride == 2 && G.sw == 1 && pad == 0 &&
      stem_conv_stream_bn(x, w, y, N, H, W, G.P, G.Q, bn.part, st))
    return;
  Epi e{y, K, 1, 1.f, 0.f, nullptr, 0};
  auto run = [&](auto cf) {
    using CF = decltype(cf);
    const int tn = (K + CF::BN - 1) / CF::BN, tm = (M + CF::BM - 1) / CF::BM;
    if (bn.mode == 1) { conv_fwd_kernel<CF, 1, true><<<tm * tn, CF::NTH, 0, st>>>(G, x, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else { conv_fwd_kernel<CF, 0, true><<<tm * tn, CF::NTH, 0, st>>>(G, x, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
  };
  const int sc = g_conv_stages[3] > 0 ? g_conv_stages[3] : 1;
  if (conv_skinny(K)) run_sched<256, 64>(sc, run);
  else run_sched<128, 128>(sc, run);
}

// 128x128 data gradients: where the default picks the 2-stage ring (short grid, long K: the 7x7 3x3
// layers) the register-pipelined single stage is 10 % faster; elsewhere the plain single stage wins
// now that the mode-3 epilogue fits 4 workgroups per CU (profiles/r01_rp/lr_dgrad_sched.txt)
static int dgrad_sched(int sc, const ConvGeom& G) {
  return (g_conv_stages[1] <= 0 && G.R * G.S > 1 && sc == 2) ? 3 : sc;
}

// zero_rest = 0: rows of dx no residue class reaches (a 1x1 stride-2 dgrad: all but the even (h, w)) are
// left unwritten -- for a consumer that reads only the written rows (BnEpi::old_sub2)
static int conv_dgrad_strided(const ConvGeom& G, const bf16_t* dy, const bf16_t* w, bf16_t* dx, float beta,
                              hipStream_t st, const BnEpi& bn, int zero_rest) {
  const int s = G.stride;
  bool empty = false;
  for (int ph = 0; ph < s; ++ph)
    for (int pw = 0; pw < s; ++pw) {
      const int r0 = ((ph + G.pad) % s + s) % s, s0 = ((pw + G.pad) % s + s) % s;
      if (r0 >= G.R || s0 >= G.S || ph >= G.H || pw >= G.W) empty = true;
    }
  if (empty && bn.mode != 0) return 0;  // rows no launch writes would be missing from the statistics
  if (empty && beta == 0.f && zero_rest) {  // residue classes no tap reaches are zero
    fill_zero(dx, (long long)G.N * G.H * G.W * G.C * sizeof(bf16_t), st);
    beta = 1.f;
  }
  Epi e{dx, G.C, 1, 1.f, beta, nullptr, 0};
  const bool skinny = conv_skinny(G.C);
  const int BM = skinny ? 256 : 128, BN = skinny ? 64 : 128;
  const int tn = (G.C + BN - 1) / BN;
  StrideClasses SC;
  int nc = 0, max_tiles = 0;
  for (int ph = 0; ph < s; ++ph)
    for (int pw = 0; pw < s; ++pw) {
      StrideClass S;
      S.ph = ph; S.pw = pw;
      S.r0 = ((ph + G.pad) % s + s) % s;
      S.s0 = ((pw + G.pad) % s + s) % s;
      if (S.r0 >= G.R || S.s0 >= G.S || ph >= G.H || pw >= G.W) continue;
      S.nr = (G.R - S.r0 + s - 1) / s;
      S.ns = (G.S - S.s0 + s - 1) / s;
      S.Hc = (G.H - ph + s - 1) / s;
      S.Wc = (G.W - pw + s - 1) / s;
      S.dh = (ph + G.pad - S.r0) / s;
      S.dw = (pw + G.pad - S.s0) / s;
      S.fHWc = FastDiv(S.Hc * S.Wc); S.fWc = FastDiv(S.Wc); S.fNS = FastDiv(S.ns);
      S.tiles = (G.N * S.Hc * S.Wc + BM - 1) / BM * tn;
      max_tiles = S.tiles > max_tiles ? S.tiles : max_tiles;
      SC.c[nc++] = S;
    }
  if (nc == 0) return bn.mode == 0;
  // heaviest residue class (most taps) first: blocks dispatch in y-major order
  std::stable_sort(SC.c, SC.c + nc, [](const StrideClass& a, const StrideClass& b) {
    return a.nr * a.ns > b.nr * b.ns;
  });
  const dim3 grid(max_tiles, nc);
  const int sc = conv_stages(1, (long long)max_tiles * BM / tn, G.C, G.R * G.S * G.K / (s * s));
  auto run = [&](auto cf) {
    using CF = decltype(cf);
    if (bn.mode == 2) { conv_dgrad_s_kernel<CF, 2><<<grid, CF::NTH, 0, st>>>(G, SC, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else if (bn.mode == 3) { conv_dgrad_s_kernel<CF, 3><<<grid, CF::NTH, 0, st>>>(G, SC, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else { conv_dgrad_s_kernel<CF><<<grid, CF::NTH, 0, st>>>(G, SC, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
  };
  if (skinny) run_sched<256, 64>(sc, run);
  else run_sched<128, 128>(dgrad_sched(sc, G), run);
  return 1;
}

int conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int N, int H, int W, int C, int K, int R, int S,
               int stride, int pad, float beta, hipStream_t st, const BnEpi& bn, const bf16_t* wT, int zero_rest) {
  // 64 -> 64 3x3 / s1 / p1 with the BN-backward mode-3 epilogue (ResNet-50 stage 1): the direct halo-tile form
  if (R == 3 && S == 3 && stride == 1 && pad == 1 && beta == 0.f && g_conv_tile[1] == 0 && g_conv_stages[1] <= 0 &&
      conv3x3_halo_bn_ok(C, K, H, W) && conv3x3_halo_bn_dgrad(dy, w, dx, N, H, W, bn, st))
    return 1;
  ConvGeom G = make_geom(N, H, W, C, K, R, S, stride, pad);
  if (stride != 1) return conv_dgrad_strided(G, dy, w, dx, beta, st, bn, zero_rest);
  const int M = N * H * W;
  Epi e{dx, C, 1, 1.f, beta, nullptr, 0};
  auto run = [&](auto cf) {
    using CF = decltype(cf);
    const int tn = (C + CF::BN - 1) / CF::BN, tm = (M + CF::BM - 1) / CF::BM;
    if (bn.mode == 2) { conv_dgrad_kernel<CF, 2><<<tm * tn, CF::NTH, 0, st>>>(G, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else if (bn.mode == 3) { conv_dgrad_kernel<CF, 3><<<tm * tn, CF::NTH, 0, st>>>(G, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
    else { conv_dgrad_kernel<CF><<<tm * tn, CF::NTH, 0, st>>>(G, dy, w, e, tn, bn); DTG_LAUNCH_CHECK(); }
  };
  if (run_forced_tile(1, run)) return 1;
  const int sc = conv_stages(1, M, C, R * S * K);
  if (conv_skinny(C)) run_sched<256, 64>(sc, run);
  else run_sched<128, 128>(dgrad_sched(sc, G), run);
  return 1;
}

int conv_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w,
                     int target_wgs) {
  if (int hs = conv3x3_halo_wgrad_split(N, H, W, C, K, R, S, stride, pad, stride_w)) return hs;  // conv_halo.hip
  if (int ls = conv3x3_lin_wgrad_split(N, H, W, C, K, R, S, stride, pad, stride_w)) return ls;
  ConvGeom G = make_geom(N, H, W, C, K, R, S, stride, pad, stride_w);
  const int M = N * G.P * G.Q, No = R * S * C;
  const long long tiles = K <= 64 ? (long long)((No + 255) / 256) : (long long)((K + 127) / 128) * ((No + 127) / 128);
  // target workgroups (default 1024 = 4 single-stage workgroups per CU; measured 3-5 % faster than 512 on the
  // 14x14 / 28x28 3x3 layers, 256 is 25 % slower); more splits also grow the fp32 slabs the reduce pass re-reads
  const long long target = target_wgs > 0 ? target_wgs : 1024;
  // up to 1024 splits when the fp32 slabs stay small (<= 64 MB): the stem's single 64 x 224 output tile
  // needs 1024 splits to reach 1024 workgroups (at 256 it ran 256 workgroups, one per CU)
  const long long slab = (long long)K * No * 4;
  int s = 1;
  while (tiles * s < target && (long long)M / (s * 2) >= 1024 && (s < 256 || (s < 1024 && 2 * s * slab <= (64LL << 20))))
    s *= 2;
  return s;
}

void conv_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, int dw_bf16, float beta, float* ws, int split, int N,
                int H, int W, int C, int K, int R, int S, int stride, int pad, hipStream_t st, int stride_w,
                int sched) {
  if (split == conv3x3_halo_wgrad_split(N, H, W, C, K, R, S, stride, pad, stride_w)) {  // stage-1 3x3: halo tiles
    conv3x3_halo_wgrad(dy, x, ws, split, N, H, st);
    gemm_splitk_reduce(ws, split, K, R * S * C, Epi{dw, R * S * C, dw_bf16, 1.f, beta, nullptr, 0}, st);
    return;
  }
  if (split == conv3x3_lin_wgrad_split(N, H, W, C, K, R, S, stride, pad, stride_w)) {  // stages 2-4: linear halo
    conv3x3_lin_wgrad(dy, x, ws, split, N, H, W, C, K, st);
    gemm_splitk_reduce(ws, split, K, R * S * C, Epi{dw, R * S * C, dw_bf16, 1.f, beta, nullptr, 0}, st);
    return;
  }
  ConvGeom G = make_geom(N, H, W, C, K, R, S, stride, pad, stride_w);
  const int M = N * G.P * G.Q, No = R * S * C;
  int kps = (M + split - 1) / split;
  kps = (kps + BK - 1) / BK * BK;
  split = (M + kps - 1) / kps;
  Epi e{dw, No, dw_bf16, 1.f, beta, nullptr, 0};
  auto run = [&](auto cf) {
    using CF = decltype(cf);
    const int tn = (No + CF::BN - 1) / CF::BN, tm = (K + CF::BM - 1) / CF::BM;
    dim3 grid(tm * tn, split);
    conv_wgrad_kernel<CF><<<grid, CF::NTH, 0, st>>>(G, dy, x, ws, tn, kps); DTG_LAUNCH_CHECK();
  };
  const int sc = sched >= 1 && sched <= 3 && g_conv_stages[2] <= 0 ? sched : conv_stages(2);
  if (K <= 64) run_sched<64, 256>(sc, run);  // 64 output channels: one 64-row tile
  else run_sched<128, 128>(sc, run);
  gemm_splitk_reduce(ws, split, K, No, e, st);
}

}  // namespace dtg
