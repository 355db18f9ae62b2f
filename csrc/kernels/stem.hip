// ResNet-50 stem tail, fused: BatchNorm -> ReLU -> 3x3/2 max-pool on the 7x7/2 conv's output
// y [N, 112, 112, 64] (NHWC bf16), the largest activation of the network (411 MB at batch 256).
//
// Unfused, the tail streams y five times and writes two more full-size tensors:
//   fwd  stats(y) ; apply(y) -> a ; maxpool(a) -> out, idx                     (read y 2x, a 1x, write a)
//   bwd  maxpool_bwd(dout, idx) -> da ; reduce(da, a, y) ; dx(da, a, y) -> dy   (write da, read da/a/y 2x)
// Fused:
//   fwd  the statistics come from the conv's epilogue (bn_epi.cuh mode 1); ONE pass reads y, applies
//        scale/shift + ReLU in registers and max-pools: a never exists.
//   bwd  the pre-pool gradient is never stored either: both passes recompute it per input pixel as a
//        gather over the <= ceil(k/s)^2 pooled outputs whose window covers the pixel (their saved
//        argmax must point back at it), masked by relu'(bn(y)) recomputed from y and the saved
//        statistics.  Pass 1 reduces sum(dp), sum(dp*xhat) per channel (chunk partials -> the
//        deterministic BN finalize), pass 2 writes dy = a*dp + bx*y + c0 for the conv's wgrad.
// Bytes at batch 256: fwd 411 MB in + 154 MB out (was ~1.8 GB), bwd 2 x (154 + 411) MB in + 411 MB out
// (was ~2.6 GB).
//
// Tie semantics equal the unfused path: values are rounded to bf16 (what apply would have stored)
// before the window comparison, and the first maximum in window order wins.
#include <stdlib.h>

#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/bn_finalize.cuh"
#include "dtg/mfma_gemm.cuh"  // gemm::FastDiv

namespace dtg {

struct StemGeom {
  int N, H, W, C, P, Q, k, s, pad;
  gemm::FastDiv fW, fH;
};

__device__ __forceinline__ float bn_relu_bf(float y, float sc, float sf) {
  return bf2f(f2bf(fmaxf(fmaf(y, sc, sf), 0.f)));
}

// ---- forward: out[n,p,q,c] = max over the window of bf16(relu(y*scale + shift)), idx = argmax ----
// KT > 0: the window size as a compile-time constant: all KT*KT 16-byte loads are issued before the
// first comparison (clamped addresses + a validity flag) and held as raw bf16 vectors (4 VGPRs each,
// not 8 floats), so the window's loads are in flight together without the register cost of the
// earlier unrolled form.  KT = 0: runtime g.k (any window).
template <int KT>
__global__ void __launch_bounds__(256) stem_pool_fwd_kernel(const bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                            bf16_t* __restrict__ out, uint8_t* __restrict__ idx,
                                                            bf16_t* __restrict__ yam, StemGeom g) {
  const unsigned c8n = g.C >> 3;
  const unsigned total = (unsigned)g.N * g.P * g.Q * c8n;  // < 2^31 (host check)
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % c8n);
    unsigned t = i / c8n;
    const int q = (int)(t % (unsigned)g.Q);
    t /= (unsigned)g.Q;
    const int p = (int)(t % (unsigned)g.P);
    const int n = (int)(t / (unsigned)g.P);
    float sc[8], sf[8], m[8];
    uint32_t ym[4] = {0u, 0u, 0u, 0u};  // y at the argmax as raw bf16 pairs (4 VGPRs: the gather's occupancy)
    load8_f32(coef + c8 * 8, sc);
    load8_f32(coef + g.C + c8 * 8, sf);
    uint32_t am[2] = {0u, 0u};  // window argmax, 4 channels per word
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
    const int h0 = p * g.s - g.pad, w0 = q * g.s - g.pad;
    const bf16_t* yn = y + (long long)n * g.H * g.W * g.C + c8 * 8;
    auto take = [&](const uint4& raw, bool ok, uint8_t wi) {
      float v[8];
      gemm::unpack8_bf16(raw, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float a = ok ? bn_relu_bf(v[k], sc[k], sf[k]) : -INFINITY;
        if (a > m[k]) {  // strict: the first maximum in window order wins ties
          m[k] = a;
          am[k >> 2] = (am[k >> 2] & ~(0xffu << (8 * (k & 3)))) | ((uint32_t)wi << (8 * (k & 3)));
          const uint32_t word = (k >> 1) == 0 ? raw.x : (k >> 1) == 1 ? raw.y : (k >> 1) == 2 ? raw.z : raw.w;
          ym[k >> 1] = (k & 1) ? ((ym[k >> 1] & 0xffffu) | (word & 0xffff0000u))
                               : ((ym[k >> 1] & 0xffff0000u) | (word & 0xffffu));
        }
      }
    };
    if constexpr (KT > 0) {
      uint4 raw[KT * KT];
      bool okk[KT * KT];
#pragma unroll
      for (int rr = 0; rr < KT; ++rr) {
        const int h = h0 + rr;
        const bool hok = (unsigned)h < (unsigned)g.H;
#pragma unroll
        for (int cc = 0; cc < KT; ++cc) {
          const int w = w0 + cc;
          const bool ok = hok && (unsigned)w < (unsigned)g.W;
          okk[rr * KT + cc] = ok;
          raw[rr * KT + cc] =
              *reinterpret_cast<const uint4*>(yn + ((long long)(hok ? h : 0) * g.W + (ok ? w : 0)) * g.C);
        }
      }
#pragma unroll
      for (int j = 0; j < KT * KT; ++j) take(raw[j], okk[j], (uint8_t)j);
    } else {
      for (int rr = 0; rr < g.k; ++rr) {
        const int h = h0 + rr;
        const bool hok = (unsigned)h < (unsigned)g.H;
        for (int cc = 0; cc < g.k; ++cc) {
          const int w = w0 + cc;
          const bool ok = hok && (unsigned)w < (unsigned)g.W;
          const uint4 raw = *reinterpret_cast<const uint4*>(yn + ((long long)(hok ? h : 0) * g.W + (ok ? w : 0)) * g.C);
          take(raw, ok, (uint8_t)(rr * g.k + cc));
        }
      }
    }
    const long long o = (((long long)n * g.P + p) * g.Q + q) * g.C + c8 * 8;
    store8_bf16(out + o, m);
    *reinterpret_cast<uint2*>(idx + o) = make_uint2(am[0], am[1]);
    if (yam) *reinterpret_cast<uint4*>(yam + o) = make_uint4(ym[0], ym[1], ym[2], ym[3]);  // pooled bwd statistics
  }
}

// The same pass for ResNet's geometry (3x3 / stride 2 / pad 1, H = 2P, W = 2Q) walking down a segment of pooled rows:
// a thread owns (n, q, 8 channels, kPoolSeg rows) and keeps the window's bottom input row (2p + 1) in registers as
// the next window's top row (2(p + 1) - 1), so every input row is loaded once per segment instead of by the two
// windows that share it (the row-parallel form above re-reads part of y through HBM): 611 -> 553 us at batch 1024
// (profiles/r06_pool_rows; prefetching the next window's rows as well measured 590 us -- fewer waves resident).
// Window order, tie rule and outputs are those of stem_pool_fwd_kernel.
constexpr int kPoolSeg = 14;
__global__ void __launch_bounds__(256) stem_pool_fwd_rows_kernel(const bf16_t* __restrict__ y,
                                                                 const float* __restrict__ coef,
                                                                 bf16_t* __restrict__ out, uint8_t* __restrict__ idx,
                                                                 bf16_t* __restrict__ yam, StemGeom g, int nseg) {
  const unsigned c8n = g.C >> 3;
  const unsigned total = (unsigned)g.N * nseg * g.Q * c8n;  // < 2^31 (host check)
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % c8n);
    unsigned t = i / c8n;
    const int q = (int)(t % (unsigned)g.Q);
    t /= (unsigned)g.Q;
    const int seg = (int)(t % (unsigned)nseg);
    const int n = (int)(t / (unsigned)nseg);
    const int p0 = seg * kPoolSeg, p1 = min(g.P, p0 + kPoolSeg);
    float sc[8], sf[8];
    load8_f32(coef + c8 * 8, sc);
    load8_f32(coef + g.C + c8 * 8, sf);
    const int w0 = 2 * q - 1;
    const bool okc[3] = {w0 >= 0, true, true};  // w0 + 1, w0 + 2 <= 2Q - 1 < W
    const bf16_t* yn = y + (long long)n * g.H * g.W * g.C + c8 * 8;
    auto ld = [&](int h, int cc) -> uint4 {
      return *reinterpret_cast<const uint4*>(yn + ((long long)h * g.W + (okc[cc] ? w0 + cc : 0)) * g.C);
    };
    uint4 top[3];
    const bool top_ok0 = p0 > 0;
#pragma unroll
    for (int cc = 0; cc < 3; ++cc) top[cc] = ld(top_ok0 ? 2 * p0 - 1 : 0, cc);
    bool top_ok = top_ok0;
    for (int p = p0; p < p1; ++p) {
      uint4 mid[3], bot[3];
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) {
        mid[cc] = ld(2 * p, cc);
        bot[cc] = ld(2 * p + 1, cc);
      }
      float m[8];
      uint32_t ym[4] = {0u, 0u, 0u, 0u};
      uint32_t am[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < 8; ++k) m[k] = -INFINITY;
      auto take = [&](const uint4& raw, bool ok, uint8_t wi) {
        float v[8];
        gemm::unpack8_bf16(raw, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float a = ok ? bn_relu_bf(v[k], sc[k], sf[k]) : -INFINITY;
          if (a > m[k]) {  // strict: the first maximum in window order wins ties
            m[k] = a;
            am[k >> 2] = (am[k >> 2] & ~(0xffu << (8 * (k & 3)))) | ((uint32_t)wi << (8 * (k & 3)));
            const uint32_t word = (k >> 1) == 0 ? raw.x : (k >> 1) == 1 ? raw.y : (k >> 1) == 2 ? raw.z : raw.w;
            ym[k >> 1] = (k & 1) ? ((ym[k >> 1] & 0xffffu) | (word & 0xffff0000u))
                                 : ((ym[k >> 1] & 0xffff0000u) | (word & 0xffffu));
          }
        }
      };
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) take(top[cc], top_ok && okc[cc], (uint8_t)cc);
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) take(mid[cc], okc[cc], (uint8_t)(3 + cc));
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) take(bot[cc], okc[cc], (uint8_t)(6 + cc));
      const long long o = (((long long)n * g.P + p) * g.Q + q) * g.C + c8 * 8;
      store8_bf16(out + o, m);
      *reinterpret_cast<uint2*>(idx + o) = make_uint2(am[0], am[1]);
      if (yam) *reinterpret_cast<uint4*>(yam + o) = make_uint4(ym[0], ym[1], ym[2], ym[3]);
#pragma unroll
      for (int cc = 0; cc < 3; ++cc) top[cc] = bot[cc];
      top_ok = true;
    }
  }
}

static int g_pool_rows = 1;
void stem_pool_rows_set(int on) { g_pool_rows = on; }

// dp at input pixel m = (n, h, w), channels c0..c0+7: sum of the pooled gradients routed to it,
// masked by relu'(bn(y)) (yv = y at the pixel, sc/sf = the forward scale/shift).  With k <= 2s (the
// host checks it) a pixel lies in at most 2 x 2 windows: the pooled rows p_hi - 1, p_hi and columns
// q_hi - 1, q_hi.  All four candidates are loaded unconditionally (clamped addresses, invalid ones
// masked by an impossible window index) so their loads are independent and in flight together.
__device__ __forceinline__ void stem_dp(const bf16_t* __restrict__ dout, const uint8_t* __restrict__ idx,
                                        const StemGeom& g, long long m, int c0, const float (&yv)[8],
                                        const float (&sc)[8], const float (&sf)[8], float (&dp)[8]) {
  uint32_t nh, w, n, h;
  g.fW.divmod((uint32_t)m, nh, w);
  g.fH.divmod(nh, n, h);
  const int hp = (int)h + g.pad, wp = (int)w + g.pad;
  const int p_lo = hp >= g.k ? (hp - g.k) / g.s + 1 : 0, p_hi = min(g.P - 1, hp / g.s);
  const int q_lo = wp >= g.k ? (wp - g.k) / g.s + 1 : 0, q_hi = min(g.Q - 1, wp / g.s);
  uint2 pk[4];
  uint4 dv[4];  // raw bf16 pairs: 16 VGPRs instead of 32 (occupancy of the latency-bound gather)
  uint32_t wi[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int p = p_hi - 1 + (j >> 1), q = q_hi - 1 + (j & 1);
    const bool ok = p >= p_lo && q >= q_lo;  // (p, q <= hi by construction; lo >= 0)
    const int pc = ok ? p : p_hi, qc = ok ? q : q_hi;
    wi[j] = ok ? (uint32_t)((hp - p * g.s) * g.k + (wp - q * g.s)) : 0xffu;  // 0xff: matches no index
    const long long o = (((long long)n * g.P + pc) * g.Q + qc) * g.C + c0;
    pk[j] = *reinterpret_cast<const uint2*>(idx + o);
    dv[j] = *reinterpret_cast<const uint4*>(dout + o);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t word = k < 4 ? pk[j].x : pk[j].y;
      const uint32_t pair = (k >> 1) == 0 ? dv[j].x : (k >> 1) == 1 ? dv[j].y : (k >> 1) == 2 ? dv[j].z : dv[j].w;
      const float d = __uint_as_float((k & 1) ? (pair & 0xffff0000u) : (pair << 16));
      acc += ((word >> (8 * (k & 3))) & 0xffu) == wi[j] ? d : 0.f;
    }
    dp[k] = fmaf(yv[k], sc[k], sf[k]) > 0.f ? acc : 0.f;
  }
}

// ---- backward pass 1: per-chunk sum(dp), sum(dp * xhat) ------------------------------------------
template <int TPR>
__global__ void __launch_bounds__(kBlk) stem_bwd_reduce_kernel(const bf16_t* __restrict__ dout,
                                                               const uint8_t* __restrict__ idx,
                                                               const bf16_t* __restrict__ y,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               const float* __restrict__ smean,
                                                               const float* __restrict__ sinv, StemGeom g, long long M,
                                                               long long rpc, float* __restrict__ part) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  __shared__ float sh[2][RPP][CW + 4];
  const int C = g.C;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < C) {
    float mu[8], is[8], ga[8], be[8], sc[8], sf[8];
    load8_f32(smean + c0, mu);
    load8_f32(sinv + c0, is);
    load8_f32(gamma + c0, ga);
    load8_f32(beta + c0, be);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = ga[k] * is[k];
      sf[k] = be[k] - mu[k] * sc[k];
    }
    const long long m0 = (long long)blockIdx.x * rpc;
    const long long m1 = m0 + rpc < M ? m0 + rpc : M;
    for (long long m = m0 + ty; m < m1; m += RPP) {
      float yv[8], dp[8];
      load8_bf16(y + m * C + c0, yv);
      stem_dp(dout, idx, g, m, c0, yv, sc, sf, dp);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += dp[k];
        q[k] += dp[k] * (yv[k] - mu[k]) * is[k];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sh[0][ty][tx * 8 + k] = s[k];
    sh[1][ty][tx * 8 + k] = q[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < CW; c += kBlk) {
    float ts = 0.f, tq = 0.f;
#pragma unroll 4
    for (int r = 0; r < RPP; ++r) {
      ts += sh[0][r][c];
      tq += sh[1][r][c];
    }
    const int cc = blockIdx.y * CW + c;
    if (cc < C) {
      part[((long long)blockIdx.x * 2 + 0) * C + cc] = ts;
      part[((long long)blockIdx.x * 2 + 1) * C + cc] = tq;
    }
  }
}

// ---- backward pass 2: dy = a*dp + bx*y + c0 ------------------------------------------------------
template <int TPR>
__global__ void __launch_bounds__(kBlk) stem_bwd_dx_kernel(const bf16_t* __restrict__ dout,
                                                           const uint8_t* __restrict__ idx,
                                                           const bf16_t* __restrict__ y, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ smean,
                                                           const float* __restrict__ sinv,
                                                           const float* __restrict__ coef, StemGeom g, long long M,
                                                           long long rpc, bf16_t* __restrict__ dy) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  const int C = g.C;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  if (c0 >= C) return;
  float sc[8], sf[8], a[8], bx[8], cc[8];
  {
    float mu[8], is[8], ga[8], be[8];
    load8_f32(smean + c0, mu);
    load8_f32(sinv + c0, is);
    load8_f32(gamma + c0, ga);
    load8_f32(beta + c0, be);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = ga[k] * is[k];
      sf[k] = be[k] - mu[k] * sc[k];
    }
  }
  load8_f32(coef + c0, a);
  load8_f32(coef + C + c0, bx);
  load8_f32(coef + 2 * C + c0, cc);
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  for (long long m = m0 + ty; m < m1; m += RPP) {
    float yv[8], dp[8], o[8];
    load8_bf16(y + m * C + c0, yv);
    stem_dp(dout, idx, g, m, c0, yv, sc, sf, dp);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(a[k], dp[k], fmaf(bx[k], yv[k], cc[k]));
    store8_bf16(dy + m * C + c0, o);
  }
}

// ---- backward pass 1 at pooled resolution ----------------------------------------------------------------
// Every pooled gradient lands on exactly one input pixel, its window argmax, and is masked there by
// relu'(bn(y)).  So sum(dp) = sum over pooled outputs of dout * [bn(y_am) > 0] and sum(dp * xhat) adds
// dout * [bn(y_am) > 0] * xhat(y_am), y_am = y at the argmax, which the forward pool saved (yam): the same
// terms as the pixel-resolution pass in another summation order, from the pooled dout + y_am (1/2 of y's
// bytes at stride 2) instead of y, the pooled dout and the argmax through the window gather.  Each thread
// keeps one 8-channel chunk (the grid stride is a multiple of C / 8: the host requires 256 % (C / 8) == 0),
// U chunks' loads in flight per iteration; block-reduced and added into one of kBnStatSlots zeroed slots.
template <int U>
__global__ void __launch_bounds__(256) stem_bwd_pooled_stats_kernel(const bf16_t* __restrict__ dout,
                                                                    const bf16_t* __restrict__ yam,
                                                                    const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta,
                                                                    const float* __restrict__ smean,
                                                                    const float* __restrict__ sinv, int C,
                                                                    long long chunks, float* __restrict__ part) {
  __shared__ float red[2][256][9];
  const int c8n = C >> 3, c8 = threadIdx.x % c8n, c0 = c8 * 8;
  float sc[8], sf[8], mu[8], is[8];
  {
    float ga[8], be[8];
    load8_f32(smean + c0, mu);
    load8_f32(sinv + c0, is);
    load8_f32(gamma + c0, ga);
    load8_f32(beta + c0, be);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = ga[k] * is[k];
      sf[k] = be[k] - mu[k] * sc[k];
    }
  }
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto one = [&](const uint4& dr, const uint4& yr) {
    float d[8], yv[8];
    gemm::unpack8_bf16(dr, d);
    gemm::unpack8_bf16(yr, yv);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float dp = fmaf(yv[k], sc[k], sf[k]) > 0.f ? d[k] : 0.f;  // the pixel pass's mask expression
      s[k] += dp;
      q[k] += dp * (yv[k] - mu[k]) * is[k];
    }
  };
  const long long stride = (long long)gridDim.x * 256;
  long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < chunks; i += U * stride) {
    uint4 dr[U], yr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dr[u] = *reinterpret_cast<const uint4*>(dout + (i + u * stride) * 8);
      yr[u] = *reinterpret_cast<const uint4*>(yam + (i + u * stride) * 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(dr[u], yr[u]);
  }
  for (; i < chunks; i += stride)
    one(*reinterpret_cast<const uint4*>(dout + i * 8), *reinterpret_cast<const uint4*>(yam + i * 8));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[0][threadIdx.x][k] = s[k];
    red[1][threadIdx.x][k] = q[k];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    const int cc8 = c >> 3, k = c & 7;
    float ts = 0.f, tq = 0.f;
    for (int r = cc8; r < 256; r += c8n) {
      ts += red[0][r][k];
      tq += red[1][r][k];
    }
    float* slot = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * C;
    atomicAdd(slot + c, ts);
    atomicAdd(slot + C + c, tq);
  }
}

// ---- backward, banded: k = 3, s = 2, pad = 1, C = 64, H % 4 == 0 (ResNet's stem) --------------------
// One workgroup per (image, band of 4 input rows).  The pooled rows whose windows reach the band (3 rows:
// dout + argmax, 3 x Q x 64 x 3 B = 32 KB at Q = 56) are staged in LDS once, so an input pixel's <= 4
// candidate windows are LDS reads instead of 4 global gathers: 1.5x instead of 4x the pooled bytes move
// through L2, and the window geometry is shift arithmetic.  DX = false: pass 1, sum(dp) and sum(dp * xhat)
// per channel, block-reduced and added into one of kBnStatSlots zeroed slots; DX = true: pass 2,
// dy = a*dp + bx*y + c0.
constexpr int kStemBandRows = 4;

template <bool DX>
__global__ void __launch_bounds__(256) stem_bwd_band_kernel(const bf16_t* __restrict__ dout,
                                                            const uint8_t* __restrict__ idx,
                                                            const bf16_t* __restrict__ y,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ smean,
                                                            const float* __restrict__ sinv,
                                                            const float* __restrict__ coef, StemGeom g,
                                                            float* __restrict__ part, bf16_t* __restrict__ dy) {
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [3][Q][64] bf16 dout, then [3][Q][64] u8 argmax
  constexpr int C = 64;
  const int bands = g.H / kStemBandRows;
  const int n = blockIdx.x / bands, band = blockIdx.x - n * bands;
  const int h0 = band * kStemBandRows;
  const int p0 = h0 >> 1;  // pooled rows p0 .. p0 + 2 (those < P) cover input rows h0 .. h0 + 3
  bf16_t* sd = reinterpret_cast<bf16_t*>(lds);
  uint8_t* si = reinterpret_cast<uint8_t*>(lds + 3 * g.Q * C * 2);
  const int qc = g.Q * 8;  // 8-channel chunks per pooled row
  for (int i = threadIdx.x; i < 3 * qc; i += 256) {
    const int pr = i / qc;
    if (p0 + pr < g.P) {
      const long long o = (((long long)n * g.P + p0) * g.Q) * C + (long long)i * 8;
      *reinterpret_cast<uint4*>(sd + i * 8) = *reinterpret_cast<const uint4*>(dout + o);
      *reinterpret_cast<uint2*>(si + i * 8) = *reinterpret_cast<const uint2*>(idx + o);
    }
  }
  const int c8 = threadIdx.x & 7, c0 = c8 * 8;  // fixed per thread: 256 is a multiple of 8 chunks
  float sc[8], sf[8], mu[8], is[8], a[8], bx[8], cc[8];
  {
    float ga[8], be[8];
    load8_f32(smean + c0, mu);
    load8_f32(sinv + c0, is);
    load8_f32(gamma + c0, ga);
    load8_f32(beta + c0, be);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sc[k] = ga[k] * is[k];
      sf[k] = be[k] - mu[k] * sc[k];
    }
  }
  if constexpr (DX) {
    load8_f32(coef + c0, a);
    load8_f32(coef + C + c0, bx);
    load8_f32(coef + 2 * C + c0, cc);
  }
  __syncthreads();
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int chunks = kStemBandRows * g.W * 8;
  auto pix_off = [&](int i, int& h, int& w) {
    const int pix = i >> 3;
    const int hr = pix / g.W;
    w = pix - hr * g.W;
    h = h0 + hr;
    return (((long long)n * g.H + h) * g.W + w) * C + c0;
  };
  auto one = [&](int h, int w, long long off, const float (&yv)[8]) {
    const int hp = h + 1, wp = w + 1;  // padded coordinates
    const int p_hi = min(g.P - 1, hp >> 1), q_hi = min(g.Q - 1, wp >> 1);
    const int p_lo = hp >= 3 ? ((hp - 3) >> 1) + 1 : 0, q_lo = wp >= 3 ? ((wp - 3) >> 1) + 1 : 0;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p = p_hi - 1 + (j >> 1), qq = q_hi - 1 + (j & 1);
      if (p >= p_lo && qq >= q_lo) {
        const int li = ((p - p0) * g.Q + qq) * C + c0;
        const uint4 dv = *reinterpret_cast<const uint4*>(sd + li);
        const uint2 pk = *reinterpret_cast<const uint2*>(si + li);
        const uint32_t wi = (uint32_t)((hp - 2 * p) * 3 + (wp - 2 * qq));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t word = k < 4 ? pk.x : pk.y;
          const uint32_t pair = (k >> 1) == 0 ? dv.x : (k >> 1) == 1 ? dv.y : (k >> 1) == 2 ? dv.z : dv.w;
          const float d = __uint_as_float((k & 1) ? (pair & 0xffff0000u) : (pair << 16));
          acc[k] += ((word >> (8 * (k & 3))) & 0xffu) == wi ? d : 0.f;
        }
      }
    }
    float dp[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) dp[k] = fmaf(yv[k], sc[k], sf[k]) > 0.f ? acc[k] : 0.f;
    if constexpr (DX) {
      float o[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(a[k], dp[k], fmaf(bx[k], yv[k], cc[k]));
      store8_bf16(dy + off, o);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += dp[k];
        q[k] += dp[k] * (yv[k] - mu[k]) * is[k];
      }
    }
  };
  // pass 2: kStemU pixels per thread per iteration, all their y loads in flight before any window work (664 vs
  // 727 us at batch 1024); pass 1 measured slower that way (837 vs 775 us) and keeps one pixel per iteration
  constexpr int kStemU = DX ? 4 : 1;
  int i = threadIdx.x;
  for (; i + (kStemU - 1) * 256 < chunks; i += kStemU * 256) {
    int hh[kStemU], ww[kStemU];
    long long oo[kStemU];
    float yv[kStemU][8];
#pragma unroll
    for (int u = 0; u < kStemU; ++u) {
      oo[u] = pix_off(i + u * 256, hh[u], ww[u]);
      load8_bf16(y + oo[u], yv[u]);
    }
#pragma unroll
    for (int u = 0; u < kStemU; ++u) one(hh[u], ww[u], oo[u], yv[u]);
  }
  for (; i < chunks; i += 256) {
    int h, w;
    const long long off = pix_off(i, h, w);
    float yv[8];
    load8_bf16(y + off, yv);
    one(h, w, off, yv);
  }
  if constexpr (!DX) {
    __syncthreads();  // the staged rows are no longer read: reuse the LDS for the block reduction
    float* red = reinterpret_cast<float*>(lds);  // [2][32 thread rows][64 channels]
    const int r = threadIdx.x >> 3;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[r * C + c0 + k] = s[k];
      red[32 * C + r * C + c0 + k] = q[k];
    }
    __syncthreads();
    if (threadIdx.x < C) {
      float ts = 0.f, tq = 0.f;
#pragma unroll 8
      for (int j = 0; j < 32; ++j) {
        ts += red[j * C + threadIdx.x];
        tq += red[32 * C + j * C + threadIdx.x];
      }
      float* slot = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * C;
      atomicAdd(slot + threadIdx.x, ts);
      atomicAdd(slot + C + threadIdx.x, tq);
    }
  }
}

// dynamic LDS of the banded backward (see stem_bn_pool_bwd); must fit one workgroup's LDS (160 KB on gfx950),
// larger images (wide rows) take the per-pixel gather form instead
static size_t stem_band_lds(int Q, int C) {
  const size_t a = (size_t)3 * Q * C * 3, b = (size_t)2 * 32 * C * 4;
  return a > b ? a : b;
}

static bool stem_band_ok(int H, int C, int k, int s, int pad, int P, int Q) {
  return k == 3 && s == 2 && pad == 1 && C == 64 && H % kStemBandRows == 0 && P == (H - 1) / 2 + 1 &&
         stem_band_lds(Q, C) <= (size_t)160 * 1024;
}

// ---- input packing for the pixel-pair stem conv (ops/conv.py stem_pairs) ---------------------------
// x [N, H, W, C] (C <= 4, NHWC bf16) -> xp [N, H + 2*pad, Wp, 4] zero-padded (pad rows/columns on the
// top/left, the rest on the bottom/right, channels C..3 zero): one thread per 16-byte output chunk
// (two padded pixels), so the padding zeros and the copy are one pass (F.pad: a fill + a strided copy).
__global__ void __launch_bounds__(256) stem_pack_pairs_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xp,
                                                              int N, int H, int W, int C, int pad, int Hp, int Wp2) {
  const long long total = (long long)N * Hp * Wp2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int u = (int)(i % Wp2);
    const long long t = i / Wp2;
    const int hp = (int)(t % Hp);
    const int n = (int)(t / Hp);
    const int h = hp - pad;
    uint32_t w4[4] = {0u, 0u, 0u, 0u};  // 8 bf16: pixel 2u (channels 0..3), pixel 2u + 1
    if ((unsigned)h < (unsigned)H) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int w = 2 * u + e - pad;
        if ((unsigned)w < (unsigned)W) {
          const bf16_t* src = x + (((long long)n * H + h) * W + w) * C;
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (c < C) w4[e * 2 + (c >> 1)] |= (uint32_t)src[c] << (16 * (c & 1));
        }
      }
    }
    *reinterpret_cast<uint4*>(xp + i * 8) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

void stem_pack_pairs(const bf16_t* x, bf16_t* xp, int N, int H, int W, int C, int pad, int Hp, int Wp,
                     hipStream_t st) {
  const long long total = (long long)N * Hp * (Wp / 2);
  hipLaunchKernelGGL(stem_pack_pairs_kernel, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, x, xp, N, H, W, C,
                     pad, Hp, Wp / 2); DTG_LAUNCH_CHECK();
}

static StemGeom stem_geom(int N, int H, int W, int C, int k, int s, int pad, int P, int Q) {
  StemGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.P = P; g.Q = Q; g.k = k; g.s = s; g.pad = pad;
  g.fW = gemm::FastDiv((uint32_t)W);
  g.fH = gemm::FastDiv((uint32_t)H);
  return g;
}

// The gather passes are latency-bound (dependent index math and up to 8 small loads per row), so the
// reduction runs on ~4x the row chunks of a plain BN reduction (1024 workgroups = 4 per CU); the
// finalize reads the extra partials once.
static BnGeom stem_reduce_geom(long long M, int C) {
  BnGeom g = bn_geom(M, C);
  const int rpp = kBlk / g.tpr;
  long long nc = 1024 / g.gy;
  const long long max_chunks = (M + rpp - 1) / rpp;
  if (nc > max_chunks) nc = max_chunks;
  if (nc < 1) nc = 1;
  g.rows_per_chunk = (M + nc - 1) / nc;
  g.nchunk = (int)((M + g.rows_per_chunk - 1) / g.rows_per_chunk);
  return g;
}

// partial slots of the reduction passes: the gather form's per-chunk partials, at least kBnStatSlots (the
// banded and pooled passes add into that many zeroed slots)
static long long stem_part_slots(const BnGeom& g) { return g.nchunk > kBnStatSlots ? g.nchunk : kBnStatSlots; }

long long stem_bwd_workspace_floats(long long M, int C) {
  const BnGeom g = stem_reduce_geom(M, C);
  return stem_part_slots(g) * 2 * C + 3LL * C;
}

bool stem_pooled_stats_ok(int C) { return C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0; }

void stem_bn_pool_fwd(const bf16_t* y, const float* part, const float* gamma, const float* beta, float* rmean,
                      float* rvar, float* smean, float* sinv, float* coef, bf16_t* out, uint8_t* idx, int N, int H,
                      int W, int C, int k, int s, int pad, int P, int Q, float momentum, float eps, hipStream_t st,
                      bf16_t* yam) {
  const long long M = (long long)N * H * W;
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, kBnStatSlots, M, C, 0, gamma, beta, rmean, rvar, smean,
                                                         sinv, momentum, eps, coef, nullptr, nullptr, 0); DTG_LAUNCH_CHECK();
  const StemGeom g = stem_geom(N, H, W, C, k, s, pad, P, Q);
  const long long total = (long long)N * P * Q * (C / 8);
  // 3x3 / 2 / 1 windows over an even-sized input (ResNet): the row-walking form; other 3x3 windows: the unrolled
  // form with raw-vector loads; other windows: the runtime loop
  if (g_pool_rows && k == 3 && s == 2 && pad == 1 && H == 2 * P && W == 2 * Q) {
    const int nseg = (P + kPoolSeg - 1) / kPoolSeg;
    const long long tr = (long long)N * nseg * Q * (C / 8);
    hipLaunchKernelGGL(stem_pool_fwd_rows_kernel, dim3(grid_for(tr, 256, 8192)), dim3(256), 0, st, y, coef, out, idx,
                       yam, g, nseg);
  } else if (k == 3)
    hipLaunchKernelGGL(stem_pool_fwd_kernel<3>, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, y, coef, out, idx, yam, g);
  else
    hipLaunchKernelGGL(stem_pool_fwd_kernel<0>, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, y, coef, out, idx, yam, g);
  DTG_LAUNCH_CHECK();
}

void stem_bn_pool_bwd(const bf16_t* dout, const uint8_t* idx, const bf16_t* y, const float* gamma, const float* beta,
                      const float* smean, const float* sinv, bf16_t* dy, float* dgamma, float* dbeta, int accum,
                      float* ws, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, hipStream_t st,
                      const bf16_t* yam) {
  const long long M = (long long)N * H * W;
  const BnGeom bg = stem_reduce_geom(M, C);
  const StemGeom g = stem_geom(N, H, W, C, k, s, pad, P, Q);
  float* part = ws;
  float* coef = ws + stem_part_slots(bg) * 2 * C;
  const bool band = stem_band_ok(H, C, k, s, pad, P, Q) && bg.nchunk >= kBnStatSlots;
  const size_t lds = stem_band_lds(Q, C);
  const unsigned nb = (unsigned)(N * (H / kStemBandRows));
  // pass 1: sum(dp), sum(dp * xhat) -- at pooled resolution when the forward saved y at the argmax, else at
  // pixel resolution through the window gather (banded for ResNet's geometry)
  int nslots = kBnStatSlots;
  if (yam && stem_pooled_stats_ok(C)) {
    fill_zero(part, (long long)kBnStatSlots * 2 * C * sizeof(float), st);
    const long long chunks = (long long)N * P * Q * (C / 8);
    hipLaunchKernelGGL(stem_bwd_pooled_stats_kernel<4>, dim3(grid_for(chunks, 256, 2048)), dim3(256), 0, st, dout,
                       yam, gamma, beta, smean, sinv, C, chunks, part); DTG_LAUNCH_CHECK();
  } else if (band) {
    fill_zero(part, (long long)kBnStatSlots * 2 * C * sizeof(float), st);
    hipLaunchKernelGGL(stem_bwd_band_kernel<false>, dim3(nb), dim3(256), lds, st, dout, idx, y, gamma, beta, smean,
                       sinv, nullptr, g, part, nullptr); DTG_LAUNCH_CHECK();
  } else {
    dim3 grid(bg.nchunk, bg.gy);
    DTG_TPR_SWITCH(bg.tpr, stem_bwd_reduce_kernel<T><<<grid, kBlk, 0, st>>>(dout, idx, y, gamma, beta, smean, sinv, g,
                                                                           M, bg.rows_per_chunk, part)); DTG_LAUNCH_CHECK();
    nslots = bg.nchunk;
  }
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, nslots, M, C, accum ? 2 : 1, gamma, nullptr, nullptr,
                                                         nullptr, const_cast<float*>(smean), const_cast<float*>(sinv),
                                                         0.f, 0.f, coef, dgamma, dbeta); DTG_LAUNCH_CHECK();
  // pass 2: dy = a*dp + bx*y + c0
  if (band) {
    hipLaunchKernelGGL(stem_bwd_band_kernel<true>, dim3(nb), dim3(256), lds, st, dout, idx, y, gamma, beta, smean,
                       sinv, coef, g, nullptr, dy); DTG_LAUNCH_CHECK();
    return;
  }
  const long long rpa = elementwise_rpc(bg, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), bg.gy);
  DTG_TPR_SWITCH(bg.tpr, stem_bwd_dx_kernel<T><<<ga, kBlk, 0, st>>>(dout, idx, y, gamma, beta, smean, sinv, coef, g, M,
                                                                   rpa, dy)); DTG_LAUNCH_CHECK();
}

// Stem weight gradient from the padded-channel wgrad layouts into the parameter's own [K, R, S, C] memory
// (channels_last [K, C, R, S]): grad[k, r, s, c] += src[k, r, s', 8-chunk]; pair form (the pixel-pair conv,
// ops/conv.py stem_pairs): s' = s / 2, lane (s % 2) * 4 + c of a [K, R, S2, 8] buffer; plain form: s' = s,
// lane c of [K, R, S, 8].  One pass replaces a fill, a permuted copy, a cast and an add.
template <bool GBF16>
__global__ void __launch_bounds__(256) stem_dw_add_kernel(const float* __restrict__ src, void* __restrict__ grad, int K,
                                                          int R, int S, int C, int S2, int pair) {
  const int total = K * R * S * C;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c = i % C, s = (i / C) % S, r = (i / (C * S)) % R, k = i / (C * S * R);
    const int sp = pair ? s / 2 : s, lane = pair ? (s & 1) * 4 + c : c;
    const float v = src[((long long)(k * R + r) * S2 + sp) * 8 + lane];
    if constexpr (GBF16) {
      bf16_t* g = reinterpret_cast<bf16_t*>(grad);
      g[i] = f2bf(bf2f(g[i]) + v);
    } else {
      float* g = reinterpret_cast<float*>(grad);
      g[i] += v;
    }
  }
}

void stem_dw_add(const float* src, void* grad, int grad_bf16, int K, int R, int S, int C, int S2, int pair,
                 hipStream_t st) {
  const int total = K * R * S * C;
  const int grid = (total + 255) / 256;
  if (grad_bf16) stem_dw_add_kernel<true><<<grid, 256, 0, st>>>(src, grad, K, R, S, C, S2, pair);
  else stem_dw_add_kernel<false><<<grid, 256, 0, st>>>(src, grad, K, R, S, C, S2, pair);
  DTG_LAUNCH_CHECK();
}

// Pixel-pair stem weights (ops/conv.py stem_pairs): w [K, C, R, S] in channels_last memory ([K][R][S][C]) ->
// wp [K][KP] bf16, column (r, s2, lane) = r * S2 * 8 + s2 * 8 + lane with lane = (s % 2) * 4 + c, s = 2 s2 + s % 2;
// taps s >= S, channels c >= C and the columns past R * S2 * 8 are zero.  One pass per step instead of a pad /
// permute / pad chain of framework kernels.
__global__ void __launch_bounds__(256) stem_pack_weights_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp,
                                                                int K, int C, int R, int S, int S2, int KP) {
  const int total = K * KP;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int k = i / KP, j = i % KP;
    bf16_t v = 0;
    if (j < R * S2 * 8) {
      const int r = j / (S2 * 8), rem = j % (S2 * 8), lane = rem & 7;
      const int s = (rem >> 3) * 2 + (lane >> 2), c = lane & 3;
      if (s < S && c < C) v = w[((long long)(k * R + r) * S + s) * C + c];
    }
    wp[i] = v;
  }
}

void stem_pack_weights(const bf16_t* w, bf16_t* wp, int K, int C, int R, int S, int S2, int KP, hipStream_t st) {
  const int total = K * KP;
  stem_pack_weights_kernel<<<(total + 255) / 256, 256, 0, st>>>(w, wp, K, C, R, S, S2, KP); DTG_LAUNCH_CHECK();
}

}  // namespace dtg
