#include <stdlib.h>
// NHWC BatchNorm for training, fused with the residual add and ReLU that follow it in ResNet
// bottlenecks:   y = relu( (x - mean) * invstd * gamma + beta  [+ residual] )
//
// Memory-bound (HBM3E): every pass streams bf16 rows with 16-byte lanes.  A block owns a fixed
// slab of CW = TPR*8 channels and walks rows, so each lane keeps its 8 channels' scale/shift and
// partial sums in registers; no per-element channel index arithmetic.  Statistics are fp32 per
// row-chunk, reduced deterministically (no atomics) in double by a finalize kernel.
//
// Passes (training):  fwd = stats(x) -> finalize -> apply(x,res)             3 launches
//                     bwd = reduce(dy,y,x) -> finalize -> dx(dy,y,x)          3 launches
// The relu mask in backward comes from the saved output y (which the next conv already keeps
// alive for its own backward), so no mask tensor is materialised.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/bn_finalize.cuh"

namespace dtg {

long long bn_workspace_floats(long long M, int C) {
  BnGeom g = bn_geom(M, C);
  return (long long)g.nchunk * 2 * C + 4LL * C;
}

// ---- pass 1 (fwd): per-chunk sum / sum of squares ------------------------------------------
template <int TPR>
__global__ void __launch_bounds__(kBlk) bn_stats_kernel(const bf16_t* __restrict__ x, long long M, int C,
                                                        long long rpc, float* __restrict__ part) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  __shared__ float sh[2][RPP][CW + 4];
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < C) {
    long long m = m0 + ty;
    // 2-deep unroll keeps two 16B loads in flight per lane
    for (; m + RPP < m1; m += 2 * RPP) {
      float a[8], b[8];
      load8_bf16(x + m * C + c0, a);
      load8_bf16(x + (m + RPP) * C + c0, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += a[k] + b[k]; q[k] += a[k] * a[k] + b[k] * b[k]; }
    }
    if (m < m1) {
      float a[8];
      load8_bf16(x + m * C + c0, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += a[k]; q[k] += a[k] * a[k]; }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { sh[0][ty][tx * 8 + k] = s[k]; sh[1][ty][tx * 8 + k] = q[k]; }
  __syncthreads();
  for (int c = threadIdx.x; c < CW; c += kBlk) {
    float ts = 0.f, tq = 0.f;
#pragma unroll 4
    for (int r = 0; r < RPP; ++r) { ts += sh[0][r][c]; tq += sh[1][r][c]; }
    const int cc = blockIdx.y * CW + c;
    if (cc < C) {
      part[((long long)blockIdx.x * 2 + 0) * C + cc] = ts;
      part[((long long)blockIdx.x * 2 + 1) * C + cc] = tq;
    }
  }
}

// ---- pass 2 (fwd): apply scale/shift (+residual) (+relu) -------------------------------------
__device__ __forceinline__ uint8_t pos_bits8(const float (&v)[8]) {
  uint32_t b = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) b |= (v[k] > 0.f ? 1u : 0u) << k;
  return (uint8_t)b;
}

// packed relu-mask byte of this lane's 8 channels -> bits[off >> 3].  The 4 lanes tx = 4i .. 4i+3 of a row
// hold 4 consecutive bytes: with C % 32 == 0 they are gathered by two lane shuffles into one 4-byte store by
// the first of them (a byte store per lane measured ~1/5 of the apply pass's bandwidth lost)
__device__ __forceinline__ void store_bits(uint8_t* bits, long long off, const float (&v)[8], int tx, int C) {
  const uint32_t b = pos_bits8(v);
  if ((C & 31) == 0) {
    uint32_t w = b << (8 * (tx & 3));
    w |= __shfl_xor(w, 1, 64);
    w |= __shfl_xor(w, 2, 64);
    if ((tx & 3) == 0) *reinterpret_cast<uint32_t*>(bits + (off >> 3)) = w;
  } else {
    bits[off >> 3] = (uint8_t)b;
  }
}

// RU rows per loop iteration, all their loads issued before any math (the launcher picks RU = 2 with one
// iteration per thread: elementwise_rpc)
template <int TPR, bool RES, bool RELU, int RU = 4>
__global__ void __launch_bounds__(kBlk) bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                        bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                        long long M, int C, long long rpc,
                                                        uint8_t* __restrict__ bits = nullptr) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  if (c0 >= C) return;
  float sc[8], sf[8];
  load8_f32(coef + c0, sc);
  load8_f32(coef + C + c0, sf);
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  auto finish = [&](float (&a)[8], const float (&r)[8], long long off) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = a[k] * sc[k] + sf[k];
      if constexpr (RES) v += r[k];
      if constexpr (RELU) v = fmaxf(v, 0.f);
      a[k] = v;
    }
    store8_bf16(y + off, a);
    if (bits) store_bits(bits, off, a, tx, C);  // off = m*C + c0, both multiples of 8
  };
  long long m = m0 + ty;
  for (; m + (RU - 1) * RPP < m1; m += RU * RPP) {  // RU rows per iteration: every load in flight before any math
    float a[RU][8], r[RU][8];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      load8_bf16(x + (m + u * RPP) * C + c0, a[u]);
      if constexpr (RES) load8_bf16(res + (m + u * RPP) * C + c0, r[u]);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) finish(a[u], r[u], (m + u * RPP) * C + c0);
  }
  for (; m < m1; m += RPP) {
    const long long o0 = m * C + c0;
    float a0[8], r0[8];
    load8_bf16(x + o0, a0);
    if constexpr (RES) load8_bf16(res + o0, r0);
    finish(a0, r0, o0);
  }
}

// ---- fwd, projection blocks: out = relu(bn3(x) + bn_d(r)), both BNs applied in one pass ---------
template <int TPR, int RU = 4>
__global__ void __launch_bounds__(kBlk) bn_apply2_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                         bf16_t* __restrict__ y, const float* __restrict__ coef,
                                                         const float* __restrict__ coef2, long long M, int C,
                                                         long long rpc, uint8_t* __restrict__ bits) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  if (c0 >= C) return;
  float sc[8], sf[8], sc2[8], sf2[8];
  load8_f32(coef + c0, sc);
  load8_f32(coef + C + c0, sf);
  load8_f32(coef2 + c0, sc2);
  load8_f32(coef2 + C + c0, sf2);
#pragma unroll
  for (int k = 0; k < 8; ++k) sf[k] += sf2[k];
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  auto finish = [&](float (&a)[8], const float (&b)[8], long long o) {
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = fmaxf(fmaf(a[k], sc[k], fmaf(b[k], sc2[k], sf[k])), 0.f);
    store8_bf16(y + o, a);
    if (bits) store_bits(bits, o, a, tx, C);
  };
  long long m = m0 + ty;
  for (; m + (RU - 1) * RPP < m1; m += RU * RPP) {
    float a[RU][8], b[RU][8];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      load8_bf16(x + (m + u * RPP) * C + c0, a[u]);
      load8_bf16(r + (m + u * RPP) * C + c0, b[u]);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) finish(a[u], b[u], (m + u * RPP) * C + c0);
  }
  for (; m < m1; m += RPP) {
    const long long o0 = m * C + c0;
    float a0[8], b0[8];
    load8_bf16(x + o0, a0);
    load8_bf16(r + o0, b0);
    finish(a0, b0, o0);
  }
}

// ---- pass 1 (bwd): sum(dp), sum(dp*xhat), dp = dy * [y>0] -----------------------------------
template <int TPR, bool RELU>
__global__ void __launch_bounds__(kBlk) bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ y,
                                                             const bf16_t* __restrict__ x,
                                                             const float* __restrict__ smean,
                                                             const float* __restrict__ sinv, long long M, int C,
                                                             long long rpc, float* __restrict__ part) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  __shared__ float sh[2][RPP][CW + 4];
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c0 < C) {
    float mu[8], is[8];
    load8_f32(smean + c0, mu);
    load8_f32(sinv + c0, is);
    const long long m0 = (long long)blockIdx.x * rpc;
    const long long m1 = m0 + rpc < M ? m0 + rpc : M;
    auto acc = [&](float (&g)[8], const float (&xv)[8], const float (&yv)[8]) {
      if constexpr (RELU) {
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[k] += g[k]; q[k] += g[k] * (xv[k] - mu[k]) * is[k]; }
    };
    long long m = m0 + ty;
    for (; m + RPP < m1; m += 2 * RPP) {
      const long long o0 = m * C + c0, o1 = (m + RPP) * C + c0;
      float g0[8], g1[8], x0[8], x1[8], y0[8], y1[8];
      load8_bf16(dy + o0, g0);
      load8_bf16(dy + o1, g1);
      load8_bf16(x + o0, x0);
      load8_bf16(x + o1, x1);
      if constexpr (RELU) {
        load8_bf16(y + o0, y0);
        load8_bf16(y + o1, y1);
      }
      acc(g0, x0, y0);
      acc(g1, x1, y1);
    }
    if (m < m1) {
      const long long o0 = m * C + c0;
      float g0[8], x0[8], y0[8];
      load8_bf16(dy + o0, g0);
      load8_bf16(x + o0, x0);
      if constexpr (RELU) load8_bf16(y + o0, y0);
      acc(g0, x0, y0);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { sh[0][ty][tx * 8 + k] = s[k]; sh[1][ty][tx * 8 + k] = q[k]; }
  __syncthreads();
  for (int c = threadIdx.x; c < CW; c += kBlk) {
    float ts = 0.f, tq = 0.f;
#pragma unroll 4
    for (int r = 0; r < RPP; ++r) { ts += sh[0][r][c]; tq += sh[1][r][c]; }
    const int cc = blockIdx.y * CW + c;
    if (cc < C) {
      part[((long long)blockIdx.x * 2 + 0) * C + cc] = ts;
      part[((long long)blockIdx.x * 2 + 1) * C + cc] = tq;
    }
  }
}

// ---- pass 2 (bwd): dx = a*dp + bx*x + c0 ; dres = dp ------------------------------------------
template <int TPR, bool RELU, bool DRES, bool NT = true, int RU = 4>
__global__ void __launch_bounds__(kBlk) bn_bwd_dx_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                         const bf16_t* __restrict__ x, const float* __restrict__ coef,
                                                         bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                                         long long M, int C, long long rpc) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  if (c0 >= C) return;
  float a[8], bx[8], cc[8];
  load8_f32(coef + c0, a);
  load8_f32(coef + C + c0, bx);
  load8_f32(coef + 2 * C + c0, cc);
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  auto finish = [&](float (&g)[8], const float (&xv)[8], const float (&yv)[8], long long off) {
    if constexpr (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = yv[k] > 0.f ? g[k] : 0.f;
    }
    if constexpr (DRES) store8_bf16(dres + off, g);
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = a[k] * g[k] + bx[k] * xv[k] + cc[k];
    store8_bf16(dx + off, o);
  };
  // dp and the saved BN input are read for the last time in this step: non-temporal, so the dx written
  // here stays cached for the dgrad / wgrad GEMMs that read it next
  auto ld = [&](const bf16_t* p, float (&v)[8]) {
    if constexpr (NT) load8_bf16_nt(p, v);
    else load8_bf16(p, v);
  };
  long long m = m0 + ty;
  for (; m + (RU - 1) * RPP < m1; m += RU * RPP) {  // RU rows per iteration, every load in flight first
    float g[RU][8], xv[RU][8], yv[RU][8];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long long o = (m + u * RPP) * C + c0;
      ld(dy + o, g[u]);
      ld(x + o, xv[u]);
      if constexpr (RELU) load8_bf16(y + o, yv[u]);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) finish(g[u], xv[u], yv[u], (m + u * RPP) * C + c0);
  }
  for (; m < m1; m += RPP) {
    const long long o0 = m * C + c0;
    float g0[8], x0[8], y0[8];
    ld(dy + o0, g0);
    ld(x + o0, x0);
    if constexpr (RELU) load8_bf16(y + o0, y0);
    finish(g0, x0, y0, o0);
  }
}

// RU = 2 rows per loop iteration of the streaming passes: with elementwise_rpc's two rows per thread, one
// iteration with every load in flight, then the stores
#define DTG_RU_SWITCH(...) \
  { constexpr int RU = 2; __VA_ARGS__; }

// ---------------------------------------------------------------------------------------------
static void bn_apply_launch(const BnGeom& g, const bf16_t* x, const bf16_t* res, bf16_t* y, const float* coef,
                            long long M, int C, int relu, hipStream_t st, uint8_t* bits = nullptr) {
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  DTG_TPR_SWITCH(g.tpr, DTG_RU_SWITCH({
    if (res) {
      if (relu) { bn_apply_kernel<T, true, true, RU><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa, bits); DTG_LAUNCH_CHECK(); }
      else { bn_apply_kernel<T, true, false, RU><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa, bits); DTG_LAUNCH_CHECK(); }
    } else {
      if (relu) { bn_apply_kernel<T, false, true, RU><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa, bits); DTG_LAUNCH_CHECK(); }
      else { bn_apply_kernel<T, false, false, RU><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa, bits); DTG_LAUNCH_CHECK(); }
    }
  }));
}

void bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                  float* rmean, float* rvar, float* smean, float* sinv, float* ws, long long M, int C,
                  float momentum, float eps, int relu, hipStream_t st) {
  const BnGeom g = bn_geom(M, C);
  float* part = ws;
  float* coef = ws + (long long)g.nchunk * 2 * C;
  dim3 grid(g.nchunk, g.gy);
  DTG_TPR_SWITCH(g.tpr, bn_stats_kernel<T><<<grid, kBlk, 0, st>>>(x, M, C, g.rows_per_chunk, part)); DTG_LAUNCH_CHECK();
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, g.nchunk, M, C, 0, gamma, beta, rmean, rvar, smean, sinv,
                                                    momentum, eps, coef, nullptr, nullptr); DTG_LAUNCH_CHECK();
  bn_apply_launch(g, x, res, y, coef, M, C, relu, st);
}

// Statistics already reduced by a GEMM / conv epilogue (kBnStatSlots partials): finalize + apply.
void bn_fwd_from_part(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                      float* rmean, float* rvar, float* smean, float* sinv, const float* part, float* ws, long long M,
                      int C, float momentum, float eps, int relu, hipStream_t st, uint8_t* bits) {
  const BnGeom g = bn_geom(M, C);
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, kBnStatSlots, M, C, 0, gamma, beta, rmean, rvar, smean,
                                                    sinv, momentum, eps, ws, nullptr, nullptr, 1); DTG_LAUNCH_CHECK();
  bn_apply_launch(g, x, res, y, ws, M, C, relu, st, bits);
}

// Inference: coefficients from running statistics (tiny launch) then the same apply pass.
__global__ void bn_infer_coef_kernel(const float* gamma, const float* beta, const float* rmean, const float* rvar,
                                     float eps, int C, float* coef) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rvar[c] + eps);
  const float sc = (gamma ? gamma[c] : 1.f) * inv;
  coef[c] = sc;
  coef[C + c] = (beta ? beta[c] : 0.f) - rmean[c] * sc;
}

void bn_fwd_infer(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                  const float* rmean, const float* rvar, float* ws, long long M, int C, float eps, int relu,
                  hipStream_t st) {
  const BnGeom g = bn_geom(M, C);
  float* coef = ws;
  bn_infer_coef_kernel<<<(C + 255) / 256, 256, 0, st>>>(gamma, beta, rmean, rvar, eps, C, coef); DTG_LAUNCH_CHECK();
  dim3 grid(g.nchunk, g.gy);
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  DTG_TPR_SWITCH(g.tpr, {
    if (res) {
      if (relu) { bn_apply_kernel<T, true, true><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa); DTG_LAUNCH_CHECK(); }
      else { bn_apply_kernel<T, true, false><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa); DTG_LAUNCH_CHECK(); }
    } else {
      if (relu) { bn_apply_kernel<T, false, true><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa); DTG_LAUNCH_CHECK(); }
      else { bn_apply_kernel<T, false, false><<<ga, kBlk, 0, st>>>(x, res, y, coef, M, C, rpa); DTG_LAUNCH_CHECK(); }
    }
  });
}

void bn_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* gamma, const float* smean,
            const float* sinv, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* ws, long long M, int C,
            int relu, int accum, hipStream_t st) {
  const BnGeom g = bn_geom(M, C);
  float* part = ws;
  float* coef = ws + (long long)g.nchunk * 2 * C;
  dim3 grid(g.nchunk, g.gy);
  DTG_TPR_SWITCH(g.tpr, {
    if (relu) { bn_bwd_reduce_kernel<T, true><<<grid, kBlk, 0, st>>>(dy, y, x, smean, sinv, M, C, g.rows_per_chunk, part); DTG_LAUNCH_CHECK(); }
    else { bn_bwd_reduce_kernel<T, false><<<grid, kBlk, 0, st>>>(dy, y, x, smean, sinv, M, C, g.rows_per_chunk, part); DTG_LAUNCH_CHECK(); }
  });
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, g.nchunk, M, C, accum ? 2 : 1, gamma, nullptr, nullptr, nullptr,
                                                    const_cast<float*>(smean), const_cast<float*>(sinv), 0.f, 0.f,
                                                    coef, dgamma, dbeta); DTG_LAUNCH_CHECK();
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  DTG_TPR_SWITCH(g.tpr, {
    if (relu) {
      if (dres) { bn_bwd_dx_kernel<T, true, true><<<ga, kBlk, 0, st>>>(dy, y, x, coef, dx, dres, M, C, rpa); DTG_LAUNCH_CHECK(); }
      else { bn_bwd_dx_kernel<T, true, false><<<ga, kBlk, 0, st>>>(dy, y, x, coef, dx, dres, M, C, rpa); DTG_LAUNCH_CHECK(); }
    } else {
      if (dres) { bn_bwd_dx_kernel<T, false, true><<<ga, kBlk, 0, st>>>(dy, y, x, coef, dx, dres, M, C, rpa); DTG_LAUNCH_CHECK(); }
      else { bn_bwd_dx_kernel<T, false, false><<<ga, kBlk, 0, st>>>(dy, y, x, coef, dx, dres, M, C, rpa); DTG_LAUNCH_CHECK(); }
    }
  });
}

// Two BNs from epilogue partials applied in one pass: y = relu(bn(x) + bn2(r)) (projection blocks).
void bn_fwd2_from_part(const bf16_t* x, const bf16_t* r, bf16_t* y, const float* part, const float* part2,
                       const float* gamma, const float* beta, float* rmean, float* rvar, float* smean, float* sinv,
                       const float* gamma2, const float* beta2, float* rmean2, float* rvar2, float* smean2,
                       float* sinv2, float* ws, long long M, int C, float momentum, float eps, hipStream_t st,
                       uint8_t* bits) {
  const BnGeom g = bn_geom(M, C);
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, kBnStatSlots, M, C, 0, gamma, beta, rmean, rvar, smean,
                                                    sinv, momentum, eps, ws, nullptr, nullptr, 1); DTG_LAUNCH_CHECK();
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part2, kBnStatSlots, M, C, 0, gamma2, beta2, rmean2, rvar2,
                                                    smean2, sinv2, momentum, eps, ws + 2LL * C, nullptr, nullptr, 1); DTG_LAUNCH_CHECK();
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  DTG_TPR_SWITCH(g.tpr, DTG_RU_SWITCH(bn_apply2_kernel<T, RU><<<ga, kBlk, 0, st>>>(x, r, y, ws, ws + 2LL * C, M, C, rpa,
                                                                                 bits))); DTG_LAUNCH_CHECK();
}

// ---- bwd, projection blocks: dx = a*dp + bx*x + c0 and dx2 = a2*dp + bx2*x2 + c02, one read of dp -----
template <int TPR, int RU = 4>
__global__ void __launch_bounds__(kBlk) bn_bwd_dx2_kernel(const bf16_t* __restrict__ dp, const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ x2,
                                                          const float* __restrict__ coef,
                                                          const float* __restrict__ coef2, bf16_t* __restrict__ dx,
                                                          bf16_t* __restrict__ dx2, long long M, int C, long long rpc) {
  constexpr int RPP = kBlk / TPR, CW = TPR * 8;
  const int tx = threadIdx.x % TPR, ty = threadIdx.x / TPR;
  const int c0 = blockIdx.y * CW + tx * 8;
  if (c0 >= C) return;
  float a[8], bx[8], cc[8], a2[8], bx2[8], cc2[8];
  load8_f32(coef + c0, a);
  load8_f32(coef + C + c0, bx);
  load8_f32(coef + 2 * C + c0, cc);
  load8_f32(coef2 + c0, a2);
  load8_f32(coef2 + C + c0, bx2);
  load8_f32(coef2 + 2 * C + c0, cc2);
  const long long m0 = (long long)blockIdx.x * rpc;
  const long long m1 = m0 + rpc < M ? m0 + rpc : M;
  auto finish = [&](const float (&g)[8], const float (&xv)[8], const float (&x2v)[8], long long o) {
    float o1[8], o2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o1[k] = fmaf(a[k], g[k], fmaf(bx[k], xv[k], cc[k]));
      o2[k] = fmaf(a2[k], g[k], fmaf(bx2[k], x2v[k], cc2[k]));
    }
    store8_bf16(dx + o, o1);
    store8_bf16(dx2 + o, o2);
  };
  long long m = m0 + ty;
  for (; m + (RU - 1) * RPP < m1; m += RU * RPP) {
    float g[RU][8], xv[RU][8], x2v[RU][8];
#pragma unroll
    for (int u = 0; u < RU; ++u) {
      const long long o = (m + u * RPP) * C + c0;
      load8_bf16(dp + o, g[u]);
      load8_bf16(x + o, xv[u]);
      load8_bf16(x2 + o, x2v[u]);
    }
#pragma unroll
    for (int u = 0; u < RU; ++u) finish(g[u], xv[u], x2v[u], (m + u * RPP) * C + c0);
  }
  for (; m < m1; m += RPP) {
    const long long o = m * C + c0;
    float g[8], xv[8], x2v[8];
    load8_bf16(dp + o, g);
    load8_bf16(x + o, xv);
    load8_bf16(x2 + o, x2v);
    finish(g, xv, x2v, o);
  }
}

void bn_bwd2_from_part(const bf16_t* dp, const bf16_t* x, const bf16_t* x2, const float* part, const float* part2,
                       const float* gamma, const float* smean, const float* sinv, const float* gamma2,
                       const float* smean2, const float* sinv2, bf16_t* dx, bf16_t* dx2, float* dgamma, float* dbeta,
                       float* dgamma2, float* dbeta2, float* ws, long long M, int C, int accum, hipStream_t st) {
  const BnGeom g = bn_geom(M, C);
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, kBnStatSlots, M, C, accum ? 2 : 1, gamma, nullptr, nullptr,
                                                    nullptr, const_cast<float*>(smean), const_cast<float*>(sinv), 0.f,
                                                    0.f, ws, dgamma, dbeta, 1); DTG_LAUNCH_CHECK();
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part2, kBnStatSlots, M, C, accum ? 2 : 1, gamma2, nullptr,
                                                    nullptr, nullptr, const_cast<float*>(smean2),
                                                    const_cast<float*>(sinv2), 0.f, 0.f, ws + 3LL * C, dgamma2,
                                                    dbeta2, 1); DTG_LAUNCH_CHECK();
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  DTG_TPR_SWITCH(g.tpr, DTG_RU_SWITCH(bn_bwd_dx2_kernel<T, RU><<<ga, kBlk, 0, st>>>(dp, x, x2, ws, ws + 3LL * C, dx,
                                                                                   dx2, M, C, rpa))); DTG_LAUNCH_CHECK();
}

// Backward from mode-2 epilogue partials: dp is already relu-masked, so the dx pass reads dp and x.
// Two halves, also callable on their own (the BN-folded 1x1 dgrads, models/resnet_fused.py): the finalize
// turns the partials into dgamma / dbeta and coef = [a, bx, c] with dx = a*dp + bx*x + c per channel ...
void bn_bwd_coef_from_part(const float* part, const float* gamma, const float* smean, const float* sinv, float* coef,
                           float* dgamma, float* dbeta, long long M, int C, int accum, hipStream_t st) {
  bn_finalize_kernel<16><<<(C + 63) / 64, 1024, 0, st>>>(part, kBnStatSlots, M, C, accum ? 2 : 1, gamma, nullptr, nullptr,
                                                    nullptr, const_cast<float*>(smean), const_cast<float*>(sinv), 0.f,
                                                    0.f, coef, dgamma, dbeta, 1); DTG_LAUNCH_CHECK();
}

// ... and the dx pass applies them (one read of dp and x, one write of dx; dres: a copy of dp)
void bn_dx_from_coef(const bf16_t* dp, const bf16_t* x, const float* coef, bf16_t* dx, bf16_t* dres, long long M, int C,
                     hipStream_t st) {
  const BnGeom g = bn_geom(M, C);
  const long long rpa = elementwise_rpc(g, M);
  dim3 ga((unsigned)((M + rpa - 1) / rpa), g.gy);
  const float* ws = coef;
  DTG_TPR_SWITCH(g.tpr, DTG_RU_SWITCH({
    if (dres) { bn_bwd_dx_kernel<T, false, true, true, RU><<<ga, kBlk, 0, st>>>(dp, nullptr, x, ws, dx, dres, M, C,
                                                                                      rpa); DTG_LAUNCH_CHECK(); }
    else { bn_bwd_dx_kernel<T, false, false, true, RU><<<ga, kBlk, 0, st>>>(dp, nullptr, x, ws, dx, dres, M, C, rpa); DTG_LAUNCH_CHECK(); }
  }));
}

void bn_bwd_from_part(const bf16_t* dp, const bf16_t* x, const float* gamma, const float* smean, const float* sinv,
                      const float* part, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* ws, long long M,
                      int C, int accum, hipStream_t st) {
  bn_bwd_coef_from_part(part, gamma, smean, sinv, ws, dgamma, dbeta, M, C, accum, st);
  bn_dx_from_coef(dp, x, ws, dx, dres, M, C, st);
}

}  // namespace dtg
