// BatchNorm host geometry (rows x channel-slab decomposition) and the statistics finalize kernel,
// shared by batchnorm.hip and the fused stem kernels (stem.hip).
#pragma once
#include <stdlib.h>
#include "dtg/common.h"

namespace dtg {

constexpr int kBlk = 512;   // 8 waves: RPP = 512/TPR rows in flight per block

struct BnGeom {
  int tpr;    // threads per row (8 channels each)
  int cw;     // channels per block slab
  int gy;     // slabs
  int nchunk; // row chunks
  long long rows_per_chunk;
};

inline BnGeom bn_geom(long long M, int C) {
  BnGeom g;
  const int cw_need = C < 512 ? C : 512;
  g.tpr = 8;
  while (g.tpr * 8 < cw_need && g.tpr < 64) g.tpr *= 2;
  g.cw = g.tpr * 8;
  g.gy = (C + g.cw - 1) / g.cw;
  const int rpp = kBlk / g.tpr;
  long long max_chunks = (M + rpp - 1) / rpp;
  // <= 256 row chunks: keeps the finalize reduction short (<= 16 partials per finalize lane)
  long long nc = 256 / g.gy;
  if (nc < 1) nc = 1;
  if (nc > max_chunks) nc = max_chunks;
  g.rows_per_chunk = (M + nc - 1) / nc;
  g.nchunk = (int)((M + g.rows_per_chunk - 1) / g.rows_per_chunk);
  return g;
}

// The elementwise passes (apply, dx) write no partials, so their grid is free: each workgroup takes
// 2 x RPP rows, i.e. every thread streams exactly two rows of its 8 channels (all loads in flight, then the
// stores) and exits.  Measured against the previous ~2048 long-running workgroups (tools/bn_bench.py,
// profiles/r03_bn_grid): ResNet-50's largest apply+residual pass 5.0 -> 5.7 TB/s, its dx pass 5.1 -> 6.2
// TB/s, i.e. the 6.0 TB/s of a plain torch.add moving the same bytes.
inline long long elementwise_rpc(const BnGeom& g, long long M) {
  (void)M;
  return 2LL * (kBlk / g.tpr);
}

// ---- finalize: reduce chunk partials (double), emit per-channel coefficients -----------------
// mode 0 (fwd):  out0 = scale = gamma*invstd, out1 = shift = beta - mean*scale,
//                save_mean/save_invstd, running stats update.
// mode 1 (bwd):  a = gamma*invstd; dgamma = sum(dp*xhat), dbeta = sum(dp);
//                dx = a*dp + bx*x + c0   with bx = -a*invstd*dgamma/M, c0 = -a*dbeta/M - bx*mean
// G chunk groups per channel (16 = 1024 threads; 4 = 256 threads measured slower for the 32 epilogue
// slots too: the kernel is latency-, not occupancy-bound)
template <int G = 16>
__global__ void __launch_bounds__(64 * G) bn_finalize_kernel(const float* __restrict__ part, int nchunk, long long M,
                                                           int C, int mode, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, float* __restrict__ rmean,
                                                           float* __restrict__ rvar, float* __restrict__ smean,
                                                           float* __restrict__ sinv, float momentum, float eps,
                                                           float* __restrict__ coef, float* __restrict__ dgamma,
                                                           float* __restrict__ dbeta, int zero_after = 0) {
  __shared__ double sh[2][G][64];
  const int cl = threadIdx.x % 64, r = threadIdx.x / 64;
  const int c = blockIdx.x * 64 + cl;
  float s0 = 0.f, s1 = 0.f, q0 = 0.f, q1 = 0.f;  // two independent chains per sum
  if (c < C) {
    int k = r;
    for (; k + G < nchunk; k += 2 * G) {
      s0 += part[((long long)k * 2 + 0) * C + c];
      q0 += part[((long long)k * 2 + 1) * C + c];
      s1 += part[((long long)(k + G) * 2 + 0) * C + c];
      q1 += part[((long long)(k + G) * 2 + 1) * C + c];
    }
    if (k < nchunk) {
      s0 += part[((long long)k * 2 + 0) * C + c];
      q0 += part[((long long)k * 2 + 1) * C + c];
    }
    if (zero_after) {  // epilogue-statistics slots come from a reused pool: leave them zeroed
      float* pz = const_cast<float*>(part);
      for (int kk = r; kk < nchunk; kk += G) {
        pz[((long long)kk * 2 + 0) * C + c] = 0.f;
        pz[((long long)kk * 2 + 1) * C + c] = 0.f;
      }
    }
  }
  sh[0][r][cl] = (double)s0 + (double)s1;
  sh[1][r][cl] = (double)q0 + (double)q1;
  __syncthreads();
  double s = 0.0, q = 0.0;
  if (r == 0) {
#pragma unroll
    for (int j = 0; j < G; ++j) { s += sh[0][j][cl]; q += sh[1][j][cl]; }
  }
  if (r != 0 || c >= C) return;
  const double invM = 1.0 / (double)M;
  const float g = gamma ? gamma[c] : 1.f;
  if (mode == 0) {
    const double mean = s * invM;
    double var = q * invM - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = g * invstd;
    coef[c] = sc;
    coef[C + c] = (beta ? beta[c] : 0.f) - (float)mean * sc;
    if (smean) smean[c] = (float)mean;
    if (sinv) sinv[c] = invstd;
    if (rmean) rmean[c] = (1.f - momentum) * rmean[c] + momentum * (float)mean;
    if (rvar) {
      const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  } else {
    // s = sum(dp), q = sum(dp * xhat)
    const float mean = smean[c], invstd = sinv[c];
    const float a = g * invstd;
    const float bx = (float)(-(double)a * invstd * q * invM);
    const float c0 = (float)(-(double)a * s * invM) - bx * mean;
    coef[c] = a;
    coef[C + c] = bx;
    coef[2 * C + c] = c0;
    // mode 2 accumulates into persistent (flat-buffer) gradients instead of overwriting
    if (dgamma) dgamma[c] = (mode == 2 ? dgamma[c] : 0.f) + (float)q;
    if (dbeta) dbeta[c] = (mode == 2 ? dbeta[c] : 0.f) + (float)s;
  }
}

}  // namespace dtg

#define DTG_TPR_SWITCH(tpr, ...)                       \
  switch (tpr) {                                       \
    case 8: { constexpr int T = 8; __VA_ARGS__; } break;   \
    case 16: { constexpr int T = 16; __VA_ARGS__; } break; \
    case 32: { constexpr int T = 32; __VA_ARGS__; } break; \
    default: { constexpr int T = 64; __VA_ARGS__; } break; \
  }
