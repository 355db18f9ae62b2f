// NHWC bf16 pooling (ResNet stem max-pool 3x3/2, MNIST 2x2/2 max-pool, global average pool).
// A thread owns 8 consecutive channels (one 16-byte vector) of one output/input pixel.
//   max-pool fwd: y = max over the window, plus the window index of the max per element (uint8)
//   max-pool bwd: gather form -- every input pixel visits the <= ceil(k/s)^2 outputs whose window
//                 covers it and adds dy where the saved index points back at it: no atomics, no
//                 zero-fill pass, deterministic.
//   avg-pool:     fwd reduces H*W per (n, c8); bwd broadcasts dy / (H*W).
#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

struct PoolGeom {
  int N, H, W, C, P, Q, k, s, pad;
};

__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeom g) {
  const unsigned c8n = g.C >> 3;
  const unsigned total = (unsigned)g.N * g.P * g.Q * c8n;  // < 2^31 (host check): 32-bit index math
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % c8n);
    unsigned t = i / c8n;
    const int q = (int)(t % (unsigned)g.Q);
    t /= (unsigned)g.Q;
    const int p = (int)(t % (unsigned)g.P);
    const int n = (int)(t / (unsigned)g.P);
    float m[8];
    uint8_t am[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      m[k] = -INFINITY;
      am[k] = 0;
    }
    const int h0 = p * g.s - g.pad, w0 = q * g.s - g.pad;
    for (int r = 0; r < g.k; ++r) {
      const int h = h0 + r;
      if (h < 0 || h >= g.H) continue;
      for (int c = 0; c < g.k; ++c) {
        const int w = w0 + c;
        if (w < 0 || w >= g.W) continue;
        float v[8];
        load8_bf16(x + (((long long)n * g.H + h) * g.W + w) * g.C + c8 * 8, v);
        const uint8_t wi = (uint8_t)(r * g.k + c);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (v[k] > m[k]) {  // strict: the first maximum in window order wins ties
            m[k] = v[k];
            am[k] = wi;
          }
      }
    }
    const long long o = (((long long)n * g.P + p) * g.Q + q) * g.C + c8 * 8;
    store8_bf16(y + o, m);
    if (idx) {
      uint2 pk;
      pk.x = am[0] | (am[1] << 8) | (am[2] << 16) | ((uint32_t)am[3] << 24);
      pk.y = am[4] | (am[5] << 8) | (am[6] << 16) | ((uint32_t)am[7] << 24);
      *reinterpret_cast<uint2*>(idx + o) = pk;
    }
  }
}

__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const bf16_t* __restrict__ dy,
                                                          const uint8_t* __restrict__ idx, bf16_t* __restrict__ dx,
                                                          PoolGeom g) {
  const unsigned c8n = g.C >> 3;
  const unsigned total = (unsigned)g.N * g.H * g.W * c8n;  // < 2^31 (host check): 32-bit index math
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int c8 = (int)(i % c8n);
    unsigned t = i / c8n;
    const int w = (int)(t % (unsigned)g.W);
    t /= (unsigned)g.W;
    const int h = (int)(t % (unsigned)g.H);
    const int n = (int)(t / (unsigned)g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // outputs p with p*s - pad <= h <= p*s - pad + k - 1
    const int hp = h + g.pad, wp = w + g.pad;
    const int p_lo = hp >= g.k ? (hp - g.k) / g.s + 1 : 0, p_hi = min(g.P - 1, hp / g.s);
    const int q_lo = wp >= g.k ? (wp - g.k) / g.s + 1 : 0, q_hi = min(g.Q - 1, wp / g.s);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = hp - p * g.s;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int c = wp - q * g.s;
        const uint8_t wi = (uint8_t)(r * g.k + c);
        const long long o = (((long long)n * g.P + p) * g.Q + q) * g.C + c8 * 8;
        const uint2 pk = *reinterpret_cast<const uint2*>(idx + o);
        float d[8];
        load8_bf16(dy + o, d);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t word = k < 4 ? pk.x : pk.y;
          if (((word >> (8 * (k & 3))) & 0xff) == wi) acc[k] += d[k];
        }
      }
    }
    store8_bf16(dx + (((long long)n * g.H + h) * g.W + w) * g.C + c8 * 8, acc);
  }
}

// y[n, c] = mean over H*W of x[n, :, :, c]; block = (n, 256 channel-vectors... ) -- one thread per (n, c8)
// with 8 row-partials combined through LDS.
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                          int N, int HW, int C) {
  __shared__ float red[8][32 * 8 + 4];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int n = blockIdx.y;
  const int c8 = blockIdx.x * 32 + cl;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (c8 * 8 < C)
    for (int r = rl; r < HW; r += 8) {
      float v[8];
      load8_bf16(x + ((long long)n * HW + r) * C + c8 * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v[k];
    }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[rl][cl * 8 + k] = acc[k];
  __syncthreads();
  if (rl == 0 && c8 * 8 < C) {
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += red[r][cl * 8 + k];
      o[k] = t / HW;
    }
    store8_bf16(y + (long long)n * C + c8 * 8, o);
  }
}

__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx,
                                                          int N, int HW, int C) {
  const int c8n = C >> 3;
  const long long total = (long long)N * HW * c8n;
  const float inv = 1.f / HW;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % c8n);
    const int n = (int)(i / c8n / HW);
    float d[8];
    load8_bf16(dy + (long long)n * C + c8 * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] *= inv;
    store8_bf16(dx + i * 8, d);
  }
}

void maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int k, int s, int pad, int P,
                 int Q, hipStream_t st) {
  PoolGeom g{N, H, W, C, P, Q, k, s, pad};
  const long long total = (long long)N * P * Q * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, x, y, idx, g); DTG_LAUNCH_CHECK();
}

void maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int k, int s, int pad,
                 int P, int Q, hipStream_t st) {
  PoolGeom g{N, H, W, C, P, Q, k, s, pad};
  const long long total = (long long)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, dy, idx, dx, g); DTG_LAUNCH_CHECK();
}

void avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((C / 8 + 31) / 32, N), dim3(256), 0, st, x, y, N, HW, C); DTG_LAUNCH_CHECK();
}

void avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st) {
  const long long total = (long long)N * HW * (C / 8);
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, dy, dx, N, HW, C); DTG_LAUNCH_CHECK();
}

}  // namespace dtg
