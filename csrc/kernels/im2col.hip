// im2col / col2im for NHWC convolutions whose channel count the implicit-GEMM kernels do not
// cover (C % 64 != 0: MNIST's 1- and 32-channel inputs, tiny stems).  The convolution itself then
// runs on the MFMA GEMM (gemm.hip) with its fused bias/ReLU epilogue:
//   fwd    y[NPQ, K]  = cols[NPQ, Kp] W[K, Kp]^T          (Kp = R*S*C rounded up to 8, zero pad)
//   wgrad  dW[K, Kp]  = dy^T cols
//   dgrad  dcols      = dy W;  dx = col2im(dcols)          (gather form: no atomics)
// Column order inside a row is (r, s, c) with c fastest = the [K][R][S][C] weight layout.
#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

struct ColGeom {
  int N, H, W, C, R, S, stride, pad, P, Q, Kp;
};

// one thread per (row m, column kk); 8 columns at a time when C % 8 == 0 (then an 8-group never
// straddles two taps)
template <bool VEC>
__global__ void __launch_bounds__(256) im2col_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ cols,
                                                     ColGeom g) {
  const int per = VEC ? 8 : 1;
  const int groups = g.Kp / per;
  const long long total = (long long)g.N * g.P * g.Q * groups;
  const int RSC = g.R * g.S * g.C;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int kg = (int)(i % groups);
    const long long m = i / groups;
    const int q = (int)(m % g.Q);
    const long long t = m / g.Q;
    const int p = (int)(t % g.P);
    const int n = (int)(t / g.P);
    const int kk = kg * per;
    bf16_t* dst = cols + m * g.Kp + kk;
    if (VEC) {
      float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (kk < RSC) {
        const int c = kk % g.C, rs = kk / g.C, s = rs % g.S, r = rs / g.S;
        const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
        if (h >= 0 && h < g.H && w >= 0 && w < g.W) load8_bf16(x + (((long long)n * g.H + h) * g.W + w) * g.C + c, v);
      }
      store8_bf16(dst, v);
    } else {
      bf16_t v = 0;
      if (kk < RSC) {
        const int c = kk % g.C, rs = kk / g.C, s = rs % g.S, r = rs / g.S;
        const int h = p * g.stride - g.pad + r, w = q * g.stride - g.pad + s;
        if (h >= 0 && h < g.H && w >= 0 && w < g.W) v = x[(((long long)n * g.H + h) * g.W + w) * g.C + c];
      }
      *dst = v;
    }
  }
}

// dx[n,h,w,c] = sum over taps (r,s) whose output (p,q) exists of dcols[(n,p,q), (r,s,c)]
template <bool VEC>
__global__ void __launch_bounds__(256) col2im_kernel(const bf16_t* __restrict__ dcols, bf16_t* __restrict__ dx,
                                                     ColGeom g) {
  const int per = VEC ? 8 : 1;
  const int cg = g.C / per;
  const long long total = (long long)g.N * g.H * g.W * cg;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cg) * per;
    long long t = i / cg;
    const int w = (int)(t % g.W);
    t /= g.W;
    const int h = (int)(t % g.H);
    const int n = (int)(t / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = 0; r < g.R; ++r) {
      const int hp = h + g.pad - r;
      if (hp < 0 || hp % g.stride) continue;
      const int p = hp / g.stride;
      if (p >= g.P) continue;
      for (int s = 0; s < g.S; ++s) {
        const int wp = w + g.pad - s;
        if (wp < 0 || wp % g.stride) continue;
        const int q = wp / g.stride;
        if (q >= g.Q) continue;
        const bf16_t* src = dcols + (((long long)n * g.P + p) * g.Q + q) * g.Kp + (r * g.S + s) * g.C + c;
        if (VEC) {
          float v[8];
          load8_bf16(src, v);
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[k] += v[k];
        } else {
          acc[0] += bf2f(*src);
        }
      }
    }
    bf16_t* d = dx + (((long long)n * g.H + h) * g.W + w) * g.C + c;
    if (VEC) store8_bf16(d, acc);
    else *d = f2bf(acc[0]);
  }
}

static ColGeom col_geom(int N, int H, int W, int C, int R, int S, int stride, int pad, int Kp) {
  ColGeom g{N, H, W, C, R, S, stride, pad, (H + 2 * pad - R) / stride + 1, (W + 2 * pad - S) / stride + 1, Kp};
  return g;
}

void im2col(const bf16_t* x, bf16_t* cols, int N, int H, int W, int C, int R, int S, int stride, int pad, int Kp,
            hipStream_t st) {
  ColGeom g = col_geom(N, H, W, C, R, S, stride, pad, Kp);
  const bool vec = (C % 8 == 0) && (Kp % 8 == 0);
  const long long total = (long long)N * g.P * g.Q * (vec ? Kp / 8 : Kp);
  if (vec) { hipLaunchKernelGGL(im2col_kernel<true>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, x, cols, g); DTG_LAUNCH_CHECK(); }
  else { hipLaunchKernelGGL(im2col_kernel<false>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, x, cols, g); DTG_LAUNCH_CHECK(); }
}

void col2im(const bf16_t* dcols, bf16_t* dx, int N, int H, int W, int C, int R, int S, int stride, int pad, int Kp,
            hipStream_t st) {
  ColGeom g = col_geom(N, H, W, C, R, S, stride, pad, Kp);
  const bool vec = (C % 8 == 0) && (Kp % 8 == 0);
  const long long total = (long long)N * H * W * (vec ? C / 8 : C);
  if (vec) { hipLaunchKernelGGL(col2im_kernel<true>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, dcols, dx, g); DTG_LAUNCH_CHECK(); }
  else { hipLaunchKernelGGL(col2im_kernel<false>, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, dcols, dx, g); DTG_LAUNCH_CHECK(); }
}

}  // namespace dtg
