// Experimental (round 3): 3x3 / stride 1 / pad 1 convolution for 64 input and 64 output channels (ResNet-50's
// layer-1 conv2, NHWC bf16) as a DIRECT convolution from an LDS halo tile, to test whether the implicit-GEMM
// kernel's L2 traffic is what limits it (profiles/r03_conv_l2: the implicit GEMM gathers every input pixel once
// per filter tap, 9x through L2, with the L2 channels busy 94 % of every cycle).
//
// One workgroup (4 waves) = one band of TH = 4 output rows of one image (4 x W pixels, W <= 60) x all 64 output
// channels.  The band's input rows with their 1-pixel halo, (TH + 2) x (W + 2) pixels x 64 channels, are staged
// ONCE into LDS (zeros outside the image), together with all 9 taps of the weights; every tap's A fragments are
// then read from the halo at the shifted pixel, so each input byte crosses L2 about (TH + 2) / TH times instead
// of 9.  Layout of both LDS images: [pixel or output channel][64 channels] with the 16-byte chunk XOR-swizzled
// by (row & 7), as frag_kc reads it.  Output through an LDS staging pass as 16-byte stores.
#include <stdlib.h>

#include "dtg/common.h"
#include "dtg/kernels.h"
#include "lab.h"
#include "dtg/mfma_gemm.cuh"

namespace dtg {
using namespace gemm;

namespace {

constexpr int kTH = 4, kC = 64;

__device__ __forceinline__ int swz_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

// WGLB: the weight fragments come straight from global memory (L1/L2-resident, 72 KB), one tap ahead in
// registers, so the LDS holds only the halo (44.5 KB at W = 56: three workgroups per CU instead of one)
template <bool WGLB>
__global__ void __launch_bounds__(256) conv3x3_halo_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                          bf16_t* __restrict__ y, int N, int H, int W) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int HW2 = W + 2;
  const int halo_px = (kTH + 2) * HW2;
  lds_char* halo = smem;                      // [halo_px][64]
  lds_char* wt = smem + halo_px * 128;        // [9][64 k][64 c]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bands = H / kTH;
  const int n = blockIdx.x / bands, oh0 = (blockIdx.x % bands) * kTH;

  // ---- stage the halo (zero outside the image) and the weights: 16-byte chunks, plain loads + LDS stores
  for (int i = tid; i < halo_px * 8; i += 256) {
    const int hp = i >> 3, ch = i & 7;
    const int hr = hp / HW2, hc = hp - hr * HW2;
    const int ih = oh0 - 1 + hr, iw = hc - 1;
    u32x4v v = {0u, 0u, 0u, 0u};
    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
      v = *reinterpret_cast<const u32x4v*>(x + (((long long)n * H + ih) * W + iw) * kC + ch * 8);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(halo + swz_off(hp, ch)) = v;
  }
  if constexpr (!WGLB) {
    for (int i = tid; i < 9 * 64 * 8; i += 256) {  // w [k][r][s][c] -> wt[t = r*3 + s][k][c]
      const int ch = i & 7, k = (i >> 3) & 63, t = i >> 9;
      const u32x4v v = *reinterpret_cast<const u32x4v*>(w + ((long long)k * 9 + t) * kC + ch * 8);
      *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(wt + t * 64 * 128 + swz_off(k, ch)) = v;
    }
  }
  __syncthreads();

  // ---- wave `wave` owns output pixels [64 wave, 64 wave + 64) of the band (the band has kTH * W <= 240)
  const int npx = kTH * W;
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int hbase[4];  // halo pixel of this lane's output pixel in each 16-row fragment, tap (0, 0)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int p = wave * 64 + i * 16 + (lane & 15);
    p = p < npx ? p : npx - 1;  // rows past the band compute a duplicate; not stored
    const int oh = p / W, ow = p - oh * W;
    hbase[i] = oh * HW2 + ow;
  }
  const int g = lane >> 4;
  if constexpr (WGLB) {
    // B fragment (output channel j*16 + lane%16, channels ks*32 + 8g..) of tap t: w[(n*9 + t)*64 + ...]
    auto ldb = [&](int t, v8bf (&b)[2][4]) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          b[ks][j] = *reinterpret_cast<const v8bf*>(w + ((long long)(j * 16 + (lane & 15)) * 9 + t) * kC + ks * 32 + 8 * g);
    };
    v8bf bc[2][4], bn[2][4];
    ldb(0, bc);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) ldb(t + 1, bn);
      const int dr = t / 3, ds = t - dr * 3, dpx = dr * HW2 + ds;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        v8bf a[4];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          a[i] = *reinterpret_cast<const lds_v8bf*>(halo + swz_off(hbase[i] + dpx, ks * 4 + g));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bc[ks][j], acc[i][j], 0, 0, 0);
      }
      if (t + 1 < 9) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < 4; ++j) bc[ks][j] = bn[ks][j];
      }
    }
  } else {
#pragma unroll 1
  for (int t = 0; t < 9; ++t) {
    const int dr = t / 3, ds = t - dr * 3, dpx = dr * HW2 + ds;
    const lds_char* wtt = wt + t * 64 * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8bf a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = *reinterpret_cast<const lds_v8bf*>(halo + swz_off(hbase[i] + dpx, ks * 4 + g));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *reinterpret_cast<const lds_v8bf*>(wtt + swz_off(j * 16 + (lane & 15), ks * 4 + g));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  }
  __syncthreads();  // halo / weights no longer read: reuse the LDS for the output staging

  // ---- epilogue: each wave stages its 64 x 64 tile as bf16 [pixel][64] (128-B rows) and stores 16-B chunks
  lds_char* st = smem + wave * 64 * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = i * 16 + g * 4 + r, col = j * 16 + (lane & 15);
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(st + pr * 128 + col * 2) = f2bf(acc[i][j][r]);
      }
  __syncthreads();
  const long long out0 = ((long long)n * H + oh0) * W;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int idx = k * 64 + lane, pr = idx >> 3, ch = idx & 7;
    const int p = wave * 64 + pr;
    if (p < npx) {
      const u32x4v v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4v*>(st + pr * 128 + ch * 16);
      *reinterpret_cast<u32x4v*>(y + (out0 + p) * kC + ch * 8) = v;
    }
  }
}


// Persistent, software-pipelined form: one workgroup per CU keeps all 9 weight taps resident in LDS (72 KB) and
// walks a contiguous run of bands with the halo double-buffered (2 x 44.5 KB at W = 56): the next band's halo
// is loaded into registers (11 x 16 B per thread) while the MFMAs run on the current one, then written to the
// other LDS buffer after the epilogue, so the global-load latency hides behind compute.  Every workgroup exits
// after its run of bands (uniform loop bound).
constexpr int kPF = 11;  // 16-byte halo chunks per thread: (kTH + 2) * (W + 2) * 8 <= 256 * kPF

// part != nullptr: BatchNorm forward statistics of the stored (bf16) output, sum and sum of squares per
// channel, kept in registers across the workgroup's bands and added once into part[blockIdx % kBnStatSlots]
// (the conv_fwd_bn contract, kernels.h: BnEpi mode 1)
template <bool STATS>
__global__ void __launch_bounds__(256) conv3x3_halo_pp_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                             bf16_t* __restrict__ y, int N, int H, int W,
                                                             float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int HW2 = W + 2, halo_px = (kTH + 2) * HW2, hbytes = halo_px * 128;
  lds_char* wt = smem;  // [9][64 k][64 c]
  lds_char* hbuf[2] = {smem + 9 * 64 * 128, smem + 9 * 64 * 128 + hbytes};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bands = H / kTH, total = N * bands;
  const int b0 = (int)((long long)blockIdx.x * total / gridDim.x);
  const int b1 = (int)((long long)(blockIdx.x + 1) * total / gridDim.x);

  for (int i = tid; i < 9 * 64 * 8; i += 256) {  // w [k][r][s][c] -> wt[t = r*3 + s][k][c]
    const int ch = i & 7, k = (i >> 3) & 63, t = i >> 9;
    const u32x4v v = *reinterpret_cast<const u32x4v*>(w + ((long long)k * 9 + t) * kC + ch * 8);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(wt + t * 64 * 128 + swz_off(k, ch)) = v;
  }
  u32x4v pf[kPF];
  auto gload = [&](int band) {
    const int n = band / bands, oh0 = (band - n * bands) * kTH;
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int i = tid + k * 256, hp = i >> 3, ch = i & 7;
      const int hr = hp / HW2, hc = hp - hr * HW2, ih = oh0 - 1 + hr, iw = hc - 1;
      u32x4v v = {0u, 0u, 0u, 0u};
      if (i < halo_px * 8 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
        v = *reinterpret_cast<const u32x4v*>(x + (((long long)n * H + ih) * W + iw) * kC + ch * 8);
      pf[k] = v;
    }
  };
  auto lstore = [&](lds_char* hb) {
#pragma unroll
    for (int k = 0; k < kPF; ++k) {
      const int i = tid + k * 256;
      if (i < halo_px * 8)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(hb + swz_off(i >> 3, i & 7)) = pf[k];
    }
  };
  if (b0 < b1) {
    gload(b0);
    lstore(hbuf[0]);
  }
  __syncthreads();

  const int npx = kTH * W;
  int hbase[4];  // halo pixel of this lane's output pixel in each 16-row fragment, tap (0, 0)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int p = wave * 64 + i * 16 + (lane & 15);
    p = p < npx ? p : npx - 1;
    const int oh = p / W, ow = p - oh * W;
    hbase[i] = oh * HW2 + ow;
  }
  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};  // channel j*16 + lane%16
  int cur = 0;
  for (int band = b0; band < b1; ++band) {
    if (band + 1 < b1) gload(band + 1);
    const lds_char* halo = hbuf[cur];
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 18 (tap, k-half) steps, fully unrolled, fragments for step s + 1 read from LDS while step s's MFMAs run
    v8bf a[2][4], b[2][4];
    auto ldf = [&](int s, v8bf (&af)[4], v8bf (&bf)[4]) {
      const int t = s >> 1, ks = s & 1, dr = t / 3, dpx = dr * HW2 + (t - dr * 3);
      const lds_char* wtt = wt + t * 64 * 128;
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = *reinterpret_cast<const lds_v8bf*>(halo + swz_off(hbase[i] + dpx, ks * 4 + g));
#pragma unroll
      for (int j = 0; j < 4; ++j) bf[j] = *reinterpret_cast<const lds_v8bf*>(wtt + swz_off(j * 16 + (lane & 15), ks * 4 + g));
    };
    ldf(0, a[0], b[0]);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      if (s + 1 < 18) ldf(s + 1, a[(s + 1) & 1], b[(s + 1) & 1]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s & 1][i], b[s & 1][j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();  // every wave is done with hbuf[cur]: reuse it for the output staging
    lds_char* st = hbuf[cur] + wave * 64 * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int pr = i * 16 + g * 4 + r, col = j * 16 + (lane & 15);
          const bf16_t v = f2bf(acc[i][j][r]);
          *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(st + pr * 128 + col * 2) = v;
          if constexpr (STATS) {  // rows past the band (duplicates) weigh 0
            const float f = wave * 64 + pr < npx ? bf2f(v) : 0.f;
            ssum[j] += f;
            ssq[j] += f * f;
          }
        }
    __syncthreads();
    const int n = band / bands, oh0 = (band - n * bands) * kTH;
    const long long out0 = ((long long)n * H + oh0) * W;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = k * 64 + lane, pr = idx >> 3, ch = idx & 7;
      const int p = wave * 64 + pr;
      if (p < npx) {
        const u32x4v v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4v*>(st + pr * 128 + ch * 16);
        *reinterpret_cast<u32x4v*>(y + (out0 + p) * kC + ch * 8) = v;
      }
    }
    if (band + 1 < b1) lstore(hbuf[cur ^ 1]);
    __syncthreads();  // next halo visible; this band's staging reads done
    cur ^= 1;
  }
  if constexpr (STATS) {  // lanes l, l + 16, l + 32, l + 48 hold the same channels: fold, then one atomic per channel and wave
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        ssum[j] += __shfl_xor(ssum[j], o);
        ssq[j] += __shfl_xor(ssq[j], o);
      }
    }
    if (g == 0 && b0 < b1) {
      float* slot = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * kC;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        atomicAdd(slot + j * 16 + lane, ssum[j]);
        atomicAdd(slot + kC + j * 16 + lane, ssq[j]);
      }
    }
  }
}

}  // namespace

// Schedule: 0 persistent + double-buffered halo, weights resident in LDS (the only one built into the
// launcher); the per-band modes 1 (weights from global) and 2 (weights staged per band) stay compiled for
// tools/conv_halo_ab.py history but are not selectable any more (both measured slower, profiles/r03_*halo*)
static int halo_mode() { return 0; }

static size_t conv3x3_halo_lds(int W, int mode) {
  const size_t halo = (size_t)(kTH + 2) * (W + 2) * 128, wts = 9 * 64 * 128, stage = 4 * 64 * 128;
  if (mode == 0) return wts + 2 * (halo > stage ? halo : stage);
  const size_t a = halo + (mode == 2 ? wts : 0);
  return a > stage ? a : stage;
}

int conv3x3_halo_supported(int C, int K, int H, int W, int stats) {
  const int mode = stats ? 0 : halo_mode();
  if (mode == 0 && (kTH + 2) * (W + 2) * 8 > 256 * kPF) return 0;
  return C == kC && K == kC && H % kTH == 0 && W >= 1 && kTH * W <= 256 && conv3x3_halo_lds(W, mode) <= 160 * 1024;
}

void conv3x3_halo_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, hipStream_t st, float* part) {
  static int n_cu = 0;
  if (!n_cu) {
    for (const void* f : {(const void*)conv3x3_halo_kernel<false>, (const void*)conv3x3_halo_kernel<true>,
                          (const void*)conv3x3_halo_pp_kernel<false>,
                          (const void*)conv3x3_halo_pp_kernel<true>})
      DTG_HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    int dev = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int mode = part ? 0 : halo_mode(), total = N * (H / kTH);
  const size_t lds = conv3x3_halo_lds(W, mode);
  const dim3 grid(total < n_cu ? total : n_cu);
  if (part)
    hipLaunchKernelGGL(conv3x3_halo_pp_kernel<true>, grid, dim3(256), lds, st, x, w, y, N, H, W, part);
  else if (mode == 0)
    hipLaunchKernelGGL(conv3x3_halo_pp_kernel<false>, grid, dim3(256), lds, st, x, w, y, N, H, W, part);
  else if (mode == 1)
    hipLaunchKernelGGL(conv3x3_halo_kernel<true>, dim3(total), dim3(256), lds, st, x, w, y, N, H, W);
  else
    hipLaunchKernelGGL(conv3x3_halo_kernel<false>, dim3(total), dim3(256), lds, st, x, w, y, N, H, W);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
