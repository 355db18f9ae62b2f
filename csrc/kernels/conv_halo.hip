// Direct 3x3 / stride 1 / pad 1 convolution for 64 input and 64 output channels (ResNet-50's stage-1 conv2, NHWC bf16)
// with the BN forward statistics, from an LDS halo tile.  The implicit GEMM (conv.hip) gathers every input pixel
// once per filter tap, 9x through L2, with the L2 channels busy ~94 % of every cycle (profiles/r03_conv_l2); here
// one band of kTH = 4 output rows of an image stages its input rows with their 1-pixel halo ONCE into LDS (zeros
// outside the image) and every tap's A fragments are read from the halo at the shifted pixel, so each input byte
// crosses L2 about (kTH + 2) / kTH times.  LDS images [pixel or output channel][64 channels], 16-byte chunks
// XOR-swizzled by (row & 7) as frag_kc reads them; output through an LDS staging pass as 16-byte stores.
// Built in round 3 as a lab experiment (neutral within the spread then); in the round-5 step it measured +0.25 %
// in three interleaved rounds (profiles/r05_halo), so the statistics form is the production path for that layer.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"

namespace dtg {
using namespace gemm;

namespace {

constexpr int kTH = 4, kC = 64;

__device__ __forceinline__ int swz_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

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

static size_t halo_bn_lds(int W) {
  const size_t halo = (size_t)(kTH + 2) * (W + 2) * 128, wts = 9 * 64 * 128, stage = 4 * 64 * 128;
  return wts + 2 * (halo > stage ? halo : stage);
}

int conv3x3_halo_bn_ok(int C, int K, int H, int W) {
  return C == kC && K == kC && H % kTH == 0 && W >= 1 && kTH * W <= 256 && (kTH + 2) * (W + 2) * 8 <= 256 * kPF &&
         halo_bn_lds(W) <= 160 * 1024;
}

void conv3x3_halo_bn_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, float* part, hipStream_t st) {
  static int n_cu = 0;
  if (!n_cu) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_pp_kernel<true>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    int dev = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int total = N * (H / kTH);
  const dim3 grid(total < n_cu ? total : n_cu);
  hipLaunchKernelGGL(conv3x3_halo_pp_kernel<true>, grid, dim3(256), halo_bn_lds(W), st, x, w, y, N, H, W, part);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
