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
// LDS row of output channel k in the weight image: column n of n-tile j computes channel 4n + j, so a lane's four
// accumulators of one pixel (j = 0..3) are 4 adjacent channels -- one 8-byte staging store instead of four 2-byte
// ones -- while the B-fragment reads keep rows j*16 + n (conflict-free)
__device__ __forceinline__ int wrow(int k) { return (k & 3) * 16 + (k >> 2); }

// Persistent, software-pipelined form: one workgroup per CU keeps all 9 weight taps resident in LDS (72 KB) and
// walks a contiguous run of bands with the halo double-buffered (2 x 44.5 KB at W = 56): the next band's halo
// is loaded into registers (11 x 16 B per thread) while the MFMAs run on the current one, then written to the
// other LDS buffer after the epilogue, so the global-load latency hides behind compute.  Every workgroup exits
// after its run of bands (uniform loop bound).
constexpr int kPF = 11;  // 16-byte halo chunks per thread: (kTH + 2) * (W + 2) * 8 <= 256 * kPF

// EPI 0 (forward): BatchNorm forward statistics of the stored (bf16) output, sum and sum of squares per channel,
// kept in registers across the workgroup's bands and added once into part[blockIdx % kBnStatSlots] (the
// conv_fwd_bn contract, kernels.h: BnEpi mode 1).
// EPI 1 (data gradient of the same conv, BN-backward mode 3 epilogue): x is dy, the weights are staged flipped and
// transposed (tap t of the dgrad correlation is w[k][8 - t][c], reduced over k), and each output element becomes
// dp = relu-mask bit ? dx : 0 with the partials sum(dp), sum(dp * xhat) of the BN whose input is bn.x (the
// conv_dgrad_bn contract: BnEpi mode 3 with packed mask bits, beta 0).
struct HaloBwd {
  const bf16_t* x;          // the BN input [M, 64] (xhat = (x - mean) * invstd)
  const uint8_t* bits;      // relu mask [M, 8]
  const float* mean;
  const float* invstd;
};

template <int EPI>
__global__ void __launch_bounds__(256) conv3x3_halo_pp_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                             bf16_t* __restrict__ y, int N, int H, int W,
                                                             float* __restrict__ part, HaloBwd hb) {
  constexpr bool STATS = EPI == 0;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int HW2 = W + 2, halo_px = (kTH + 2) * HW2, hbytes = halo_px * 128;
  lds_char* wt = smem;  // [9][64 k][64 c]
  lds_char* hbuf[2] = {smem + 9 * 64 * 128, smem + 9 * 64 * 128 + hbytes};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4;
  const int bands = H / kTH, total = N * bands;
  const int b0 = (int)((long long)blockIdx.x * total / gridDim.x);
  const int b1 = (int)((long long)(blockIdx.x + 1) * total / gridDim.x);

  if constexpr (EPI == 0) {
    for (int i = tid; i < 9 * 64 * 8; i += 256) {  // w [k][r][s][c] -> wt[t = r*3 + s][k][c]
      const int ch = i & 7, k = (i >> 3) & 63, t = i >> 9;
      const u32x4v v = *reinterpret_cast<const u32x4v*>(w + ((long long)k * 9 + t) * kC + ch * 8);
      *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(wt + t * 64 * 128 + swz_off(wrow(k), ch)) = v;
    }
  } else {
    for (int i = tid; i < 9 * 64 * 8; i += 256) {  // w [k][r][s][c] -> wt[t][c][k] = w[k][8 - t][c]: 8 c per load
      const int cc = i & 7, k = (i >> 3) & 63, t = i >> 9;
      const u32x4v v = *reinterpret_cast<const u32x4v*>(w + ((long long)k * 9 + (8 - t)) * kC + cc * 8);
      const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cc * 8 + e;
        const uint16_t h16 = (uint16_t)(e & 1 ? wd[e >> 1] >> 16 : wd[e >> 1] & 0xffffu);
        *reinterpret_cast<__attribute__((address_space(3))) uint16_t*>(wt + t * 64 * 128 + swz_off(wrow(c), k >> 3) +
                                                                       (k & 7) * 2) = h16;
      }
    }
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
  float ssum[4] = {0.f, 0.f, 0.f, 0.f}, ssq[4] = {0.f, 0.f, 0.f, 0.f};  // channel 4 (lane % 16) + j
  // EPI 1: sum(dp), sum(dp * xhat) of channels 8 (lane & 7) + e over this lane's pixels; xhat is formed per element
  // (x * invstd - mean * invstd) from the lane's 8 fixed channels, like the implicit-GEMM epilogue -- a raw-moment
  // form, invstd * (sum(dp * x) - mean * sum(dp)), cancels when |mean| >> std
  float bs[8], bq[8], xs[8], xo[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bs[e] = bq[e] = 0.f;
    xs[e] = xo[e] = 0.f;
    if constexpr (EPI == 1) {
      const int c = (lane & 7) * 8 + e;
      xs[e] = hb.invstd[c];
      xo[e] = -hb.mean[c] * xs[e];
    }
  }
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
    const int n_ = band / bands, oh0_ = (band - n_ * bands) * kTH;
    const long long px0 = ((long long)n_ * H + oh0_) * W;
    u32x4v xv[8];
    uint32_t mb[8];
    if constexpr (EPI == 1) {  // the epilogue's BN input and mask bits, in flight under the staging below
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int idx = k * 64 + lane, pr = idx >> 3, ch = idx & 7, p = wave * 64 + pr;
        const long long o = px0 + (p < npx ? p : npx - 1);
        xv[k] = *reinterpret_cast<const u32x4v*>(hb.x + o * kC + ch * 8);
        mb[k] = hb.bits[o * (kC / 8) + ch];
      }
    }
    __syncthreads();  // every wave is done with hbuf[cur]: reuse it for the output staging
    lds_char* st = hbuf[cur] + wave * 64 * 128;
    typedef unsigned int u32x2v __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = i * 16 + g * 4 + r;
        uint32_t hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // channel 4 (lane & 15) + j
          const bf16_t v = f2bf(acc[i][j][r]);
          hv[j] = (uint32_t)v;
          if constexpr (STATS) {  // rows past the band (duplicates) weigh 0
            const float f = wave * 64 + pr < npx ? bf2f(v) : 0.f;
            ssum[j] += f;
            ssq[j] += f * f;
          }
        }
        *reinterpret_cast<__attribute__((address_space(3))) u32x2v*>(st + pr * 128 + (lane & 15) * 8) =
            u32x2v{hv[0] | (hv[1] << 16), hv[2] | (hv[3] << 16)};
      }
    __syncthreads();
    const long long out0 = px0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = k * 64 + lane, pr = idx >> 3, ch = idx & 7;
      const int p = wave * 64 + pr;
      if (p < npx) {
        u32x4v v = *reinterpret_cast<const __attribute__((address_space(3))) u32x4v*>(st + pr * 128 + ch * 16);
        if constexpr (EPI == 1) {  // dp = mask ? dx : 0 and the BN-backward partials (raw moment of x)
          const uint32_t vd[4] = {v.x, v.y, v.z, v.w}, xd[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w};
          uint32_t od[4];
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const uint32_t lo_m = (mb[k] >> (2 * e2)) & 1u, hi_m = (mb[k] >> (2 * e2 + 1)) & 1u;
            const uint32_t lo = lo_m ? (vd[e2] & 0xffffu) : 0u, hi = hi_m ? (vd[e2] & 0xffff0000u) : 0u;
            od[e2] = lo | hi;
            const float dl = __uint_as_float(lo << 16), dh = __uint_as_float(hi);
            bs[2 * e2] += dl;
            bs[2 * e2 + 1] += dh;
            const float xl = fmaf(__uint_as_float(xd[e2] << 16), xs[2 * e2], xo[2 * e2]);
            const float xh = fmaf(__uint_as_float(xd[e2] & 0xffff0000u), xs[2 * e2 + 1], xo[2 * e2 + 1]);
            bq[2 * e2] = fmaf(dl, xl, bq[2 * e2]);
            bq[2 * e2 + 1] = fmaf(dh, xh, bq[2 * e2 + 1]);
          }
          v.x = od[0]; v.y = od[1]; v.z = od[2]; v.w = od[3];
        }
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
        atomicAdd(slot + 4 * lane + j, ssum[j]);
        atomicAdd(slot + kC + 4 * lane + j, ssq[j]);
      }
    }
  }
  if constexpr (EPI == 1) {  // lanes sharing lane & 7 hold the same channels: fold, convert, one atomic each
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 8; o < 64; o <<= 1) {
        bs[e] += __shfl_xor(bs[e], o);
        bq[e] += __shfl_xor(bq[e], o);
      }
    if (lane < 8 && b0 < b1) {
      float* slot = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * kC;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = lane * 8 + e;
        atomicAdd(slot + c, bs[e]);
        atomicAdd(slot + kC + c, bq[e]);  // sum(dp * xhat)
      }
    }
  }
}


// Weight gradient of the same conv, dW[k][r][s][c] = sum over pixels p of dy[p][k] * x[p + (r - 1, s - 1)][c]: a GEMM
// 64 (k) x 576 (tap, c) reduced over pixels, so both operands are needed pixel-major -- exactly how NHWC stores them.
// Each band stages its dy rows ([px][64 k]) and its x rows with the 1-pixel halo ONCE into LDS and every operand
// fragment is a transposed read (ds_read_b64_tr_b16: 4 pixel rows x 16 channels per 16-lane group); a tap's B
// fragment reads the halo rows of the shifted pixels, so x crosses L2 (kTH + 2) / kTH times instead of 9 times
// through an im2col gather (conv.hip's implicit wgrad).  Persistent: one workgroup per CU walks a contiguous run of
// bands, accumulating its 64 x 576 fp32 partial in registers (wave w: the column tiles 9w .. 9w + 8); the next
// band's dy + halo are loaded into registers a few chunks per 32-pixel step and written to the other LDS buffer two
// steps later, under this band's MFMAs.  One fp32 slab per workgroup, summed by the split-K reduce.
// LDS images: 128-B rows, 16-B chunks XOR-swizzled by (row & 7) ^ 4 * ((row >> 3) & 1) (the two 4-row blocks a
// 32-lane half reads, 8 rows apart, land in different banks).  The halo rows are 64 pixels apart (W + 2 <= 64), so
// a fragment row's swizzle is a per-lane constant (A) or a per-lane table entry XOR one per-step bit (B), and every
// read address is one VALU op (or none) instead of a swizzle evaluation: the first version spent ~2000 VALU
// instructions per band on read addresses and ran the MFMA pipe at 24 %.
__device__ __forceinline__ int wswz(int row, int chunk) {
  return row * 128 + ((chunk ^ (row & 7) ^ ((row >> 1) & 4)) << 4);
}

template <int W, int kDist>  // kDist: steps between a staging chunk's global load and its LDS write
__global__ void __launch_bounds__(256) conv3x3_halo_wgrad_kernel(const bf16_t* __restrict__ x,
                                                                const bf16_t* __restrict__ dy,
                                                                float* __restrict__ ws, int N, int H) {
  static_assert(W % 8 == 0 && W + 2 <= 64, "8-pixel fragment groups inside an image row; 64-pixel halo pitch");
  constexpr int HP = 64, hrows = kTH + 2, hbytes = hrows * HP * 128;
  constexpr int npx = kTH * W, nst = npx / 32, dyrows = npx;
  static_assert(npx % 32 == 0, "whole 32-pixel reduction steps");
  constexpr int bufb = hbytes + dyrows * 128;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, q = (lane & 15) >> 2, pl = lane & 3;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bands = H / kTH, total = N * bands;
  const int b0 = (int)((long long)blockIdx.x * total / gridDim.x);
  const int b1 = (int)((long long)(blockIdx.x + 1) * total / gridDim.x);

  // a band's halo (hrows x 64 pixels, columns past W + 1 unused) and dy rows as 16-byte chunks, kXP + kDP per
  // thread (global, not flat, loads: address_space(1)); halo pixels outside the image read the zero page, so no
  // chunk needs a select after its load (the
  // compiler hoists such selects right behind the loads and waits for them there).  Branch-free: a load under a
  // lane condition splits the code into blocks, and the compiler then drains every outstanding load at the join.
  // LDS-DMA is not used: the compiler drains in-flight DMA before the first LDS read of each step, which
  // serialised the next band's loads with this band's MFMAs.
  constexpr int kXP = hrows * HP * 8 / 256, kDP = (dyrows * 8 + 255) / 256, kCH = kXP + kDP;
  auto cload = [&](int band, int ci) {
    const int n = band / bands, oh0 = (band - n * bands) * kTH;
    if (ci < kXP) {
      const int i = tid + ci * 256, r = i >> 3, ch = i & 7;
      const int ih = oh0 - 1 + (r >> 6), iw = (r & 63) - 1;
      const bool ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      const long long off = (((long long)n * H + (ok ? ih : oh0)) * W + (ok ? iw : 0)) * kC + ch * 8;
      return *reinterpret_cast<const __attribute__((address_space(1))) u32x4v*>((uintptr_t)sel(ok, x + off));
    }
    const int i = tid + (ci - kXP) * 256, r = i >> 3;
    const bool ok = r < npx;
    const long long off = (((long long)n * H + oh0) * W + (ok ? r : 0)) * kC + (i & 7) * 8;
    return *reinterpret_cast<const __attribute__((address_space(1))) u32x4v*>((uintptr_t)sel(ok, dy + off));
  };
  auto cstore = [&](lds_char* b, int ci, const u32x4v& w) {
    if (ci < kXP) {
      const int i = tid + ci * 256;
      *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(b + wswz(i >> 3, i & 7)) = w;
    } else {
      const int i = tid + (ci - kXP) * 256;
      // (unconditional when the chunks tile exactly: a conditional store makes the compiler sink its load into the
      // branch, right before the store, where nothing hides its latency)
      if (dyrows * 8 % 256 == 0 || i < dyrows * 8)
        *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(b + hbytes + wswz(i >> 3, i & 7)) = w;
    }
  };

  // read-address tables.  A (dy image, rows 32 st + 8 g + q + 4 h): the swizzle of such a row is
  // (q + 4h) ^ 4 (g & 1) for every step, so offA[h][i] + st * 4096 is the address.  B (halo, rows
  // (32 st + 8 g) / W * 64 + (32 st + 8 g) % W + 4h + q + dr * 64 + ds): with w0 = (32 st + 8 g) % W a multiple of 8,
  // the swizzle is sw(4h + q + ds) ^ 4 ((w0 >> 3) & 1), so the address is (offB[h][j] ^ (flip << 6)) + rowbase.
  auto sw16 = [](int v) { return (v & 7) ^ ((v >> 1) & 4); };
  int offA[2][4], offB[2][9];
  const int sub = (pl & 1) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 8 * g + 4 * h + q, ch = (i * 16 + 4 * pl) >> 3;
      offA[h][i] = hbytes + r * 128 + ((ch ^ sw16(r)) << 4) + sub;
    }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int jj = 9 * wave + j, t = jj >> 2, dr = t / 3, ds = t - dr * 3, ch = ((jj & 3) * 16 + 4 * pl) >> 3;
      const int v = 4 * h + q + ds;
      offB[h][j] = (dr * HP + v) * 128 + ((ch ^ sw16(v)) << 4) + sub;
    }
  }
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (b0 < b1) {
#pragma unroll
    for (int ci = 0; ci < kCH; ++ci) cstore(smem, ci, cload(b0, ci));
  }
  __syncthreads();
  // next band's chunks: kPS per step, loaded at step st and written to the other buffer kDist steps later (the
  // last sets after the band's last step)
  constexpr int kPS = (kCH + nst - 2) / (nst - 1), kSets = (kCH + kPS - 1) / kPS;
  static_assert(kSets <= nst, "every chunk set is loaded within the band's steps");
  u32x4v stg[kSets][kPS];
  int cur = 0;
  for (int band = b0; band < b1; ++band) {
    const int nb = band + 1 < b1 ? band + 1 : band;  // the last band reloads itself into the unused buffer (no branch)
    lds_char* other = smem + (cur ^ 1) * bufb;  // its last readers passed the previous barrier
    const uint32_t buf = (uint32_t)(uintptr_t)(smem + cur * bufb);
    // fragments double-buffered: step st + 1's 26 reads are issued before step st's 36 MFMAs
    v8bf a[2][4], b[2][9];
    auto ldf = [&](int st, v8bf (&af)[4], v8bf (&bf)[9]) {
      const int pix = 32 * st + 8 * g, orow = pix / W, w0 = pix - orow * W;
      uint32_t rb = buf + (uint32_t)(orow * HP + w0) * 128u, fl = (uint32_t)((w0 >> 3) & 1) << 6;
      asm volatile("" : "+v"(rb), "+v"(fl));  // this step's addresses are computed in this step (not hoisted)
      const uint32_t ab = buf + st * 4096;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)(ab + offA[0][i]));
        const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)(ab + offA[1][i]));
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)((offB[0][j] ^ fl) + rb));
        const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)((offB[1][j] ^ fl) + rb));
        bf[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    };
    ldf(0, a[0], b[0]);
#pragma unroll
    for (int st = 0; st < nst; ++st) {
      if (st < kSets) {
#pragma unroll
        for (int k = 0; k < kPS; ++k)
          if (st * kPS + k < kCH) stg[st][k] = cload(nb, st * kPS + k);
      }
      if (st + 1 < nst) ldf(st + 1, a[(st + 1) & 1], b[(st + 1) & 1]);
#pragma unroll
      for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st & 1][i], b[st & 1][j], acc[i][j], 0, 0, 0);
      if (st >= kDist && st - kDist < kSets) {
#pragma unroll
        for (int k = 0; k < kPS; ++k)
          if ((st - kDist) * kPS + k < kCH)
            cstore(other, (st - kDist) * kPS + k, stg[st - kDist][k]);
      }
    }
#pragma unroll
    for (int s2 = nst - kDist; s2 < kSets; ++s2)
#pragma unroll
      for (int k = 0; k < kPS; ++k)
        if (s2 * kPS + k < kCH) cstore(other, s2 * kPS + k, stg[s2][k]);
    __syncthreads();  // next band visible; every wave is done reading this one before it is overwritten
    cur ^= 1;
  }
  float* slab = ws + (long long)blockIdx.x * (kC * 9 * kC);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[(i * 16 + g * 4 + r) * (9 * kC) + (9 * wave + j) * 16 + (lane & 15)] = acc[i][j][r];
}

// Linear-halo weight gradient for any 3x3 / s1 / p1 layer with C, K multiples of 64 (ResNet-50 stages 2-4: 28x28 x 128,
// 14x14 x 256, 7x7 x 512).  The whole batch is laid out as one tall virtual image: each image row padded with zero
// columns to a pitch HP (a multiple of 8 >= W + 1) and each image followed by one zero row (VR = H + 1 rows per
// image); the pad column / row doubles as the next row's left halo / the next image's top halo.  Output position
// p = (img * VR + oh) * HP + ow (dy = 0 on the pad) then reads tap (dr, ds) of x at the SAME linear index plus
// dr * HP + ds, so a band of BP = 256 consecutive positions needs the x rows [p0, p0 + BP + 2 HP + 2): the halo
// costs 2 HP + 2 rows per band (1.14-1.38x x reads; stage 1's kernel re-reads 2 of every 4 image rows) and no read
// address needs a division.  Every fragment row is 32 st + (a per-lane constant), so each transposed read is buffer
// base + st * 4096 + a per-lane table entry (the swizzle of a row depends on row & 15 only): no address VALU in
// the MFMA loop.
// Staging: a wave's 64 lanes move 8 consecutive positions x 8 16-byte chunks, and with HP a multiple of 8 those 8
// positions never straddle a virtual row -- so the row, image and their validity are wave-uniform (SALU), and a
// chunk costs ~4 VALU (the column check and a buffer offset; out-of-range offsets read 0 through the buffer
// descriptor's range check).  The first version decomposed every position per lane (~800 VALU per band, 36 % of the
// wave cycles, profiles/r06_lin_wgrad).  The next band's chunks are loaded in the band's first 3 steps and written
// to the other buffer in its last 3 (5 steps of MFMAs hide the load latency).
// Work split: a workgroup owns one 64 (k) x 576 (tap, c) block of dW -- channel blocks (kb, cb), the stage-1
// accumulator layout -- over a contiguous run of bands; the (kb, cb) pairs of one band range sit on the same XCD
// (they read the same dy / x rows through its L2).  One fp32 slab per band range, summed by the split-K reduce.
// Pad positions: 1 - HW / (VR HP) = 16 % (28x28), 18 % (14x14), 23 % (7x7) of the MFMAs.
template <int W, int H>
struct LinGeom {
  static constexpr int HP = (W + 1 + 7) / 8 * 8, VR = H + 1, NST = 8, BP = NST * 32;
  static constexpr int XW = (BP + 2 * HP + 2 + 31) / 32 * 32;  // staged x rows (whole 32-row chunk groups)
  static constexpr int xbytes = XW * 128, bufb = xbytes + BP * 128;
  static constexpr int kXP = XW / 32, kDP = BP / 32, kCH = kXP + kDP;
  static constexpr int kLS = 3, kPS = (kCH + kLS - 1) / kLS;  // chunks loaded per step in steps 0 .. kLS - 1
  static constexpr int kDist = NST - 1 - kLS;                 // set s stored at step s + kDist (<= NST - 2)
  static constexpr size_t lds = 2 * (size_t)bufb;
};

template <int W, int H>
__global__ void __launch_bounds__(256) conv3x3_lin_wgrad_kernel(const bf16_t* __restrict__ x,
                                                               const bf16_t* __restrict__ dy,
                                                               float* __restrict__ ws, int N, int C, int K, int G) {
  using LG = LinGeom<W, H>;
  constexpr int HP = LG::HP, VR = LG::VR, NST = LG::NST, BP = LG::BP, xbytes = LG::xbytes, bufb = LG::bufb;
  constexpr int kXP = LG::kXP, kCH = LG::kCH, kPS = LG::kPS, kLS = LG::kLS, kDist = LG::kDist;
  static_assert(HP % 8 == 0 && kLS + kDist == NST - 1 && kLS * kPS >= kCH, "staging schedule");
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4, q = (lane & 15) >> 2, pl = lane & 3;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // (band range, channel-block pair) of this workgroup: grid = G * P (a power of 2 >= 8), XCD = blockIdx % 8, so
  // an XCD holds gridDim / 8 slots; the pairs of one band range fill an XCD's slots (or span P / slots XCDs)
  const int P = (K >> 6) * (C >> 6), bid = blockIdx.x, xcd = bid & 7, slot = bid >> 3, slots = gridDim.x >> 3;
  int rg, pair;
  if (P <= slots) {
    rg = xcd * (slots / P) + slot / P;
    pair = slot % P;
  } else {
    const int xr = P / slots;
    rg = xcd / xr;
    pair = (xcd % xr) * slots + slot;
  }
  const int cbn = C >> 6, kb = pair / cbn, cb = pair - kb * cbn;
  const int T = N * VR * HP, NB = (T + BP - 1) / BP;
  const int b0 = (int)((long long)NB * rg / G), b1 = (int)((long long)NB * (rg + 1) / G);
  // buffer descriptors over the whole tensors: an offset past the end reads 0 (the pad and out-of-batch chunks)
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, (int)((long long)N * H * W * C * 2),
                                                                       0x00020000);
  const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dy, 0, (int)((long long)N * H * W * K * 2),
                                                                       0x00020000);
  const int j = lane >> 3, ch = lane & 7;
  const int xlane = (j * C + cb * 64 + ch * 8) * 2, dlane = (j * K + kb * 64 + ch * 8) * 2;  // bytes
  constexpr int kBad = 0x7ffffff0;

  // chunk ci of a band: rows 8 wave + j + 32 ci (x window for ci < kXP, else the band's dy rows); the 8 positions of
  // a wave's chunk share one virtual row (HP % 8 == 0), so everything but the column is wave-uniform
  auto cload = [&](int band, int ci) {
    const bool isx = ci < kXP;
    const int pos = band * BP + 8 * wave + 32 * (isx ? ci : ci - kXP);  // uniform
    const int R = pos / HP, cu = pos - R * HP, img = R / VR, rr = R - img * VR;
    int voff;
    if (isx) {  // x(img, rr - 1, cu + j - 1)
      const int lim = (rr >= 1 && img < N) ? W : 0;
      const int ubase = ((img * H + rr - 1) * W + cu - 1) * C * 2;
      voff = (unsigned)(cu + j - 1) < (unsigned)lim ? ubase + xlane : kBad;
    } else {    // dy(img, rr, cu + j)
      const int lim = (rr < H && img < N) ? W : 0;
      const int ubase = ((img * H + rr) * W + cu) * K * 2;
      voff = (unsigned)(cu + j) < (unsigned)lim ? ubase + dlane : kBad;
    }
    return __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(isx ? rx : rd, voff, 0, 0));
  };
  auto cstore = [&](lds_char* b, int ci, const u32x4v& v) {
    const int row = 8 * wave + j + 32 * (ci < kXP ? ci : ci - kXP);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(b + (ci < kXP ? 0 : xbytes) + wswz(row, ch)) = v;
  };

  // read-address tables (see above): A = dy rows 32 st + 8 g + 4 h + q; B = x rows of the same positions + tap offset
  auto sw16 = [](int v) { return (v & 7) ^ ((v >> 1) & 4); };
  // (absolute LDS byte addresses in buffer 0; buffer 1 is bufb higher -- toggled once per band, so every read in
  // the unrolled steps is table entry + st * 4096, an immediate offset of the ds_read)
  uint32_t offA[2][4], offB[2][9];
  const uint32_t base0 = (uint32_t)(uintptr_t)smem;
  const int sub = (pl & 1) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 8 * g + 4 * h + q, c8 = (i * 16 + 4 * pl) >> 3;
      offA[h][i] = base0 + xbytes + r * 128 + ((c8 ^ sw16(r)) << 4) + sub;
    }
#pragma unroll
    for (int jx = 0; jx < 9; ++jx) {
      const int jj = 9 * wave + jx, t = jj >> 2, dr = t / 3, ds = t - dr * 3, c8 = ((jj & 3) * 16 + 4 * pl) >> 3;
      const int v = 8 * g + 4 * h + q + dr * HP + ds;
      offB[h][jx] = base0 + v * 128 + ((c8 ^ sw16(v)) << 4) + sub;
    }
  }
  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jx = 0; jx < 9; ++jx) acc[i][jx] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (b0 < b1) {
#pragma unroll
    for (int ci = 0; ci < kCH; ++ci) cstore(smem, ci, cload(b0, ci));
  }
  __syncthreads();
  u32x4v stg[kLS][kPS];
  int cur = 0;
  v8bf a[2][4], b[2][9];
  auto ldf = [&](int st, v8bf (&af)[4], v8bf (&bf)[9]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)offA[0][i] + st * 512);
      const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)offA[1][i] + st * 512);
      af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int jx = 0; jx < 9; ++jx) {
      const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)offB[0][jx] + st * 512);
      const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(uintptr_t)offB[1][jx] + st * 512);
      bf[jx] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
  };
  ldf(0, a[0], b[0]);
  for (int band = b0; band < b1; ++band) {
    const int nb = band + 1 < b1 ? band + 1 : band;  // the last band reloads itself into the unused buffer (no branch)
    lds_char* other = smem + (cur ^ 1) * bufb;
#pragma unroll
    for (int st = 0; st < NST; ++st) {
      if (st == NST - 1) {
        // the barrier ending step NST - 2 made the other buffer (stored in steps kDist .. NST - 2) visible and every
        // read of this one is done: the read tables move over, and the next band's first fragments are read under
        // this band's last MFMAs (no per-band pipeline drain)
        const uint32_t delta = cur ? (uint32_t)(-bufb) : (uint32_t)bufb;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int i = 0; i < 4; ++i) offA[h][i] += delta;
#pragma unroll
          for (int jx = 0; jx < 9; ++jx) offB[h][jx] += delta;
        }
      }
      // one scheduling region per step: the next step's 26 fragment reads interleaved one per MFMA with this step's
      // 36 MFMAs (left alone, the scheduler sinks each read next to its consumer and every 4 MFMAs wait out an LDS
      // latency; issued as one block, the 4-bit lgkm counter stalls the wave after 15 of them)
      __builtin_amdgcn_sched_barrier(0);
      if (st < kLS) {
#pragma unroll
        for (int k = 0; k < kPS; ++k)
          if (st * kPS + k < kCH) stg[st][k] = cload(nb, st * kPS + k);
      }
      ldf((st + 1) % NST, a[(st + 1) & 1], b[(st + 1) & 1]);
#pragma unroll
      for (int jx = 0; jx < 9; ++jx)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i][jx] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[st & 1][i], b[st & 1][jx], acc[i][jx], 0, 0, 0);
      if (st >= kDist && st - kDist < kLS) {
#pragma unroll
        for (int k = 0; k < kPS; ++k)
          if ((st - kDist) * kPS + k < kCH) cstore(other, (st - kDist) * kPS + k, stg[st - kDist][k]);
      }
#pragma unroll
      for (int k = 0; k < 26; ++k) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 10, 0);
      __builtin_amdgcn_sched_barrier(0);
      if (st == NST - 2) __syncthreads();  // other buffer complete; this one's last fragments (step NST - 1) read
    }
    cur ^= 1;
  }
  // this workgroup's 64 x 576 block of slab rg: rows kb * 64 + ..., columns t * C + cb * 64 + ...
  const int NC = 9 * C;
  float* slab = ws + (long long)rg * K * NC + (long long)(kb * 64) * NC + cb * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int jx = 0; jx < 9; ++jx) {
      const int jj = 9 * wave + jx, t = jj >> 2, c16 = jj & 3;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[(long long)(i * 16 + g * 4 + r) * NC + t * C + c16 * 16 + (lane & 15)] = acc[i][jx][r];
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

static int halo_cus() {
  static int n_cu = 0;
  if (!n_cu) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_pp_kernel<0>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_pp_kernel<1>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    int dev = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  return n_cu;
}

static int g_halo_fwd = 1;
void conv3x3_halo_fwd_set(int on) { g_halo_fwd = on; }  // 0 off (implicit GEMM), 1 on

bool conv3x3_halo_bn_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, float* part, hipStream_t st) {
  if (!g_halo_fwd) return false;
  const int n_cu = halo_cus(), total = N * (H / kTH);
  const dim3 grid(total < n_cu ? total : n_cu);
  hipLaunchKernelGGL(conv3x3_halo_pp_kernel<0>, grid, dim3(256), halo_bn_lds(W), st, x, w, y, N, H, W, part,
                     HaloBwd{});
  DTG_LAUNCH_CHECK();
  return true;
}

static int g_halo_dgrad = 1;
void conv3x3_halo_dgrad_set(int on) { g_halo_dgrad = on; }  // 0 off, 1 on, > 1 on with a grid of that size

bool conv3x3_halo_bn_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dp, int N, int H, int W, const BnEpi& bn,
                           hipStream_t st) {
  if (!g_halo_dgrad || bn.mode != 3 || !bn.maskbits || !bn.x || bn.x2 || bn.old_sub2 || !bn.mean || !bn.invstd)
    return false;
  // on > 1: a grid of that many workgroups (one per CU), leaving the rest of the chip to the side stream's wgrads
  const int n_cu = g_halo_dgrad > 1 ? g_halo_dgrad : halo_cus(), total = N * (H / kTH);
  halo_cus();
  const dim3 grid(total < n_cu ? total : n_cu);
  hipLaunchKernelGGL(conv3x3_halo_pp_kernel<1>, grid, dim3(256), halo_bn_lds(W), st, dy, w, dp, N, H, W, bn.part,
                     HaloBwd{bn.x, bn.maskbits, bn.mean, bn.invstd});
  DTG_LAUNCH_CHECK();
  return true;
}

// ---- weight gradient (conv_wgrad for 64 -> 64, 3x3 / s1 / p1, W = 56) ----
constexpr int kWgW = 56;
static size_t halo_wgrad_lds() {
  constexpr int halo = (kTH + 2) * 64 * 128, dyb = kTH * kWgW * 128;
  return 2 * (size_t)(halo + dyb);
}
static int g_halo_wgrad = 1;
// 0 off, 1 on (2 / 3: shorter staging distance), >= 8: on with at most that many workgroups (A/B runs: a side-stream
// grid below the CU count leaves CUs to the main stream)
void conv3x3_halo_wgrad_set(int on) { g_halo_wgrad = on; }

int conv3x3_halo_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w) {
  if (!g_halo_wgrad || C != kC || K != kC || R != 3 || S != 3 || stride != 1 || pad != 1 ||
      (stride_w != 0 && stride_w != 1) || W != kWgW || H % kTH != 0 || halo_wgrad_lds() > 160 * 1024)
    return 0;
  static int n_cu = 0;
  if (!n_cu) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_wgrad_kernel<kWgW, 2>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_wgrad_kernel<kWgW, 3>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_halo_wgrad_kernel<kWgW, 4>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    n_cu = halo_cus();
  }
  const int total = N * (H / kTH), cap = g_halo_wgrad >= 8 && g_halo_wgrad < n_cu ? g_halo_wgrad : n_cu;
  return total < cap ? total : cap;
}

// ---- linear-halo weight gradient (3x3 / s1 / p1, C and K multiples of 64, H = W in {7, 14, 28}) ----
// 0 off (implicit GEMM), 1 on (128 workgroups), a power of 2 in [64, 256]: on with that many workgroups.  The kernel
// runs on the weight-gradient side stream, one 155-KB-LDS workgroup per CU, so its grid is the number of CUs the main
// stream's kernels cannot use while it runs: 128 workgroups measured +0.5 % on the ResNet step against 256 (in 2.1x
// the kernel time) and 64 -0.3 % against 128 (profiles/r06_lin_wgrad/ab_grid*.log)
static constexpr int kLinGridDefault = 128;
static int g_lin_wgrad = 1;
static int g_lin_grid = kLinGridDefault;
void conv3x3_lin_wgrad_set(int on) {
  g_lin_wgrad = on;
  g_lin_grid = (on >= 64 && on <= 256 && (on & (on - 1)) == 0) ? on : kLinGridDefault;
}
static int lin_pairs(int C, int K) { return (C / 64) * (K / 64); }

int conv3x3_lin_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w) {
  if (!g_lin_wgrad || R != 3 || S != 3 || stride != 1 || pad != 1 || (stride_w != 0 && stride_w != 1) || H != W ||
      (W != 7 && W != 14 && W != 28) || C % 64 || K % 64)
    return 0;
  const int P = lin_pairs(C, K);
  // grid = 256 workgroups = (band ranges) x (channel-block pairs); pairs of one range on one XCD (or two)
  // P and the per-XCD slot count must divide one another, and a range may span at most the 8 XCDs
  const int slots = g_lin_grid / 8;
  if ((P & (P - 1)) != 0 || P > g_lin_grid || (P > slots && P / slots > 8)) return 0;
  // 32-bit positions and byte offsets (buffer loads)
  if ((long long)N * (H + 1) * ((W + 8) / 8 * 8) >= (1LL << 30) || 2LL * N * H * W * (C > K ? C : K) >= (1LL << 31))
    return 0;
  static bool init = false;
  if (!init) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_lin_wgrad_kernel<28, 28>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_lin_wgrad_kernel<14, 14>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_lin_wgrad_kernel<7, 7>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    init = true;
  }
  return g_lin_grid / P;  // split-K slabs = band ranges
}

void conv3x3_lin_wgrad(const bf16_t* dy, const bf16_t* x, float* ws, int split, int N, int H, int W, int C, int K,
                       hipStream_t st) {
  const int P = lin_pairs(C, K);
  const int wgs = split * P;
  if (wgs < 8 || (wgs & (wgs - 1)) != 0)
    throw std::runtime_error("conv3x3_lin_wgrad: split x channel-block pairs must be a power of 2 >= 8");
  const dim3 grid(wgs);
  const size_t lds28 = LinGeom<28, 28>::lds, lds14 = LinGeom<14, 14>::lds, lds7 = LinGeom<7, 7>::lds;
  if (W == 28)
    hipLaunchKernelGGL((conv3x3_lin_wgrad_kernel<28, 28>), grid, dim3(256), lds28, st, x, dy, ws,
                       N, C, K, split);
  else if (W == 14)
    hipLaunchKernelGGL((conv3x3_lin_wgrad_kernel<14, 14>), grid, dim3(256), lds14, st, x, dy, ws,
                       N, C, K, split);
  else if (W == 7)
    hipLaunchKernelGGL((conv3x3_lin_wgrad_kernel<7, 7>), grid, dim3(256), lds7, st, x, dy, ws,
                       N, C, K, split);
  else
    throw std::runtime_error("conv3x3_lin_wgrad: no instance for this width");
  DTG_LAUNCH_CHECK();
}

void conv3x3_halo_wgrad(const bf16_t* dy, const bf16_t* x, float* ws, int grid, int N, int H, hipStream_t st) {
  // staging distance: 4 steps (default; 2 / 3 by conv3x3_halo_wgrad_set(2 / 3) for A/B runs): 4 measured
  // 312-319 us vs 331-335 us at 2 (profiles/r05_halo/wgrad3_dist_zp.log)
  if (g_halo_wgrad == 2)
    hipLaunchKernelGGL((conv3x3_halo_wgrad_kernel<kWgW, 2>), dim3(grid), dim3(256), halo_wgrad_lds(), st, x, dy, ws, N, H);
  else if (g_halo_wgrad == 3)
    hipLaunchKernelGGL((conv3x3_halo_wgrad_kernel<kWgW, 3>), dim3(grid), dim3(256), halo_wgrad_lds(), st, x, dy, ws, N, H);
  else
    hipLaunchKernelGGL((conv3x3_halo_wgrad_kernel<kWgW, 4>), dim3(grid), dim3(256), halo_wgrad_lds(), st, x, dy, ws, N, H);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
