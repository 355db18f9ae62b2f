// Lab (round 5, negative in the ResNet-50 step): the transposed form of csrc/kernels/bn_dx_wgrad.hip -- a
// bottleneck's BN1 dx pass fused with conv1's weight gradient.  It moves the block-input read (the act operand,
// 1.64 GB per stage-1 call at batch 1024) from the side stream onto the main stream to save the re-read of dx
// (0.41 GB): 15.75k vs 15.93k img/s with all three shapes, and each shape alone loses too
// (profiles/r05_dxw1).  Kept for tools/tests only.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"
#include "lab.h"

namespace dtg {
namespace {
using namespace gemm;

constexpr int kDR = 32;  // rows per block

// ---- transposed shapes: dx of at most 128 channels, act of 256 or 512 ------------------------------------------
// A bottleneck's BN1 dx pass and conv1's weight gradient dW1 [C = width][CI = block input channels] (ResNet-50 stage
// 1: 64 x 256; stage 2: 128 x 512, and its stride-2 entry block 128 x 256).  Unfused, the side stream re-read dx
// (the BN1 pass's output) together with the block input to form dW1.  Here one workgroup computes ALL C channels
// of each 32-row dx block in registers, stores dx (the conv1 dgrad's operand) and its MN-contiguous LDS image,
// stages the 32 x CI act block by LDS-DMA, and NW = CI / 64 waves split the act columns: wave w accumulates
// dW[0..C) x [64 w, +64) over every block of the kernel (acc[C / 16][4]).  One fp32 [C][CI] partial per
// workgroup, summed into the gradient by the split-K reduction.
template <int C_, int CI>
__global__ void __launch_bounds__(CI, CI == 256 ? 2 : 1) bn_dxT_wgrad_kernel(const bf16_t* __restrict__ dp,
                                                                          const bf16_t* __restrict__ x,
                                                                          const float* __restrict__ coef,
                                                                          bf16_t* __restrict__ dx,
                                                                          const bf16_t* __restrict__ act,
                                                                          long long ldact, float* __restrict__ slabs,
                                                                          int nblk) {
  constexpr int NW = CI / 64, NTH = CI;  // one wave per 64 act columns
  constexpr int CH8 = C_ / 8;            // 8-channel chunks per dx row
  constexpr int RS = NTH / CH8;          // row slots of the elementwise part
  constexpr int U = kDR / RS;            // rows per thread per block
  static_assert(U >= 1 && RS * U == kDR, "whole dx rows per thread");
  constexpr int kDXL = kDR * C_ * 2;     // dx block, [32 m][C] MC image
  constexpr int kACTL = kDR * CI * 2;    // act block, [32 m][CI] MC image (two slots)
  constexpr int PIECES = kDR * CI * 2 / (NTH * 16);  // LDS-DMA instructions per thread per act block
  __shared__ __attribute__((aligned(16))) char smem_raw[kDXL + 2 * kACTL];
  lds_char* sdx = (lds_char*)smem_raw;
  lds_char* sact = sdx + kDXL;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x, gid = xcd_remap(blockIdx.x, G);
  const int c8 = tid % CH8, rs = tid / CH8, c0 = c8 * 8;
  float a[8], bx[8], cc[8];
  load8_f32(coef + c0, a);
  load8_f32(coef + C_ + c0, bx);
  load8_f32(coef + 2 * C_ + c0, cc);
  DenseMC<false> sa{act, ldact, CI, 0};
  f32x4 acc[C_ / 16][4];
#pragma unroll
  for (int i = 0; i < C_ / 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto unpack = [](const u32x4v& v, float (&f)[8]) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
  };
  u32x4v g[U], xv[U];
  auto issue = [&](int b, int slot) {
    const long long m0 = (long long)b * kDR;
    stage_mc<CI, DenseMC<false>, NW, kDR>(sa, sact + slot * kACTL, 0, (int)m0, wave, lane);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long off = (m0 + rs + RS * u) * C_ + c0;
      g[u] = *reinterpret_cast<const u32x4v*>(dp + off);
      xv[u] = *reinterpret_cast<const u32x4v*>(x + off);
    }
  };
  if (gid < nblk) issue(gid, 0);
  int slot = 0;
  for (int b = gid; b < nblk; b += G, slot ^= 1) {
    const long long m0 = (long long)b * kDR;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int m = rs + RS * u;
      float gf[8], xf[8], o[8];
      unpack(g[u], gf);
      unpack(xv[u], xf);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = fmaf(a[k], gf[k], fmaf(bx[k], xf[k], cc[k]));
      u32x4v w;
      w.x = pack_bf2(o[0], o[1]);
      w.y = pack_bf2(o[2], o[3]);
      w.z = pack_bf2(o[4], o[5]);
      w.w = pack_bf2(o[6], o[7]);
      *reinterpret_cast<u32x4v*>(dx + (m0 + m) * C_ + c0) = w;
      *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(sdx + m * (C_ * 2) + ((c8 ^ mc_swz<CH8>(m)) << 4)) = w;
    }
    const bool more = b + G < nblk;
    if (more) issue(b + G, slot ^ 1);
    // act(b) landed: younger are this block's U dx stores and, when issued, block b+1's DMA and 2 U loads
    if (more) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(U + PIECES + 2 * U) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(U) : "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);  // no fragment read moves above the barrier
    v8bf fa[C_ / 16], fb[4];
#pragma unroll
    for (int i = 0; i < C_ / 16; ++i) fa[i] = frag_mc<C_>(sdx, i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = frag_mc<CI>(sact + slot * kACTL, wave * 64 + j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < C_ / 16; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the dx image and this act slot are free for the next block
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // lane (q = l & 15, gq = l >> 4) of tile (i, j) holds dW row 16 i + 4 gq + r, column 64 w + 16 j + q
  float* slab = slabs + (long long)gid * C_ * CI;
  const int q = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int i = 0; i < C_ / 16; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(i * 16 + gq * 4 + r) * CI + wave * 64 + j * 16 + q] = acc[i][j][r];
}

template <int C_, int CI>
int dxT_wgrad_grid() {
  static int G = 0;
  if (G == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DTG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bn_dxT_wgrad_kernel<C_, CI>, CI, 0));
    G = cus * (per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu));
    G -= G % 8;  // a multiple of the XCD count
    if (G < 8) G = 8;
  }
  return G;
}

bool transposed(int C, int CI) { return (C == 64 && CI == 256) || (C == 128 && (CI == 256 || CI == 512)); }

}  // namespace

namespace lab {
// dx = a * dp + bx * x + c (coef = [a, bx, c], fp32 [3 C]) and wgrad (fp32 [C, CI]) += dx^T act; slabs: G x C x CI
// fp32 (bn_dxT_wgrad_slabs); false if the shape is not one the kernel serves
int bn_dxT_wgrad_slabs(int C, int CI) {
  if (!transposed(C, CI)) return 0;
  return C == 64 ? dxT_wgrad_grid<64, 256>() : CI == 256 ? dxT_wgrad_grid<128, 256>() : dxT_wgrad_grid<128, 512>();
}

bool bn_dxT_wgrad(const bf16_t* dp, const bf16_t* x, const float* coef, bf16_t* dx, const bf16_t* act,
                  long long ldact, float* wgrad, float* slabs, long long M, int C, int CI, hipStream_t st) {
  if (!transposed(C, CI) || M % kDR || M < 64LL * kDR) return false;
  const int nblk = (int)(M / kDR);
  auto launchT = [&](auto kern, int G) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(CI), 0, st, dp, x, coef, dx, act, ldact, slabs, nblk);
    DTG_LAUNCH_CHECK();
    return G;
  };
  const int G = C == 64 ? launchT(bn_dxT_wgrad_kernel<64, 256>, dxT_wgrad_grid<64, 256>())
                : CI == 256 ? launchT(bn_dxT_wgrad_kernel<128, 256>, dxT_wgrad_grid<128, 256>())
                            : launchT(bn_dxT_wgrad_kernel<128, 512>, dxT_wgrad_grid<128, 512>());
  Epi e{wgrad, CI, 0, 1.f, 1.f, nullptr, 0};
  gemm_splitk_reduce(slabs, G, C, CI, e, st);
  return true;
}
}  // namespace lab
}  // namespace dtg
