// BatchNorm backward dx pass + the weight gradient of the 1x1 conv that produced the BN's input, fused:
//
//   dx  = a * dp + bx * x + c           (per channel; [M, C] bf16, the conv3 output gradient)
//   dx2 = a2 * dp + bx2 * x2 + c2       (projection blocks: the shortcut BN fed by the same dp, optional)
//   dW += dx^T act                      ([C, CI] fp32: conv3's weight gradient, act = its input [M, CI])
//
// ResNet-50's stage-1 conv3 weight gradient read dx (1.64 GB at batch 1024) back from HBM on the side stream
// right after this pass wrote it, and the backward is HBM-bound across both streams: skipping those three
// weight gradients made the step 0.9 ms faster (profiles/r04_dx_wgrad).  Here the dx tile never leaves the
// chip for the weight gradient: each persistent workgroup (4 waves) computes dx for a 32-row block in
// registers, stores it to HBM (for the conv3 dgrad) AND into LDS in the MN-contiguous layout of the wgrad
// operand (the chunk XOR of stage_mc, so frag_mc's transposed reads apply), stages the 32 x CI block of
// `act` by LDS-DMA, and accumulates dW = dx^T act for the whole kernel in registers (wave w: channels
// [64 w, +64) x all CI columns).  The per-workgroup partial is written to a slab and the slabs are summed into
// the fp32 gradient by the split-K reduction (gemm_splitk_reduce, beta = 1).
// A workgroup covers a 256-channel slice of dx (4 waves x 64 channels) and the matching 256 rows of dW: C = 256,
// CI = 64 (ResNet-50 stage 1) or C = 512, CI = 128 (stage 2: two slices per row block, the act block read by
// both from L2 -- the two workgroups of a row block are consecutive on one XCD).
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"

namespace dtg {

namespace {
using namespace gemm;

constexpr int kDC = 256;   // channels of one workgroup's slice
constexpr int kDR = 32;    // rows per block
constexpr int kDX_LDS = kDR * kDC * 2;   // 16 KB: dx block, [32 m][256 c] MC image

// W2 (with DUAL): also dW2 += dx2^T act2 -- the stride-1 projection shortcut's weight gradient (stage 1)
template <int CI, bool DUAL, bool W2 = false>
__global__ void __launch_bounds__(256, (CI == 64 && !W2) ? 2 : 1) bn_dx_wgrad_kernel(const bf16_t* __restrict__ dp, const bf16_t* __restrict__ x,
                                                          const float* __restrict__ coef,
                                                          const bf16_t* __restrict__ x2,
                                                          const float* __restrict__ coef2, bf16_t* __restrict__ dx,
                                                          bf16_t* __restrict__ dx2, const bf16_t* __restrict__ act,
                                                          long long ldact, float* __restrict__ slabs, int nblk,
                                                          int C, const bf16_t* __restrict__ act2, long long ldact2,
                                                          float* __restrict__ slabs2) {
  static_assert(!W2 || (DUAL && CI == 64), "the second weight gradient is the dual form's, at 256 x 64");
  constexpr int kACT_LDS = kDR * CI * 2;  // act block, [32 m][CI] MC image (two slots)
  constexpr int NJ = CI / 16;             // dW column tiles per wave
  constexpr int NX = W2 ? 2 : 1;  // dx images / act slot pairs
  __shared__ __attribute__((aligned(16))) char smem_raw[NX * (kDX_LDS + 2 * kACT_LDS)];
  lds_char* sdx = (lds_char*)smem_raw;
  lds_char* sact = sdx + kDX_LDS;
  lds_char* sdx2 = sact + 2 * kACT_LDS;  // W2 only
  lds_char* sact2 = sdx2 + kDX_LDS;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;  // a multiple of 8 and of the slice count (host)
  const int ns = C / kDC, gid = xcd_remap(blockIdx.x, G);
  const int sl = gid % ns;  // this workgroup's channel slice (fixed: G % ns == 0)
  // elementwise part: thread = (8-channel chunk c8, row slot rs); rows rs + 8 u, u < 4
  const int c8 = tid & 31, rs = tid >> 5, c0 = sl * kDC + c8 * 8;
  float a[8], bx[8], cc[8], a2[8], bx2[8], cc2[8];
  load8_f32(coef + c0, a);
  load8_f32(coef + C + c0, bx);
  load8_f32(coef + 2 * C + c0, cc);
  if constexpr (DUAL) {
    load8_f32(coef2 + c0, a2);
    load8_f32(coef2 + C + c0, bx2);
    load8_f32(coef2 + 2 * C + c0, cc2);
  }
  DenseMC<false> sa{act, ldact, CI, 0};
  DenseMC<false> sa2{act2, ldact2, CI, 0};
  f32x4 acc[4][NJ], acc2[W2 ? 4 : 1][W2 ? NJ : 1];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if constexpr (W2) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc2[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // Software-pipelined over this workgroup's blocks: block b+1's act DMA and dp / x loads are issued right after
  // block b's dx is stored, so they are in flight under block b's MFMAs and barriers.
  auto unpack = [](const u32x4v& v, float (&f)[8]) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
  };
  u32x4v g[4], xv[4], x2v[4];  // raw bf16 until used: 12 registers per row instead of 24
  auto issue = [&](int b, int slot) {
    const long long m0 = (long long)b * kDR;
    stage_mc<CI, DenseMC<false>, 4, kDR>(sa, sact + slot * kACT_LDS, 0, (int)m0, wave, lane);
    if constexpr (W2) stage_mc<CI, DenseMC<false>, 4, kDR>(sa2, sact2 + slot * kACT_LDS, 0, (int)m0, wave, lane);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long off = (m0 + rs + 8 * u) * C + c0;
      g[u] = *reinterpret_cast<const u32x4v*>(dp + off);
      xv[u] = *reinterpret_cast<const u32x4v*>(x + off);
      if constexpr (DUAL) x2v[u] = *reinterpret_cast<const u32x4v*>(x2 + off);
    }
  };
  // tiles t = gid + it G: row block t / ns, slice t % ns = sl
  const int b0 = gid / ns, gb = G / ns;
  if (b0 < nblk) issue(b0, 0);
  int slot = 0;
  for (int b = b0; b < nblk; b += gb, slot ^= 1) {
    const long long m0 = (long long)b * kDR;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int m = rs + 8 * u;
      const long long off = (m0 + m) * C + c0;
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
      *reinterpret_cast<u32x4v*>(dx + off) = w;
      // [m][256 c] image, 16-B chunk c8 at position c8 ^ mc_swz<32>(m) (stage_mc's layout)
      *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(sdx + m * (kDC * 2) +
                                                                   ((c8 ^ mc_swz<kDC / 8>(m)) << 4)) = w;
      if constexpr (DUAL) {
        float x2f[8], o2[8];
        unpack(x2v[u], x2f);
#pragma unroll
        for (int k = 0; k < 8; ++k) o2[k] = fmaf(a2[k], gf[k], fmaf(bx2[k], x2f[k], cc2[k]));
        u32x4v w2;
        w2.x = pack_bf2(o2[0], o2[1]);
        w2.y = pack_bf2(o2[2], o2[3]);
        w2.z = pack_bf2(o2[4], o2[5]);
        w2.w = pack_bf2(o2[6], o2[7]);
        *reinterpret_cast<u32x4v*>(dx2 + off) = w2;
        if constexpr (W2)
          *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(sdx2 + m * (kDC * 2) +
                                                                       ((c8 ^ mc_swz<kDC / 8>(m)) << 4)) = w2;
      }
    }
    const bool more = b + gb < nblk;
    if (more) issue(b + gb, slot ^ 1);
    // act(b) landed: younger are this block's dx stores (4, DUAL 8) and, when issued, block b+1's DMA (CI / 64
    // pieces) and loads (8, DUAL 12); the dx image is written; then both are visible to every wave
    constexpr int PIECES = (CI / 64) * (W2 ? 2 : 1);
    if (more) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(DUAL ? 8 + PIECES + 12 : 4 + PIECES + 8) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(DUAL ? 8 : 4) : "memory");
    __builtin_amdgcn_s_barrier();
    // dW[64 wave + 16 i + .., 16 j + ..] += dx^T act over the block's 32 rows (one 32-deep k-step)
    v8bf fa[4], fb[NJ];
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i] = frag_mc<kDC>(sdx, wave * 64 + i * 16, 0, lane);
#pragma unroll
    for (int j = 0; j < NJ; ++j) fb[j] = frag_mc<CI>(sact + slot * kACT_LDS, j * 16, 0, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if constexpr (W2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = frag_mc<kDC>(sdx2, wave * 64 + i * 16, 0, lane);
#pragma unroll
      for (int j = 0; j < NJ; ++j) fb[j] = frag_mc<CI>(sact2 + slot * kACT_LDS, j * 16, 0, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc2[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc2[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // the dx image is free for the next block
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // this workgroup's partial: rows [256 sl, +256) of slab gid / ns ([C][CI]); lane (q = l & 15, g = l >> 4) of
  // tile (i, j) holds rows 64 w + 16 i + 4 g + r of the slice, column 16 j + q
  float* slab = slabs + ((long long)(gid / ns) * C + sl * kDC) * CI;
  const int q = lane & 15, gq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) slab[(wave * 64 + i * 16 + gq * 4 + r) * CI + j * 16 + q] = acc[i][j][r];
  if constexpr (W2) {
    float* slab2 = slabs2 + ((long long)(gid / ns) * C + sl * kDC) * CI;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) slab2[(wave * 64 + i * 16 + gq * 4 + r) * CI + j * 16 + q] = acc2[i][j][r];
  }
}

template <int CI, bool W2 = false>
int dx_wgrad_grid() {
  static int G = 0;
  if (G == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DTG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bn_dx_wgrad_kernel<CI, true, W2>, 256, 0));
    G = cus * (per_cu < 1 ? 1 : (per_cu > 2 ? 2 : per_cu));
    G -= G % 8;  // a multiple of 8 (the XCD count) and so of the slice count (<= 2) on any CU count
    if (G < 8) G = 8;
  }
  return G;
}

}  // namespace

bool bn_dx_wgrad_ok(long long M, int C, int CI) {
  return ((C == 256 && CI == 64) || (C == 512 && CI == 128)) && M % kDR == 0 && M >= 64LL * kDR;
}

int bn_dx_wgrad_slabs(int C, int CI, int w2) {
  return (w2 ? dx_wgrad_grid<64, true>() : CI == 64 ? dx_wgrad_grid<64>() : dx_wgrad_grid<128>()) / (C / kDC);
}

// dx (+ dx2) from the finalized coefficients (bn_bwd_coef_from_part: coef = [a, bx, c]) and dW += dx^T act (+ with
// act2: dW2 += dx2^T act2, dual form at 256 x 64 only, slabs2 like slabs, wgrad2 of wgrad's dtype);
// slabs: bn_dx_wgrad_slabs(C, CI) x C x CI fp32 workspace; wgrad fp32 or bf16 (the flat gradient's compute dtype)
void bn_dx_wgrad(const bf16_t* dp, const bf16_t* x, const float* coef, const bf16_t* x2, const float* coef2,
                 bf16_t* dx, bf16_t* dx2, const bf16_t* act, long long ldact, void* wgrad, int wgrad_bf16,
                 float* slabs, long long M, int C, int CI, hipStream_t st, const bf16_t* act2, long long ldact2,
                 void* wgrad2, float* slabs2) {
  const int nblk = (int)(M / kDR);
  auto launch = [&](auto kern, int G) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, st, dp, x, coef, x2, coef2, dx, dx2, act, ldact, slabs, nblk, C,
                       act2, ldact2, slabs2);
    DTG_LAUNCH_CHECK();
    return G;
  };
  int G;
  if (act2) {
    G = launch(bn_dx_wgrad_kernel<64, true, true>, dx_wgrad_grid<64, true>());
    Epi e2{wgrad2, CI, wgrad_bf16, 1.f, 1.f, nullptr, 0};
    gemm_splitk_reduce(slabs2, G / (C / kDC), C, CI, e2, st);
  } else if (CI == 64) G = x2 ? launch(bn_dx_wgrad_kernel<64, true>, dx_wgrad_grid<64>())
                              : launch(bn_dx_wgrad_kernel<64, false>, dx_wgrad_grid<64>());
  else G = x2 ? launch(bn_dx_wgrad_kernel<128, true>, dx_wgrad_grid<128>())
              : launch(bn_dx_wgrad_kernel<128, false>, dx_wgrad_grid<128>());
  Epi e{wgrad, CI, wgrad_bf16, 1.f, 1.f, nullptr, 0};
  gemm_splitk_reduce(slabs, G / (C / kDC), C, CI, e, st);
}

}  // namespace dtg
