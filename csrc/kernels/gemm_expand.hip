// Streaming "expand" GEMM + BatchNorm statistics: C[M, N] = A[M, K] W[N, K]^T with the per-channel sum and
// sum of squares of the stored (bf16-rounded) outputs, for short reductions (K = 64 / 128 / 256) into wide outputs
// (N a multiple of 256): ResNet-50's conv3 / projection 1x1 convs of stages 1-2 (3211264 x 256 x 64 and
// 802816 x 512 x 128 at batch 1024), whose time is the output write, not the MFMAs.
//
// The tiled GEMM (gemm.hip, 128x128 tiles) runs these at 3.2-3.6 TB/s: with one or two K-steps per tile every
// workgroup pays a whole pipeline fill, a staged LDS epilogue and a block reduction + atomics for its 128x128
// statistics (27 % of the kernel on the stage-1 shape, profiles/r04_expand).  Here
//   * a persistent workgroup (4 waves) owns one 256-column slice and walks 64-row blocks of A;
//   * its W slice is loaded ONCE into registers (fragment layout, 32 / 64 VGPRs for K = 64 / 128);
//   * A blocks stream through a 3-deep LDS-DMA ring with counted vmcnt waits (the DMA of block i+2 is in
//     flight under block i's MFMAs and stores; the output stores stay in flight across iterations);
//   * the MFMA operands are swapped (W fragment as src A) and W's rows are fed permuted, so a lane's four
//     accumulators of a 16-row m-tile hold two runs of 8 consecutive output columns of one row: the epilogue
//     stores straight from registers (2 x 16 B per lane and m-tile; the 4 lanes of a row write 64 contiguous
//     bytes per store instruction) and accumulates the column statistics in registers over every row the
//     workgroup writes -- one shuffle reduction and 32 atomics per lane group per KERNEL instead of an LDS
//     reduction per tile.
// Wave w covers columns [64 w, +64) of the slice; lane l (q = l & 15, g = l >> 4) of n-tile j is fed W row
// 32 (j >> 1) + 8 (q >> 2) + 4 (j & 1) + (q & 3), so D[4 g + r][q] of n-tile j is column
// 32 (j >> 1) + 8 g + 4 (j & 1) + r, row q of the m-tile.
//
// Statistics layout = the tiled path's (gemm_bf16_bn mode 1): part[slot][2][N], slot = workgroup % 32, added
// atomically into a zeroed buffer and reduced by bn_finalize.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"

namespace dtg {

namespace {
using namespace gemm;

constexpr int kXR = 64;  // rows per block
constexpr int kXS = 3;   // A ring depth

// Row gather of a 1x1 / stride-2 conv (S2): output row m = (n, p, q) of the P x Q grid reads input pixel (n, 2p, 2q)
// of the H x W NHWC input (lda = channels)
struct ExpandGather {
  int H, W;
  FastDiv fPQ, fQ;
};

// NT: non-temporal output stores; MINB: workgroups per CU the register allocation must allow (0: free)
template <int K, bool NT, int MINB, bool S2 = false>
__global__ void __launch_bounds__(256, MINB > 0 ? MINB : 1) gemm_expand_bn_kernel(const bf16_t* __restrict__ A, long long lda,
                                                             const bf16_t* __restrict__ W, long long ldw,
                                                             bf16_t* __restrict__ C, long long ldc,
                                                             float* __restrict__ part, int N, int nslice, int tiles,
                                                             ExpandGather gth) {
  constexpr int KS = K / 32;                // MFMA k-steps
  constexpr int KH = K / 64;                // 64-deep halves of an A block (each a [64][64] KC image)
  constexpr int BLK = kXR * K * 2;          // bytes of one A block
  constexpr int D = KH * 2;                 // LDS-DMA instructions per lane per block
  constexpr int T = 8;                      // 16-B stores per lane per block
  __shared__ __attribute__((aligned(16))) char smem_raw[kXS * BLK];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;                  // a multiple of 8 and of nslice (host)
  const int base = xcd_remap(blockIdx.x, G);  // consecutive logical ids share an XCD: the slices of a block too
  const int my = base < tiles ? (tiles - base + G - 1) / G : 0;
  if (my == 0) return;
  const int slice = base % nslice;          // fixed: G % nslice == 0
  const int col0 = slice * 256 + wave * 64;
  const int q = lane & 15, g = lane >> 4;

  // this wave's W fragments, once
  v8bf wf[4][KS];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int n = col0 + 32 * (j >> 1) + 8 * (q >> 2) + 4 * (j & 1) + (q & 3);
      wf[j][ks] = *reinterpret_cast<const v8bf*>(W + (long long)n * ldw + ks * 32 + 8 * g);
    }

  // A block of iteration `it` into ring slot it % kXS ([KH][64 rows][64 k] KC images, chunk XOR (row & 7)).
  // Past the last block the last one is loaded again (never read): every iteration issues exactly D
  // DMA instructions, so the counted waits below are uniform.
  // row block of iteration it: (base + it G) / nslice = rb0 + it * (G / nslice), as G % nslice == 0
  const int rb0 = base / nslice, gs = G / nslice;
  auto stage = [&](int it) {
    const int rb = rb0 + (it < my ? it : my - 1) * gs;
    lds_char* dst = smem + (it % kXS) * BLK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = (wave * 2 + i) * 8, r = r0 + (lane >> 3);
      const int c = (lane & 7) ^ (r & 7);
      long long arow = (long long)rb * kXR + r;  // the A row this lane's chunks come from
      if constexpr (S2) {
        uint32_t n, pq, pp, qq;
        gth.fPQ.divmod((uint32_t)arow, n, pq);
        gth.fQ.divmod(pq, pp, qq);
        arow = ((long long)n * gth.H + 2 * (int)pp) * gth.W + 2 * (int)qq;
      }
      const char* src = (const char*)(A + arow * lda + c * 8);
#pragma unroll
      for (int h = 0; h < KH; ++h)
        __builtin_amdgcn_global_load_lds((const void*)(src + h * 128), (lds_void*)(dst + h * kXR * 128 + r0 * 128), 16,
                                         0, 0);
    }
  };

  float s[16], sq[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) s[c] = sq[c] = 0.f;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  stage(0);
  stage(1);
  for (int it = 0; it < my; ++it) {
    // block `it` has landed once the ops issued after it are all that is left: DMA(it+1) (it = 0); DMA(it+1)
    // and stores(it-1) (it = 1); stores(it-2), DMA(it+1), stores(it-1) from then on
    if (it == 0) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
    else if (it == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D + T) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * T + D) : "memory");
    __builtin_amdgcn_s_barrier();  // every wave's part of block `it` is in LDS; slot (it - 1) % 3 is free
    stage(it + 2);
    const lds_char* ta = smem + (it % kXS) * BLK;
    const long long row0 = (long long)(rb0 + it * gs) * kXR;
    // one 16-row m-tile at a time: 4 independent accumulators (16 VGPRs) live, its epilogue overlapping the
    // next m-tile's MFMAs
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v8bf af[KS];
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) af[ks] = frag_kc(ta + (ks >> 1) * kXR * 128, 16 * i, ks & 1, lane);
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][0], af[0], zero4, 0, 0, 0);
#pragma unroll
      for (int ks = 1; ks < KS; ++ks)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], af[ks], acc[j], 0, 0, 0);
      u32x4v w0, w1;
      w0.x = pack_bf2(acc[0][0], acc[0][1]);
      w0.y = pack_bf2(acc[0][2], acc[0][3]);
      w0.z = pack_bf2(acc[1][0], acc[1][1]);
      w0.w = pack_bf2(acc[1][2], acc[1][3]);
      w1.x = pack_bf2(acc[2][0], acc[2][1]);
      w1.y = pack_bf2(acc[2][2], acc[2][3]);
      w1.z = pack_bf2(acc[3][0], acc[3][1]);
      w1.w = pack_bf2(acc[3][2], acc[3][3]);
      const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int c = 0; c < 8; ++c) {  // statistics of what the apply pass will read (the rounded values)
        const float lo = __uint_as_float(wd[c] << 16), hi = __uint_as_float(wd[c] & 0xffff0000u);
        s[2 * c] += lo;
        s[2 * c + 1] += hi;
        sq[2 * c] = fmaf(lo, lo, sq[2 * c]);
        sq[2 * c + 1] = fmaf(hi, hi, sq[2 * c + 1]);
      }
      bf16_t* dst = C + (row0 + 16 * i + q) * ldc + col0 + 8 * g;
      if constexpr (NT) {
        __builtin_nontemporal_store(w0, reinterpret_cast<u32x4v*>(dst));
        __builtin_nontemporal_store(w1, reinterpret_cast<u32x4v*>(dst + 32));
      } else {
        *reinterpret_cast<u32x4v*>(dst) = w0;
        *reinterpret_cast<u32x4v*>(dst + 32) = w1;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (dummy) DMAs land before the LDS is released

  // column statistics: sum over the 16 lanes (rows) of a lane group, then one atomic per column
#pragma unroll
  for (int c = 0; c < 16; ++c) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s[c] += __shfl_xor(s[c], o, 64);
      sq[c] += __shfl_xor(sq[c], o, 64);
    }
  }
  if (q == 0) {
    float* p = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * N + col0 + 8 * g;
#pragma unroll
    for (int c = 0; c < 16; ++c) {  // value c: column 8 g + c (c < 8), 32 + 8 g + c - 8 (c >= 8)
      const int off = c < 8 ? c : 24 + c;
      atomicAdd(p + off, s[c]);
      atomicAdd(p + N + off, sq[c]);
    }
  }
}

template <int K, bool NT, int MINB, bool S2 = false>
int expand_grid(int nslice) {
  static int per_cu = -1, cus = 0;
  if (per_cu < 0) {
    int dev = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DTG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gemm_expand_bn_kernel<K, NT, MINB, S2>, 256, 0));
    if (per_cu < 1) per_cu = 1;
  }
  int G = cus * per_cu;
  const int mult = nslice > 8 ? nslice : 8;  // a multiple of 8 and of nslice (a power of two)
  G -= G % mult;
  return G > 0 ? G : mult;
}

// ---- the ResNet stem conv as a streaming GEMM ------------------------------------------------------------
// The stem's 7x7/2 conv on pixel pairs (ops/conv.py stem_pairs: x8 [N, Hp, Wp/2, 8], 4 channels x 2 pixels per
// 16-B chunk, a (2, 1)-stride conv with R = 7 rows x S2 = 4 pair-columns = 28 taps, zero-padded to K = 256) has the
// shape of the expand GEMMs above: a short reduction into a write-bound output (12.8M pixels x 64 channels =
// 1.64 GB at batch 1024).  The tiled implicit GEMM (conv_fwd_c8, 256x64 tiles, 4 K-steps each) spent 820 us on
// it, twice its HBM time: every 256-row tile paid a pipeline fill and a staged epilogue with a block reduction of
// the BN statistics.  Here, as in gemm_expand_bn_kernel: persistent workgroups, all 64 x 256 weights in registers
// (wave w holds every column: 4 n-tiles x 8 k-steps, fed permuted), 64-row blocks of the gathered input through a
// 3-deep LDS-DMA ring (each lane's DMA source address is the gather), wave w computes m-tile w of each block and
// stores 2 x 16 B per lane straight from the MFMA registers, statistics in registers for the whole kernel.
struct StemStreamGeom {
  int Hp, Wp2, P, Q;
  FastDiv fPQ, fQ;
};

__global__ void __launch_bounds__(256, 2) stem_stream_bn_kernel(const bf16_t* __restrict__ x8,
                                                                 const bf16_t* __restrict__ W,
                                                                 bf16_t* __restrict__ C, float* __restrict__ part,
                                                                 StemStreamGeom sg, int nblocks) {
  constexpr int K = 256, KS = K / 32, KH = K / 64, N = 64;
  constexpr int BLK = kXR * K * 2;          // 32 KB: one 64-row block, [KH][64 rows][64 k] KC images
  constexpr int D = KH * 2;                 // LDS-DMA instructions per lane per block
  constexpr int T = 2;                      // 16-B stores per lane per block (one m-tile per wave)
  constexpr int TAPS = 28;                  // 7 rows x 4 pair-columns; taps 28..31 read the zero page
  constexpr int RING = 2;                   // LDS slots (2 x 32 KB: two workgroups per CU)
  __shared__ __attribute__((aligned(16))) char smem_raw[RING * BLK];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int G = gridDim.x;
  const int base = xcd_remap(blockIdx.x, G);  // consecutive logical ids (and so neighbouring blocks) share an XCD
  const int my = base < nblocks ? (nblocks - base + G - 1) / G : 0;
  if (my == 0) return;
  const int q = lane & 15, g = lane >> 4;

  v8bf wf[4][KS];  // every output column: n-tile j, fed permuted (see gemm_expand_bn_kernel)
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int n = 32 * (j >> 1) + 8 * (q >> 2) + 4 * (j & 1) + (q & 3);
      wf[j][ks] = *reinterpret_cast<const v8bf*>(W + (long long)n * K + ks * 32 + 8 * g);
    }

  // block of iteration it = logical block base + it G; past the last block the last one is loaded again (never
  // read), so every iteration issues exactly D DMA instructions and the counted waits stay uniform
  auto stage = [&](int it) {
    const int rb = base + (it < my ? it : my - 1) * G;
    lds_char* dst = smem + (it % RING) * BLK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r0 = (wave * 2 + i) * 8, r = r0 + (lane >> 3);
      uint32_t n, pq, p, qq;
      sg.fPQ.divmod((uint32_t)(rb * kXR + r), n, pq);
      sg.fQ.divmod(pq, p, qq);
      const bf16_t* rowp = x8 + (((long long)n * sg.Hp + 2 * (int)p) * sg.Wp2 + (int)qq) * 8;
#pragma unroll
      for (int h = 0; h < KH; ++h) {
        const int t = 8 * h + ((lane & 7) ^ (r & 7));  // the tap whose chunk belongs at this lane's LDS position
        const void* src = sel(t < TAPS, rowp + ((t >> 2) * sg.Wp2 + (t & 3)) * 8);
        __builtin_amdgcn_global_load_lds(src, (lds_void*)(dst + h * kXR * 128 + r0 * 128), 16, 0, 0);
      }
    }
  };

  float s[16], sq[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) s[c] = sq[c] = 0.f;
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  stage(0);
  for (int it = 0; it < my; ++it) {
    // block `it` landed once only the stores of block it-1 (issued after its DMA) can still be in flight; the other
    // workgroup of the CU hides this one's DMA latency (a 3-slot ring at one workgroup per CU measured the same)
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(T) : "memory");
    __builtin_amdgcn_s_barrier();  // every wave's part of block `it` is in LDS; the slot of block it-1 is free
    __builtin_amdgcn_sched_barrier(0);
    stage(it + RING - 1);
    const lds_char* ta = smem + (it % RING) * BLK;
    const long long row0 = (long long)(base + it * G) * kXR;
    v8bf af[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) af[ks] = frag_kc(ta + (ks >> 1) * kXR * 128, 16 * wave, ks & 1, lane);
    f32x4 acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][0], af[0], zero4, 0, 0, 0);
#pragma unroll
    for (int ks = 1; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][ks], af[ks], acc[j], 0, 0, 0);
    u32x4v w0, w1;
    w0.x = pack_bf2(acc[0][0], acc[0][1]);
    w0.y = pack_bf2(acc[0][2], acc[0][3]);
    w0.z = pack_bf2(acc[1][0], acc[1][1]);
    w0.w = pack_bf2(acc[1][2], acc[1][3]);
    w1.x = pack_bf2(acc[2][0], acc[2][1]);
    w1.y = pack_bf2(acc[2][2], acc[2][3]);
    w1.z = pack_bf2(acc[3][0], acc[3][1]);
    w1.w = pack_bf2(acc[3][2], acc[3][3]);
    const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int c = 0; c < 8; ++c) {  // statistics of what the BN pass will read (the rounded values)
      const float lo = __uint_as_float(wd[c] << 16), hi = __uint_as_float(wd[c] & 0xffff0000u);
      s[2 * c] += lo;
      s[2 * c + 1] += hi;
      sq[2 * c] = fmaf(lo, lo, sq[2 * c]);
      sq[2 * c + 1] = fmaf(hi, hi, sq[2 * c + 1]);
    }
    bf16_t* dst = C + (row0 + 16 * wave + q) * N + 8 * g;
    *reinterpret_cast<u32x4v*>(dst) = w0;
    *reinterpret_cast<u32x4v*>(dst + 32) = w1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (dummy) DMAs land before the LDS is released
#pragma unroll
  for (int c = 0; c < 16; ++c) {
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      s[c] += __shfl_xor(s[c], o, 64);
      sq[c] += __shfl_xor(sq[c], o, 64);
    }
  }
  if (q == 0) {
    float* pp = part + (long long)(blockIdx.x % kBnStatSlots) * 2 * N + 8 * g;
#pragma unroll
    for (int c = 0; c < 16; ++c) {  // value c: column 8 g + c (c < 8), 32 + 8 g + c - 8 (c >= 8)
      const int off = c < 8 ? c : 24 + c;
      atomicAdd(pp + off, s[c]);
      atomicAdd(pp + N + off, sq[c]);
    }
  }
}

}  // namespace

// K = 256 (ResNet-50's stage-3 conv3, 200704 x 1024 x 256 at batch 1024, 64x256 tiles at 2.6 TB/s before): the
// same kernel with a 96 KB ring (one workgroup per CU) and 128 VGPRs of weights per lane.  Switch for the A/B tools.
static int g_expand_k256 = 1;
void gemm_expand_k256_set(int on) { g_expand_k256 = on; }

// false (nothing launched): not a shape this kernel serves, the caller takes the tiled path
bool gemm_expand_bn(const bf16_t* A, long long lda, const bf16_t* W, long long ldw, bf16_t* C, long long ldc, int M,
                    int N, int K, float* part, hipStream_t st, int variant) {
  if ((K != 64 && K != 128 && !(K == 256 && g_expand_k256)) || N % 256 || M % kXR || (lda & 7) || (ldw & 7) ||
      (ldc & 7))
    return false;
  if ((long long)M * N < (1LL << 24)) return false;  // small problems: the tiled path fills the chip better
  const int nslice = N / 256;
  if (nslice & (nslice - 1)) return false;  // 1, 2, 4, ... (grid divisibility)
  const int tiles = (M / kXR) * nslice;
  auto launch = [&](auto kern, int G) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(256), 0, st, A, lda, W, ldw, C, ldc, part, N, nslice, tiles, ExpandGather());
  };
  // variant (A/B tool only): 0 default, 1 non-temporal stores, 2 registers for 3 workgroups per CU
  if (K == 64) {
    if (variant == 1) launch(gemm_expand_bn_kernel<64, true, 0>, expand_grid<64, true, 0>(nslice));
    else if (variant == 2) launch(gemm_expand_bn_kernel<64, false, 3>, expand_grid<64, false, 3>(nslice));
    else launch(gemm_expand_bn_kernel<64, false, 0>, expand_grid<64, false, 0>(nslice));
  } else if (K == 256) {
    launch(gemm_expand_bn_kernel<256, false, 0>, expand_grid<256, false, 0>(nslice));
  } else {
    if (variant == 1) launch(gemm_expand_bn_kernel<128, true, 0>, expand_grid<128, true, 0>(nslice));
    else if (variant == 2) launch(gemm_expand_bn_kernel<128, false, 2>, expand_grid<128, false, 2>(nslice));
    else launch(gemm_expand_bn_kernel<128, false, 0>, expand_grid<128, false, 0>(nslice));
  }
  DTG_LAUNCH_CHECK();
  return true;
}

// 1x1 / stride-2 conv + BN statistics with 256 input channels (ResNet-50's stage-2 projection, 56x56x256 -> 28x28x512
// at batch 1024: 414 us on the implicit-GEMM conv, 508 TF/s): the K = 256 expand kernel with the stride-2 row
// gather.  x [Nb, H, W, 256] NHWC, w [Kout][256], y [Nb * H/2 * W/2][Kout].  Switch for the A/B tools.
static int g_expand_s2 = 1;
void gemm_expand_s2_set(int on) { g_expand_s2 = on; }

bool conv1x1_s2_expand_bn(const bf16_t* x, int Nb, int H, int W, int Cin, const bf16_t* w, bf16_t* y, int Kout,
                          float* part, hipStream_t st) {
  if (!g_expand_s2 || Cin != 256 || Kout % 256 || (H & 1) || (W & 1)) return false;
  const int P = H / 2, Q = W / 2;
  const long long M = (long long)Nb * P * Q;
  if (M % kXR || M >= (1LL << 31) || (long long)Nb * H * W * Cin >= (1LL << 40)) return false;
  if (M * Kout < (1LL << 24)) return false;
  const int nslice = Kout / 256;
  if (nslice & (nslice - 1)) return false;
  ExpandGather gth;
  gth.H = H;
  gth.W = W;
  gth.fPQ = FastDiv((uint32_t)(P * Q));
  gth.fQ = FastDiv((uint32_t)Q);
  const int tiles = (int)(M / kXR) * nslice;
  hipLaunchKernelGGL((gemm_expand_bn_kernel<256, false, 0, true>), dim3(expand_grid<256, false, 0, true>(nslice)),
                     dim3(256), 0, st, x, (long long)Cin, w, (long long)Cin, y, (long long)Kout, part, Kout, nslice, tiles,
                     gth);
  DTG_LAUNCH_CHECK();
  return true;
}

// The stem conv of ResNet (pixel-pair form: x8 [N, Hp, Wp2, 8], w8 [64][256], (2, 1) stride, P x Q output) with the
// BN statistics into part (kBnStatSlots x 2 x 64, zeroed); false if the geometry is not that one
static int g_stem_stream = 1;
void stem_stream_set(int on) { g_stem_stream = on; }

bool stem_conv_stream_bn(const bf16_t* x8, const bf16_t* w8, bf16_t* y, int N, int Hp, int Wp2, int P, int Q,
                         float* part, hipStream_t st) {
  if (!g_stem_stream) return false;
  const long long M = (long long)N * P * Q;
  if (M % kXR || M / kXR > (1LL << 30) || (long long)N * Hp * Wp2 * 8 >= (1LL << 31)) return false;
  if (2 * (P - 1) + 7 > Hp || (Q - 1) + 4 > Wp2) return false;  // every tap inside the padded input
  StemStreamGeom sg;
  sg.Hp = Hp;
  sg.Wp2 = Wp2;
  sg.P = P;
  sg.Q = Q;
  sg.fPQ = FastDiv((uint32_t)(P * Q));
  sg.fQ = FastDiv((uint32_t)Q);
  static int G = 0;
  if (G == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    DTG_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, stem_stream_bn_kernel, 256, 0));
    G = cus * (per_cu < 1 ? 1 : per_cu);
    G -= G % 8;
    if (G < 8) G = 8;
  }
  hipLaunchKernelGGL(stem_stream_bn_kernel, dim3(G), dim3(256), 0, st, x8, w8, y, part, sg, (int)(M / kXR));
  DTG_LAUNCH_CHECK();
  return true;
}

}  // namespace dtg
