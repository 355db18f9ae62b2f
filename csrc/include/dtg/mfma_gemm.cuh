// MFMA GEMM core for gfx950 (CDNA4), shared by dense GEMM and implicit-GEMM convolution.
//
//   C[M,N] (+)= A[M,K] * B[K,N]        bf16 inputs, fp32 accumulate (v_mfma_f32_16x16x32_bf16)
//
// Tiling: 256 threads = 4 waves (2x2), block tile BM x BN x BK = 128 x 128 x 64, each wave owns a
// 64x64 sub-tile = 4x4 MFMA 16x16 accumulators (64 acc VGPRs).  Operand tiles are staged HBM->LDS
// with global_load_lds_dwordx4 (LDS-DMA, 1 KiB per wave-instruction, no VGPR round trip) into a
// 2-deep LDS ring (64 KiB: 2 blocks/CU), one barrier per K-step.
//
// Each operand is either
//   KC  ("K-contiguous")  : element (row, k) at base(row) + k          -> LDS [rows][64]  128 B rows,
//        16-B chunk XOR-swizzled by (row & 7); fragments by ds_read_b128
//   MC  ("MN-contiguous") : element (k, col) at base(k) + col          -> LDS [64][rows]  256 B rows,
//        16-B chunk XOR-swizzled by 2*f(k); fragments by 2x ds_read_b64_tr_b16 (hardware transpose)
// so the three training GEMMs (fwd X*W^T, dgrad dY*W, wgrad dY^T*X) all run without explicit
// transposes.  With LDS-DMA the destination is lane-linear, so the swizzle is applied to the
// per-lane SOURCE address and undone on the read (cdna_hip_programming.md §5.4 rule 21).
//
// Where an operand comes from is a policy object (`Src`) returning the global address of the
// 16-byte chunk a lane must fetch; dense strided matrices and im2col gathers (conv.hip) plug in
// here.  A chunk that lies outside the matrix returns the address of a zero page.
#pragma once
#include "dtg/common.h"

namespace dtg {
namespace gemm {

typedef __attribute__((ext_vector_type(8))) __bf16 v8bf;
typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) v4bf lds_v4bf;

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;               // 16 KiB per operand per stage
constexpr int LDS_BYTES = 2 * 2 * TILE_BYTES;          // 2 operands x 2 stages

// 16-byte zero page in global memory for out-of-range chunks (glds needs a global source).
__device__ __attribute__((aligned(64))) static const bf16_t g_zero_page[32] = {0};

__device__ __forceinline__ const void* zero_src() { return (const void*)g_zero_page; }

// swizzle of the 16-B chunk index (0..15) of a 256-B MC row; keeps 32-B pairs together and makes
// the 8 rows read by one ds_read_b64_tr_b16 half-wave distinct (conflict-free)
__device__ __forceinline__ int mc_swz(int k) { return (((k & 3) | (((k >> 3) & 1) << 2)) << 1); }

// ---- dense sources -------------------------------------------------------------------------
// KC: matrix stored [rows][ld] with k contiguous
struct DenseKC {
  const bf16_t* p;
  long long ld;
  int rows, K;
  __device__ __forceinline__ const void* chunk(int row, int k) const {
    if (k >= K) return zero_src();
    if (row >= rows) row = rows - 1;
    return p + (long long)row * ld + k;
  }
};
// MC: matrix stored [K][ld] with the row/col (M or N) index contiguous
struct DenseMC {
  const bf16_t* p;
  long long ld;
  int cols, K;
  __device__ __forceinline__ const void* chunk(int krow, int col) const {
    if (krow >= K || col >= cols) return zero_src();
    return p + (long long)krow * ld + col;
  }
};

// ---- staging ---------------------------------------------------------------------------------
// KC tile: 128 rows x 64 k; wave-instruction i covers 8 rows; 16 instructions per tile, 4 per wave
template <class Src>
__device__ __forceinline__ void stage_kc(const Src& src, char* lds_tile, int row0, int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r0 = (wave * 4 + i) * 8;
    const int r = r0 + (lane >> 3);
    const int cl = lane & 7;           // linear chunk position in LDS
    const int c = cl ^ (r & 7);        // source chunk that belongs there
    const void* g = src.chunk(row0 + r, k0 + c * 8);
    __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_tile + r0 * 128), 16, 0, 0);
  }
}

// MC tile: 64 k-rows x 128 cols; wave-instruction covers 4 k-rows; 16 per tile, 4 per wave
template <class Src>
__device__ __forceinline__ void stage_mc(const Src& src, char* lds_tile, int col0, int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kr0 = (wave * 4 + i) * 4;
    const int kr = kr0 + (lane >> 4);
    const int cl = lane & 15;
    const int c = cl ^ mc_swz(kr);
    const void* g = src.chunk(k0 + kr, col0 + c * 8);
    __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_tile + kr0 * 256), 16, 0, 0);
  }
}

// ---- fragment reads (one 16x32 operand fragment for mfma_f32_16x16x32_bf16) --------------------
// lane l holds X[r0 + (l&15)][ks*32 + 8*(l>>4) + j], j = 0..7
__device__ __forceinline__ v8bf frag_kc(const char* lds_tile, int r0, int ks, int lane) {
  const int r = r0 + (lane & 15);
  const int c = ks * 4 + (lane >> 4);
  return *reinterpret_cast<const v8bf*>(lds_tile + r * 128 + ((c ^ (r & 7)) << 4));
}

__device__ __forceinline__ v8bf frag_mc(const char* lds_tile, int r0, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int kA = ks * 32 + 8 * g + q;   // rows for elements 0..3
  const int kB = kA + 4;                // rows for elements 4..7
  const int ch = (r0 >> 3) + (p >> 1);  // 16-B chunk of columns r0+4p .. r0+4p+3
  const int sub = (p & 1) * 8;
  const char* a = lds_tile + kA * 256 + ((ch ^ mc_swz(kA)) << 4) + sub;
  const char* b = lds_tile + kB * 256 + ((ch ^ mc_swz(kB)) << 4) + sub;
  const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(a));
  const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(b));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <bool KC>
__device__ __forceinline__ v8bf frag(const char* t, int r0, int ks, int lane) {
  if constexpr (KC) return frag_kc(t, r0, ks, lane);
  else return frag_mc(t, r0, ks, lane);
}

template <bool KC, class Src>
__device__ __forceinline__ void stage(const Src& s, char* t, int rc0, int k0, int wave, int lane) {
  if constexpr (KC) stage_kc(s, t, rc0, k0, wave, lane);
  else stage_mc(s, t, rc0, k0, wave, lane);
}

// ---- main loop -------------------------------------------------------------------------------
// Accumulates the K range [kbeg, kend) of tile (bm, bn) into acc[4][4].
template <bool AKC, bool BKC, class SA, class SB>
__device__ __forceinline__ void mainloop(const SA& sa, const SB& sb, char* smem, int bm0, int bn0, int kbeg, int kend,
                                         f32x4 (&acc)[4][4]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  char* As[2] = {smem, smem + TILE_BYTES};
  char* Bs[2] = {smem + 2 * TILE_BYTES, smem + 3 * TILE_BYTES};
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  stage<AKC>(sa, As[0], bm0, kbeg, wave, lane);
  stage<BKC>(sb, Bs[0], bn0, kbeg, wave, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) {
      stage<AKC>(sa, As[cur ^ 1], bm0, kbeg + (kt + 1) * BK, wave, lane);
      stage<BKC>(sb, Bs[cur ^ 1], bn0, kbeg + (kt + 1) * BK, wave, lane);
    }
    const char* At = As[cur];
    const char* Bt = Bs[cur];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      v8bf a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag<AKC>(At, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = frag<BKC>(Bt, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

}  // namespace gemm
}  // namespace dtg
