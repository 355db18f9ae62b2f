// Standalone GEMM lab (not part of the package): C[M,N] = A[M,K] * B[N,K]^T, bf16 in, bf16 out,
// for iterating on main-loop schedules without rebuilding the extension.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/include tools/gemm_lab/lab.hip -o tools/gemm_lab/lab
//   tools/gemm_lab/lab M N K [iters]
// Variants are timed interleaved in one process (cdna_hip_programming.md §5.4 rule 24) on uniform
// random [-1, 1) operands, and checked against an fp32 reference GEMM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
#include "dtg/common.h"
#include "dtg/mfma_gemm.cuh"

using namespace dtg;
using namespace dtg::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// ---------------------------------------------------------------------------------------------
// v1: 256x256 tile, 4 waves (2x2), each wave 128x128 = acc[8][8] of 16x16 (256 registers), one wave
// per SIMD.  BK = 64, 2 LDS stages (128 KB), one barrier per K-tile placed between the two 32-deep
// k-steps: the ks1 fragments are read under the ks0 MFMAs, the next tile's ks0 fragments under the
// ks1 MFMAs, and the DMA of tile t+2 is issued right after the barrier (1.5 tiles of flight).
namespace v1 {
constexpr int BM = 256, NW = 4, NTH = 256;
constexpr int A_BYTES = BM * 64 * 2;             // A operand, one stage: 32 KB

template <int JN, class SA, class SB>
__device__ __forceinline__ void stage_tile(const SA& sa, const SB& sb, lds_char* buf, int bm0, int bn0, int k0, int wave,
                                           int lane) {
  stage_kc<BM, SA, NW>(sa, buf, bm0, k0, wave, lane);
  stage_kc<32 * JN, SB, NW>(sb, buf + A_BYTES, bn0, k0, wave, lane);
}

template <int JN>
__device__ __forceinline__ void read_frags(const lds_char* buf, int wm, int wn, int ks, int lane, v8bf (&a)[8],
                                           v8bf (&b)[JN]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = frag_kc(buf, wm * 128 + i * 16, ks, lane);
#pragma unroll
  for (int j = 0; j < JN; ++j) b[j] = frag_kc(buf + A_BYTES, wn * 16 * JN + j * 16, ks, lane);
}

template <int JN>
__device__ __forceinline__ void mfma_block(const v8bf (&a)[8], const v8bf (&b)[JN], f32x4 (&acc)[8][JN]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

template <int SCHED, int JN = 8>
__global__ void __launch_bounds__(NTH, 1) kern(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                               bf16_t* __restrict__ C, int M, int N, int K) {
  constexpr int BN = 32 * JN, STAGE = A_BYTES + BN * 64 * 2, LDS = 2 * STAGE;
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BN;
  DenseKC<false> sa{A, K, M, K};
  DenseKC<false> sb{B, K, N, K};
  const int nk = K / 64;
  f32x4 acc[8][JN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8bf a0[8], b0[JN], a1[8], b1[JN];
  constexpr int LPT = 8 + JN;  // LDS-DMA instructions per wave per K-tile (A: 256/32, B: 32*JN/32)
  // prologue: tiles 0 and 1 in flight, tile 0 visible, ks0 fragments of tile 0 in registers
  stage_tile<JN>(sa, sb, smem, bm0, bn0, 0, wave, lane);
  if (nk > 1) stage_tile<JN>(sa, sb, smem + STAGE, bm0, bn0, 64, wave, lane);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(smem, wm, wn, 0, lane, a0, b0);
  for (int kt = 0; kt < nk; ++kt) {
    lds_char* cur = smem + (kt & 1) * STAGE;
    lds_char* nxt = smem + ((kt + 1) & 1) * STAGE;
    // first half: ks0 MFMAs under the ks1 reads of this tile
    read_frags(cur, wm, wn, 1, lane, a1, b1);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);  // reads issued ahead of the MFMAs
    mfma_block(a0, b0, acc);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      }
    }
    // every ds_read of this tile retired; tile kt+1's DMA (this wave's part) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile kt+1 visible to all; nobody reads buffer (kt & 1) any more
    if (kt + 2 < nk) stage_tile<JN>(sa, sb, cur, bm0, bn0, (kt + 2) * 64, wave, lane);
    read_frags(nxt, wm, wn, 0, lane, a0, b0);  // (past the last tile: harmless reads of stale LDS)
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    mfma_block(a1, b1, acc);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      }
    }
  }
  // epilogue: bf16 through LDS, one 32 KB [128][128] region per wave, 16-B row stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + (lane >> 4) * 4 + r, col = j * 16 + (lane & 15);
        // 16-B chunk XOR (row & 15) keeps the column writes spread over the banks
        const int off = row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 2 * JN; c += 64) {
    const int row = c / (2 * JN), ch = c % (2 * JN);
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 256 + ((ch ^ (row & 15)) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 16 * JN + ch * 8) = v;
  }
}
}  // namespace v1


// ---------------------------------------------------------------------------------------------
// v2: 256x256 tile, 4 waves (2x2), each wave 128x128 as 4x4 v_mfma_f32_32x32x16_bf16 tiles whose 256
// accumulator registers are pinned in AGPRs by inline asm ("+a": the allocator never rotates them), BK = 64
// (4 k-steps of 16), 2 LDS stages, one barrier per K-tile before its last k-step.  Fragments for k-step
// kk+1 are read under kk's 16 MFMAs (register double buffer); the DMA of tile kt+2 is issued one piece per
// MFMA gap in tile kt's last k-step.  LDS rows are 128 B (64 k) with chunk XOR ((row >> 1) & 7): the 16
// lanes of a ds_read_b128 group (16 rows, one chunk) then hit 16 distinct 16-B slots.
namespace v2 {
constexpr int BM = 256, NTH = 256, TILE = BM * 64 * 2, STAGE = 2 * TILE, LDS = 2 * STAGE;

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

// piece i (0..7) of a [256][64] KC tile for this wave: rows (wave * 8 + i) * 8 + [0, 8)
__device__ __forceinline__ void stage_piece(const bf16_t* src, long long ld, lds_char* dst, int row0, int k0, int wave,
                                            int lane, int i) {
  const int r0 = (wave * 8 + i) * 8, r = r0 + (lane >> 3);
  const int c = (lane & 7) ^ swz(r);
  __builtin_amdgcn_global_load_lds((const void*)(src + (long long)(row0 + r) * ld + k0 + c * 8),
                                   (lds_void*)(dst + r0 * 128), 16, 0, 0);
}

// 32x32x16 operand fragment: lane l holds X[r0 + (l & 31)][16 kk + 8 (l >> 5) + j], j < 8
__device__ __forceinline__ v8bf frag32(const lds_char* t, int r0, int kk, int lane) {
  const int r = r0 + (lane & 31), c = 2 * kk + (lane >> 5);
  return *reinterpret_cast<const lds_v8bf*>(t + r * 128 + ((c ^ swz(r)) << 4));
}

#define V2_MFMA(ACC, A_, B_) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(ACC) : "v"(A_), "v"(B_))

// ABL (timing ablation, wrong results): 1 = no DMA after the prologue
template <int ABL>
__global__ void __launch_bounds__(NTH, 1) kern(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                               bf16_t* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BM;
  const int nk = K / 64;
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  v8bf fa[2][4], fb[2][4];
  auto stage_all = [&](lds_char* buf, int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) stage_piece(A, K, buf, bm0, k0, wave, lane, i);
#pragma unroll
    for (int i = 0; i < 8; ++i) stage_piece(B, K, buf + TILE, bn0, k0, wave, lane, i);
  };
  auto load = [&](const lds_char* buf, int kk, v8bf (&a)[4], v8bf (&b)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag32(buf, wm * 128 + i * 32, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag32(buf + TILE, wn * 128 + j * 32, kk, lane);
  };
  stage_all(smem, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (nk > 1) stage_all(smem + STAGE, 64);
  load(smem, 0, fa[0], fb[0]);
  for (int kt = 0; kt < nk; ++kt) {
    lds_char* cur = smem + (kt & 1) * STAGE;
    lds_char* nxt = smem + ((kt + 1) & 1) * STAGE;
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      load(cur, kk + 1, fa[(kk + 1) & 1], fb[(kk + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) V2_MFMA(acc[i][j], fa[kk & 1][i], fb[kk & 1][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // k-step 3: tile kt+1 must be visible and every read of `cur` retired before its DMA
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + 1 < nk) load(nxt, 0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
    const bool dma = ABL != 1 && kt + 2 < nk;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        V2_MFMA(acc[i][j], fa[1][i], fb[1][j]);
        const int p = i * 4 + j;  // one LDS-DMA piece per MFMA gap: A pieces 0-7, B pieces 8-15
        if (dma) {
          if (p < 8) stage_piece(A, K, cur, bm0, (kt + 2) * 64, wave, lane, p);
          else stage_piece(B, K, cur + TILE, bn0, (kt + 2) * 64, wave, lane, p - 8);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  // epilogue: bf16 through LDS, one 32 KB [128][128] region per wave, 16-B row stores
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * 32768;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i * 32 + (r >> 2) * 8 + (lane >> 5) * 4 + (r & 3), col = j * 32 + (lane & 31);
        const int off = row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 16; c += 64) {
    const int row = c / 16, ch = c % 16;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 256 + ((ch ^ (row & 15)) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 128 + ch * 8) = v;
  }
}
}  // namespace v2

// ---------------------------------------------------------------------------------------------
// v3: v2's 4-wave 256x256 tile with AGPR-pinned 32x32x16 accumulators, but BK = 32 stages in a 4-deep LDS ring
// (4 x 32 KB): the DMA of stage s+3 is issued during stage s, one 1-KB piece per 4 MFMAs over both k-steps,
// instead of 16 pieces in one k-step; one barrier per stage.  LDS rows are 64 B (32 k): chunk XOR ((row >> 2) & 3).
namespace v3 {
constexpr int BM = 256, NTH = 256, OP = BM * 32 * 2, STAGE = 2 * OP, NST = 4, LDS = NST * STAGE;

__device__ __forceinline__ int swz(int r) { return (r >> 2) & 3; }

// piece i (0..3) of a [256][32] KC operand stage for this wave: rows (wave * 4 + i) * 16 + [0, 16)
__device__ __forceinline__ void piece(const bf16_t* src, long long ld, lds_char* dst, int row0, int k0, int wave,
                                      int lane, int i) {
  const int r0 = (wave * 4 + i) * 16, r = r0 + (lane >> 2);
  const int c = (lane & 3) ^ swz(r);
  __builtin_amdgcn_global_load_lds((const void*)(src + (long long)(row0 + r) * ld + k0 + c * 8),
                                   (lds_void*)(dst + r0 * 64), 16, 0, 0);
}

__device__ __forceinline__ v8bf frag(const lds_char* t, int r0, int kk, int lane) {
  const int r = r0 + (lane & 31), c = 2 * kk + (lane >> 5);
  return *reinterpret_cast<const lds_v8bf*>(t + r * 64 + ((c ^ swz(r)) << 4));
}

__global__ void __launch_bounds__(NTH, 1) kern(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                               bf16_t* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BM;
  const int ns = K / 32;  // >= 3 (host)
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  v8bf fa[2][4], fb[2][4];
  auto buf = [&](int st) { return smem + (st & (NST - 1)) * STAGE; };
  // piece p (0..7) of stage st: A pieces 0-3, B pieces 4-7 (past the last stage: the last stage again, never read,
  // so every stage issues exactly 8 pieces and the counted waits stay uniform)
  auto dma = [&](int st, int p) {
    const int k0 = (st < ns ? st : ns - 1) * 32;
    lds_char* b = buf(st);
    if (p < 4) piece(A, K, b, bm0, k0, wave, lane, p);
    else piece(B, K, b + OP, bn0, k0, wave, lane, p - 4);
  };
  auto load = [&](int st, int kk, v8bf (&a)[4], v8bf (&b)[4]) {
    const lds_char* t = buf(st);
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag(t, wm * 128 + i * 32, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag(t + OP, wn * 128 + j * 32, kk, lane);
  };
#pragma unroll
  for (int st = 0; st < 3; ++st)
#pragma unroll
    for (int p = 0; p < 8; ++p) dma(st, p);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // stage 0 landed (stages 1, 2 in flight)
  __builtin_amdgcn_s_barrier();
  load(0, 0, fa[0], fb[0]);
  for (int s = 0; s < ns; ++s) {
    // k-step 0: first MFMA, then this stage's k-step-1 fragments, then the rest with DMA(s+3) pieces 0-3
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      V2_MFMA(acc[q >> 2][q & 3], fa[0][q >> 2], fb[0][q & 3]);
      __builtin_amdgcn_sched_barrier(0);
      if (q == 0) {
        load(s, 1, fa[1], fb[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
      if ((q & 3) == 3) {
        dma(s + 3, q >> 2);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // stage s+1 landed (younger: DMA(s+2) and the 4 pieces of DMA(s+3) just issued) and every read of stage s
    // retired, then visible to all
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    load(s + 1, 0, fa[0], fb[0]);  // (past the last stage: stale reads, unused)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      V2_MFMA(acc[q >> 2][q & 3], fa[1][q >> 2], fb[1][q & 3]);
      __builtin_amdgcn_sched_barrier(0);
      if ((q & 3) == 3) {
        dma(s + 3, 4 + (q >> 2));
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * 32768;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i * 32 + (r >> 2) * 8 + (lane >> 5) * 4 + (r & 3), col = j * 32 + (lane & 31);
        const int off = row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 16; c += 64) {
    const int row = c / 16, ch = c % 16;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 256 + ((ch ^ (row & 15)) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 128 + ch * 8) = v;
  }
}
}  // namespace v3

// ---------------------------------------------------------------------------------------------
// v4: v2's tile and AGPR-pinned accumulators with the operands staged through VGPRs instead of LDS-DMA:
// tile kt+1 is fetched by global_load_dwordx4 (16 per lane, 64 VGPRs) under k-steps 0-1 of tile kt and written
// to the other LDS buffer by ds_write_b128 under k-step 2; two barriers per tile (buffer free / buffer written).
namespace v4 {
constexpr int BM = 256, NTH = 256, TILE = BM * 64 * 2, STAGE = 2 * TILE, LDS = 2 * STAGE;
using v2::swz;
using v2::frag32;

__global__ void __launch_bounds__(NTH, 1) kern(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                               bf16_t* __restrict__ C, int M, int N, int K) {
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BM;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BM;
  const int nk = K / 64;
  f32x16 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  v8bf fa[2][4], fb[2][4];
  u32x4v g[16];  // tile kt+1 in flight: A chunks 0-7, B chunks 8-15
  // chunk i of this thread: operand rows (i & 7) * 32 + tid / 8, 16-B chunk (tid & 7) of the 128-B row
  auto gload = [&](int kt) {
    const int k0 = kt * 64;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = (i & 7) * 32 + (tid >> 3);
      const bf16_t* src = i < 8 ? A + (long long)(bm0 + r) * K : B + (long long)(bn0 + r) * K;
      g[i] = *reinterpret_cast<const u32x4v*>(src + k0 + (tid & 7) * 8);
    }
  };
  auto gstore = [&](lds_char* buf, int i) {
    const int r = (i & 7) * 32 + (tid >> 3);
    const int c = (tid & 7) ^ swz(r);
    *reinterpret_cast<__attribute__((address_space(3))) u32x4v*>(buf + (i < 8 ? 0 : TILE) + r * 128 + c * 16) = g[i];
  };
  auto load = [&](const lds_char* buf, int kk, v8bf (&a)[4], v8bf (&b)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag32(buf, wm * 128 + i * 32, kk, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag32(buf + TILE, wn * 128 + j * 32, kk, lane);
  };
  gload(0);
#pragma unroll
  for (int i = 0; i < 16; ++i) gstore(smem, i);
  __syncthreads();
  load(smem, 0, fa[0], fb[0]);
  for (int kt = 0; kt < nk; ++kt) {
    lds_char* cur = smem + (kt & 1) * STAGE;
    lds_char* nxt = smem + ((kt + 1) & 1) * STAGE;
    const bool more = kt + 1 < nk;
    if (more) gload(kt + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 3; ++kk) {
      load(cur, kk + 1, fa[(kk + 1) & 1], fb[(kk + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        V2_MFMA(acc[q >> 2][q & 3], fa[kk & 1][q >> 2], fb[kk & 1][q & 3]);
        if (kk == 2 && more) gstore(nxt, q);  // nxt was last read in tile kt-1, before this tile's first barrier
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile kt+1 written by everyone; every read of `cur` retired
    if (more) load(nxt, 0, fa[0], fb[0]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 16; ++q) V2_MFMA(acc[q >> 2][q & 3], fa[1][q >> 2], fb[1][q & 3]);
    __builtin_amdgcn_sched_barrier(0);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * 32768;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = i * 32 + (r >> 2) * 8 + (lane >> 5) * 4 + (r & 3), col = j * 32 + (lane & 31);
        const int off = row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 16; c += 64) {
    const int row = c / 16, ch = c % 16;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 256 + ((ch ^ (row & 15)) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 128 + ch * 8) = v;
  }
}
}  // namespace v4

// ---------------------------------------------------------------------------------------------
// reference: fp32 accumulate, one thread per output
__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(long long)m * K + k]) * bf2f(B[(long long)n * K + k]);
  C[(long long)m * N + n] = s;
}

static uint16_t f2bf_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f_host(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

typedef void (*launch_fn)(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, hipStream_t);

template <int S, int JN = 8>
static void launch_v1(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t st) {
  if (N % (32 * JN)) return;
  hipLaunchKernelGGL((v1::kern<S, JN>), dim3((M / 256) * (N / (32 * JN))), dim3(256), 0, st, A, B, C, M, N, K);
}

template <int ABL>
static void launch_v2(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL(v2::kern<ABL>, dim3((M / 256) * (N / 256)), dim3(256), 0, st, A, B, C, M, N, K);
}

static void launch_v3(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL(v3::kern, dim3((M / 256) * (N / 256)), dim3(256), 0, st, A, B, C, M, N, K);
}

static void launch_v4(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t st) {
  hipLaunchKernelGGL(v4::kern, dim3((M / 256) * (N / 256)), dim3(256), 0, st, A, B, C, M, N, K);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 4096;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  if (M % 256 || N % 256 || K % 64) {
    printf("shape must be multiples of 256 x 256 x 64\n");
    return 1;
  }
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
  for (auto& v : ha) v = f2bf_host(rnd());
  for (auto& v : hb) v = f2bf_host(rnd());
  bf16_t *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, ha.size() * 2));
  CK(hipMalloc(&B, hb.size() * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&R, (size_t)M * N * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, A, B, R, M, N, K);
  CK(hipDeviceSynchronize());
  std::vector<float> hr((size_t)M * N);
  CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
  struct V { const char* name; launch_fn f; std::vector<float> ms; };
  std::vector<V> vs = {{"v1 4w 128x128/wave", launch_v1<0>, {}}, {"v2 32x32x16 asm-AGPR acc", launch_v2<0>, {}},
                       {"v4 VGPR-staged operands", launch_v4, {}}};
  std::vector<uint16_t> hc((size_t)M * N);
  for (auto& v : vs) {  // correctness
    CK(hipMemset(C, 0, (size_t)M * N * 2));
    v.f(A, B, C, M, N, K, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (size_t i = 0; i < hc.size(); ++i) {
      maxerr = std::max(maxerr, (double)fabsf(bf2f_host(hc[i]) - hr[i]));
      maxref = std::max(maxref, (double)fabsf(hr[i]));
    }
    printf("%-28s max|err| %.4g (max|ref| %.4g)%s\n", v.name, maxerr, maxref, maxerr > 1e-2 * maxref ? "  WRONG" : "");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 5; ++round)
    for (auto& v : vs) {
      for (int i = 0; i < 3; ++i) v.f(A, B, C, M, N, K, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) v.f(A, B, C, M, N, K, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / iters);
    }
  const double flop = 2.0 * M * N * K;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    printf("%-28s %dx%dx%d  median %.1f us  min %.1f us  %.0f TF/s\n", v.name, M, N, K, v.ms[2] * 1e3, v.ms[0] * 1e3,
           flop / (v.ms[2] * 1e-3) / 1e12);
  }
  return 0;
}
