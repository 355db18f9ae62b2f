// GEMM lab v5 (tools-only extension dtg._lab, not linked into _C): the main-loop schedule read from hipBLASLt's
// gfx950 kernel for BERT's forward shapes (Cijk_Alik_Bljk_BBS_BH_..._MT192x256x64_MI16x16x1_..._MIWT6_8_..._PGR2_
// PLR1_..._WG32_8_1 in TensileLibrary_BB_BB_HA_Bias_SAV_UA_Type_BB_HPA_Contraction_l_Alik_Bljk_Cijk_Dijk_gfx950.co,
// disassembled with llvm-objdump; profiles/r05_gemm_schedule/README.md has the annotated loop), re-expressed in
// HIP -- not transcribed:
//
//   * 4 waves (2 x 2), one per SIMD, each owning a 128 x 96 output block = 8 x 6 tiles of
//     v_mfma_f32_16x16x32_bf16 (48 accumulators, 192 registers): 14 fragment reads (ds_read_b128) per 48 MFMAs,
//     against 8 per 16 in the 64 x 64-per-wave production tiles;
//   * operands staged through VGPRs: 14 x 16 B global loads per thread per 64-deep K-tile, each written to LDS
//     (ds_write_b128) one K-tile later and its register immediately reloaded with the K-tile after that, so one
//     whole K-tile of loads is always in flight and each write waits only for the OLDEST load (vmcnt(13));
//   * LDS double-buffered (2 x 56 KB), ONE barrier per K-tile;
//   * the next k-step's fragments are read under the current k-step's MFMAs (1 read per MFMA), the global
//     loads / LDS writes spread one pair per 4 MFMAs over the rest of the tile, and the next K-tile's first
//     fragments read under the last 14 MFMAs, after the barrier.
//
// C[M, N] = A[M, K] * B[N, K]^T, bf16 operands (K-contiguous), fp32 accumulation, bf16 out.  Tile 256 (M) x 192 (N)
// x 64; M % 256 == 0, N % 192 == 0, K % 64 == 0 (checked on the host).
#include "dtg/common.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"

#include <type_traits>

namespace dtg {
namespace lab {
using namespace gemm;

namespace {

constexpr int BM = 256, BN = 192, TI = 8, TJ = 6;
constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;  // 32 KB + 24 KB
constexpr int NLD = BM / 32 + BN / 32;                                               // 14 loads / thread / K-tile

typedef __attribute__((address_space(3))) u32x4v lds_u32x4v;

// accumulators pinned in AGPRs ("+a"): with the builtin, the allocator spilled and rotated them through the
// unified register file (172 v_accvgpr_mov + 80 write + 80 read per K-tile at 512 registers)
__device__ __forceinline__ void mfma(f32x4& acc, const v8bf& a, const v8bf& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// SCHED 0: plain program order (the compiler schedules); 1: the interleave described above
template <int SCHED>
__global__ void __launch_bounds__(256, 1) g5_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                    bf16_t* __restrict__ C, int M, int N, int K, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BN;
  const int nk = K / 64;
  // this thread's chunks: operand row i * 32 + tid / 8, 16-B chunk tid % 8 of the 128-B K-tile row
  const bf16_t* ga = A + (long long)(bm0 + (tid >> 3)) * K + (tid & 7) * 8;
  const bf16_t* gb = B + (long long)(bn0 + (tid >> 3)) * K + (tid & 7) * 8;
  const long long rs = 32LL * K;  // 32 rows
  // LDS image [rows][64 k], chunk XOR (row & 7) (frag_kc's layout); row & 7 = (tid >> 3) & 7 for every i
  const int wbase = (tid >> 3) * 128 + (((tid & 7) ^ ((tid >> 3) & 7)) << 4);
  u32x4v g[NLD];
  auto gload = [&](int i, int k0) {
    const bf16_t* p = i < 8 ? ga + i * rs + k0 : gb + (i - 8) * rs + k0;
    g[i] = *reinterpret_cast<const u32x4v*>(p);
  };
  auto gstore = [&](lds_char* buf, int i) {
    lds_char* p = i < 8 ? buf + i * 4096 + wbase : buf + A_BYTES + (i - 8) * 4096 + wbase;
    *reinterpret_cast<lds_u32x4v*>(p) = g[i];
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8bf fa[2][TI], fb[2][TJ];
  auto rd = [&](const lds_char* buf, int ks, int q) {  // fragment read q of k-step ks (q < 8: A, else B)
    if (q < TI) fa[ks][q] = frag_kc(buf, wm * 128 + q * 16, ks, lane);
    else fb[ks][q - TI] = frag_kc(buf + A_BYTES, wn * 96 + (q - TI) * 16, ks, lane);
  };

  // prologue: K-tile 0 in LDS buffer 0, K-tile 1 in registers, k-step 0 fragments of K-tile 0 read
#pragma unroll
  for (int i = 0; i < NLD; ++i) gload(i, 0);
#pragma unroll
  for (int i = 0; i < NLD; ++i) gstore(smem, i);
  if (nk > 1) {
#pragma unroll
    for (int i = 0; i < NLD; ++i) gload(i, 64);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);  // no LDS access moves across the raw barrier
#pragma unroll
  for (int q = 0; q < TI + TJ; ++q) rd(smem, 0, q);

  // one K-tile; MORE: a next K-tile exists (its registers go to LDS), MORE2: and the one after (reload them)
  auto iter = [&](int kt, auto more_c, auto more2_c) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_char* cur = smem + (kt & 1) * STAGE;
    lds_char* nxt = smem + ((kt + 1) & 1) * STAGE;
    const int k2 = (kt + 2) * 64;
    if constexpr (SCHED == 0) {
#pragma unroll
      for (int q = 0; q < TI + TJ; ++q) rd(cur, 1, q);
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma(acc[i][j], fa[0][i], fb[0][j]);
      if constexpr (more) {
#pragma unroll
        for (int i = 0; i < NLD; ++i) {
          gstore(nxt, i);
          if constexpr (more2) gload(i, k2);
        }
      }
#pragma unroll
      for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) mfma(acc[i][j], fa[1][i], fb[1][j]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);  // no LDS access moves across the raw barrier
      if constexpr (more) {
#pragma unroll
        for (int q = 0; q < TI + TJ; ++q) rd(nxt, 0, q);
      }
    } else {
      // MFMA stream of this K-tile: m = 0..95, k-step m / 48, tile (i, j) = ((m % 48) / 6, m % 6)
      // slots: m < 14: + fragment read q = m of k-step 1; 14 <= m < 70, every 4th: + (LDS write, global load) pair
      // p = (m - 14) / 4; m = 82: barrier; m >= 82: + fragment read q = m - 82 of the next K-tile's k-step 0
#pragma unroll
      for (int m = 0; m < 96; ++m) {
        const int ks = m / 48, i = (m % 48) / TJ, j = m % TJ;
        if (m == 82) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
        }
        mfma(acc[i][j], fa[ks][i], fb[ks][j]);
        if (m < 14) {
          rd(cur, 1, m);
        } else if (m < 70 && (m - 14) % 4 == 0) {
          const int p = (m - 14) / 4;
          if constexpr (more) {
            gstore(nxt, p);
            if constexpr (more2) gload(p, k2);
          }
        } else if (m >= 82) {
          if constexpr (more) rd(nxt, 0, m - 82);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int kt = 0;
  for (; kt + 2 < nk; ++kt) iter(kt, T_(), T_());  // branch-free steady state
  if (kt + 1 < nk) iter(kt++, T_(), F_());
  iter(kt, F_(), F_());

  // epilogue: each wave stages its 128 x 96 block as bf16 in LDS (24 KB per wave, swizzled 16-B chunks), then
  // writes it with 16-B stores
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * (128 * 96 * 2);
  const int q16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + g4 * 4 + r, col = j * 16 + q16;  // 12 chunks of 8 per 192-B row
        const int off = row * 192 + ((((col >> 3) + row) % 12) << 4) + (col & 7) * 2;  // chunks rotated by row
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 12; c += 64) {
    const int row = c / 12, ch = c % 12;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 192 + (((ch + row) % 12) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 96 + ch * 8) = v;
  }
}

// ---- v5p: persistent form with the K-stream continuous across tiles and a register epilogue -------------------
// Each workgroup walks tiles t = b, b + G, ... (G = one workgroup per CU); its (tile, K-tile) pairs form ONE stream,
// so the VGPR-staged loads of a tile's first two K-tiles are issued during the previous tile's last K-tiles and
// the epilogue runs while they are in flight (v5 paid a full pipeline fill + drain per tile: 0.92 vs hipBLASLt's
// 1.14 PF/s at K = 768).  The LDS is busy with the next tile then, so the epilogue stores straight from registers:
// the MFMA operands are swapped (B fragment as src A: D' = B A^T), and B's rows are written to LDS permuted, so
// that a lane's accumulators of an (m-tile, n-tile pair) are 8 consecutive output columns of one row -> one 16-B
// store through dtg's generic epilogue (epi_store8: alpha/beta, bias, activation, aux).
// LDS row rho of a 32-row B block holds n_local = 8 ((rho & 15) >> 2) + 4 (rho >> 4) + (rho & 3): fragment row i of
// n-tile j = 2 jp + jodd (rows 16 jodd + i of block jp) is output column 8 (i >> 2) + 4 jodd + (i & 3) of the block,
// so lane (q, g)'s D'[4 g + r][q] of tiles 2 jp, 2 jp + 1 are columns 32 jp + 8 g + [0, 8) of row q.
// EPI 0: bf16 C = acc; 1: + bias; 2: + bias, GELU, aux = GELU'(pre) (BERT FFN1 forward); 3: dtg's generic epilogue
template <int EPI>
__device__ __forceinline__ void epi5(const Epi& e, int N, int m, int n, float (&v)[8]) {
  if constexpr (EPI == 3) {
    epi_store8(e, N, m, n, v);
  } else {
    const long long off = (long long)m * e.ldc + n;
    if constexpr (EPI >= 1) {
      float b[8];
      load8_f32(e.bias + n, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += b[k];
    }
    if constexpr (EPI == 2) {
      float t[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        t[k] = act_grad(v[k], 2);
        v[k] = v[k] * gelu_sig(v[k]);
      }
      store8_bf16((bf16_t*)e.aux + off, t);
    }
    store8_bf16((bf16_t*)e.C + off, v);
  }
}

template <int EPI>
__global__ void __launch_bounds__(256, 1) g5p_kernel(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                                     Epi e, int M, int N, int K, int tiles_n, int ntiles) {
  __shared__ __attribute__((aligned(16))) char smem_raw[2 * STAGE];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int G = gridDim.x, b0 = blockIdx.x;
  const int my = b0 < ntiles ? (ntiles - b0 + G - 1) / G : 0;
  if (my == 0) return;
  const int nk = K / 64;
  const int S = my * nk;  // this workgroup's K-stream
  const long long rs = 32LL * K;
  const int r8 = tid >> 3, c8 = tid & 7;
  const int wa = r8 * 128 + ((c8 ^ (r8 & 7)) << 4);  // A image: row r8 (+32 i), chunk XOR row
  const int rho = 16 * ((r8 >> 2) & 1) + 4 * (r8 >> 3) + (r8 & 3);  // B image row of n_local = r8
  const int wb = rho * 128 + ((c8 ^ (rho & 7)) << 4);
  auto tile_of = [&](int i, int& bm0, int& bn0) __attribute__((always_inline)) {
    const int t = b0 + i * G;
    bm0 = (t / tiles_n) * BM;
    bn0 = (t % tiles_n) * BN;
  };
  u32x4v g[NLD];
  // buffer loads: one per-thread VGPR offset for every chunk of both operands, the tile / K-tile / row-block part
  // in the scalar offset (the 14 loads of a K-tile need no per-load 64-bit address arithmetic)
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)((long long)M * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, (int)((long long)N * K * 2), 0x00020000);
  const int voff = (r8 * K + c8 * 8) * 2;
  int sa0 = 0, sb0 = 0;
  auto gaddr = [&](int s) __attribute__((always_inline)) {  // scalar bases of stream K-tile s
    int bm0, bn0;
    tile_of(s / nk, bm0, bn0);
    const int k0 = (s % nk) * 64;
    sa0 = __builtin_amdgcn_readfirstlane((bm0 * K + k0) * 2);
    sb0 = __builtin_amdgcn_readfirstlane((bn0 * K + k0) * 2);
  };
  auto gload = [&](int i) __attribute__((always_inline)) {
    const int so = i < 8 ? sa0 + i * (int)(rs * 2) : sb0 + (i - 8) * (int)(rs * 2);
    g[i] = __builtin_bit_cast(u32x4v, __builtin_amdgcn_raw_buffer_load_b128(i < 8 ? rsa : rsb, voff, so, 0));
  };
  auto gstore = [&](lds_char* buf, int i) __attribute__((always_inline)) {
    lds_char* p = i < 8 ? buf + i * 4096 + wa : buf + A_BYTES + (i - 8) * 4096 + wb;
    *reinterpret_cast<lds_u32x4v*>(p) = g[i];
  };
  f32x4 acc[TI][TJ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8bf fa[2][TI], fb[2][TJ];
  auto rd = [&](const lds_char* buf, int ks, int q) __attribute__((always_inline)) {
    if (q < TI) fa[ks][q] = frag_kc(buf, wm * 128 + q * 16, ks, lane);
    else fb[ks][q - TI] = frag_kc(buf + A_BYTES, wn * 96 + (q - TI) * 16, ks, lane);
  };
  // Epilogue of tile i_tile, called right after its last MFMA, with `freebuf` = the LDS buffer that K-tile held
  // (every wave finished reading it before the K-tile's barrier; the next write into it is the next iteration's).
  // The accumulators stay pinned in AGPRs: each lane bounces its own f32x4s through LDS (ds_write_b128 takes AGPR
  // data; the round trip needs no cross-lane exchange and no barrier) instead of the compiler reading them out,
  // which made it rotate and spill the accumulator file; they are re-zeroed by MFMAs with a zero C operand.
  const v8bf fzero = {};
  auto epilogue = [&](int i_tile, lds_char* freebuf) __attribute__((always_inline)) {
    int bm0, bn0;
    tile_of(i_tile, bm0, bn0);
    const int q = lane & 15, g4 = lane >> 4;
    lds_char* slot = freebuf + wave * (TJ * 1024) + lane * 16;  // TJ x 1 KB per wave (one m-tile at a time)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // last MFMA results readable by DS
#pragma unroll
    for (int i = 0; i < TI; ++i) {
#pragma unroll
      for (int j = 0; j < TJ; ++j)
        asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"((unsigned)(uintptr_t)slot), "a"(acc[i][j]), "i"(j * 1024)
                     : "memory");
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int jp = 0; jp < TJ / 2; ++jp) {
        const f32x4 lo = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(slot + 2 * jp * 1024);
        const f32x4 hi = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(slot + (2 * jp + 1) * 1024);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        const int m = bm0 + wm * 128 + i * 16 + q, n = bn0 + wn * 96 + jp * 32 + g4 * 8;
        epi5<EPI>(e, N, m, n, v);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot reads done before the next m-tile's writes
    }
    // (the compiler materialises fzero with VALU moves right before this asm, and it does not know the asm is an
    // MFMA: without these wait states the first MFMA read the register's previous contents -- a fragment -- and
    // left acc[0][0] of every later tile with garbage, tools/gemm5p_debug.py)
    asm volatile("s_nop 4" ::"v"(fzero));
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
      for (int j = 0; j < TJ; ++j) asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "+a"(acc[i][j]) : "v"(fzero));
    __builtin_amdgcn_s_barrier();  // every wave's slot reads are done before the next K-tile is written over them
    __builtin_amdgcn_sched_barrier(0);
  };

  // prologue: stream K-tile 0 in LDS buffer 0, K-tile 1 in registers, k-step 0 fragments read
  gaddr(0);
#pragma unroll
  for (int i = 0; i < NLD; ++i) gload(i);
#pragma unroll
  for (int i = 0; i < NLD; ++i) gstore(smem, i);
  if (S > 1) {
    gaddr(1);
#pragma unroll
    for (int i = 0; i < NLD; ++i) gload(i);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);  // no LDS access moves across the raw barrier
#pragma unroll
  for (int q = 0; q < TI + TJ; ++q) rd(smem, 0, q);

  auto iter = [&](int s, auto more_c, auto more2_c) __attribute__((always_inline)) {
    constexpr bool more = decltype(more_c)::value, more2 = decltype(more2_c)::value;
    const lds_char* cur = smem + (s & 1) * STAGE;
    lds_char* nxt = smem + ((s + 1) & 1) * STAGE;
    if constexpr (more2) gaddr(s + 2);
#pragma unroll
    for (int m = 0; m < 96; ++m) {
      const int ks = m / 48, i = (m % 48) / TJ, j = m % TJ;
      if (m == 82) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      mfma(acc[i][j], fb[ks][j], fa[ks][i]);  // swapped: D' = B A^T
      if (m < 14) {
        rd(cur, 1, m);
      } else if (m < 70 && (m - 14) % 4 == 0) {
        const int p = (m - 14) / 4;
        if constexpr (more) {
          gstore(nxt, p);
          if constexpr (more2) gload(p);
        }
      } else if (m >= 82) {
        if constexpr (more) rd(nxt, 0, m - 82);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (s % nk == nk - 1) epilogue(s / nk, (lds_char*)cur);  // tile done: the next tile's K-tiles are in flight
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int s = 0;
  for (; s + 2 < S; ++s) iter(s, T_(), T_());
  if (s + 1 < S) iter(s++, T_(), F_());
  iter(s, F_(), F_());
}

}  // namespace

int gemm5_bf16(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int sched, hipStream_t st) {
  if (M % BM || N % BN || K % 64 || K < 64) return 0;
  const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
  if (sched == 0) g5_kernel<0><<<tiles, 256, 0, st>>>(A, B, C, M, N, K, tiles_n);
  else g5_kernel<1><<<tiles, 256, 0, st>>>(A, B, C, M, N, K, tiles_n);
  DTG_LAUNCH_CHECK();
  return 1;
}

}  // namespace lab
}  // namespace dtg

namespace dtg {
namespace lab {
// persistent v5 with dtg's generic epilogue (bias, activation, aux, alpha / beta, bf16 or fp32 out)
int gemm5p_bf16(const bf16_t* A, const bf16_t* B, void* C, int c_bf16, int M, int N, int K, const float* bias, int act,
                void* aux, int aux_mode, hipStream_t st, int grid) {
  if (M % BM || N % BN || K % 64 || K < 64) return 0;
  int dev = 0, cus = 0;
  DTG_HIP_CHECK(hipGetDevice(&dev));
  DTG_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int tiles_n = N / BN, tiles = (M / BM) * tiles_n;
  int G = tiles < cus ? tiles : cus;
  if (grid > 0 && grid < G) G = grid;  // (debug / A/B: fewer workgroups, more tiles each)
  Epi e{C, N, c_bf16, 1.f, 0.f, bias, act, aux, aux_mode};
  int epi = 3;
  if (c_bf16 && act == 0 && aux_mode == 0) epi = bias ? 1 : 0;
  else if (c_bf16 && bias && act == 2 && aux_mode == 3) epi = 2;
  if (epi == 0) g5p_kernel<0><<<G, 256, 0, st>>>(A, B, e, M, N, K, tiles_n, tiles);
  else if (epi == 1) g5p_kernel<1><<<G, 256, 0, st>>>(A, B, e, M, N, K, tiles_n, tiles);
  else if (epi == 2) g5p_kernel<2><<<G, 256, 0, st>>>(A, B, e, M, N, K, tiles_n, tiles);
  else g5p_kernel<3><<<G, 256, 0, st>>>(A, B, e, M, N, K, tiles_n, tiles);
  DTG_LAUNCH_CHECK();
  return 1;
}
}  // namespace lab
}  // namespace dtg
