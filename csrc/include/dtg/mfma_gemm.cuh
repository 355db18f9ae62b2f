// MFMA GEMM core for gfx950 (CDNA4), shared by dense GEMM and implicit-GEMM convolution.
//
//   C[M,N] (+)= A[M,K] * B[K,N]        bf16 inputs, fp32 accumulate (v_mfma_f32_16x16x32_bf16)
//
// Tiling: 256 threads = 4 waves; each wave owns a 64x64 output sub-tile = 4x4 MFMA 16x16
// accumulators (64 acc VGPRs).  Block tile BM x BN x 64 with (BM/64) x (BN/64) = 4 waves:
//   Cfg<128,128>  2x2 waves  -- general
//   Cfg<256, 64>  4x1 waves  -- skinny N (64-channel convs): A streamed once, no wasted MFMAs
// Operand tiles are staged HBM->LDS with global_load_lds_dwordx4 (LDS-DMA, 1 KiB per
// wave-instruction, no VGPR round trip).  STAGES = 2: 2-deep LDS ring, next tile's DMA in flight
// under the current tile's MFMAs, one barrier per K-step; STAGES = 1 (short K): half the LDS, so
// twice the workgroups per CU hide latency across blocks instead.
//
// All LDS accesses go through address_space(3) pointers: a generic pointer makes hipcc emit
// flat_load (counted on vmcnt AND lgkmcnt), which drains the in-flight DMA at every fragment read.
//
// Each operand is either
//   KC  ("K-contiguous")  : element (row, k) at base(row) + k          -> LDS [rows][64]  128 B rows,
//        16-B chunk XOR-swizzled by (row & 7); fragments by ds_read_b128 (conflict-free)
//   MC  ("MN-contiguous") : element (k, col) at base(k) + col          -> LDS [64][rows]  2*rows B rows,
//        16-B chunk XOR-swizzled by 2*f(k); fragments by 2x ds_read_b64_tr_b16 (hardware transpose)
// so the three training GEMMs (fwd X*W^T, dgrad dY*W, wgrad dY^T*X) all run without explicit
// transposes.  With LDS-DMA the destination is lane-linear, so the swizzle is applied to the
// per-lane SOURCE address and undone on the read (cdna_hip_programming.md §5.4 rule 21).
//
// Where an operand comes from is a policy object (`Src`) returning the global address of the
// 16-byte chunk a lane must fetch; dense strided matrices and im2col gathers (conv.hip) plug in
// here.  GUARD=false instantiations (every tile full) compute addresses with no bounds checks;
// GUARD=true ones send out-of-range chunks to a zero page.
#pragma once
#include "dtg/common.h"

namespace dtg {
namespace gemm {

typedef __attribute__((ext_vector_type(8))) __bf16 v8bf;
typedef __attribute__((ext_vector_type(4))) __bf16 v4bf;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) char lds_char;
typedef __attribute__((address_space(3))) v4bf lds_v4bf;
typedef __attribute__((address_space(3))) v8bf lds_v8bf;
typedef __attribute__((address_space(3))) float lds_float;

constexpr int BK = 64;
constexpr int NT = 256;

// BK_ = K depth of one ring stage: 64 (128-B LDS rows) or 32 (64-B rows: half the LDS per stage, so a
// deep ring still leaves room for several workgroups per CU).
// RP_ (single-stage only): register pipelining -- each K-step's operand fragments are read from LDS into
// registers up front, so the next step's LDS-DMA can be issued before this step's MFMAs (one LDS
// buffer, DMA latency overlapped with the MFMAs instead of exposed).
template <int BM_, int BN_, int STAGES_ = 2, int NW_ = 4, int BK_ = 64, bool RP_ = false>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, STAGES = STAGES_, NW = NW_, NTH = NW_ * 64, BK = BK_;
  static constexpr bool RP = RP_;
  static_assert(!RP_ || STAGES_ == 1, "register pipelining is a single-stage schedule");
  static constexpr int WM = BM / 64, WN = BN / 64;
  static_assert(WM * WN == NW, "one 64x64 sub-tile per wave");
  static_assert(STAGES >= 1 && STAGES <= 5, "ring depth");
  static_assert(BK == 64 || BK == 32, "stage depth");
  static constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  static constexpr int STAGE_BYTES = A_BYTES + B_BYTES;
  static constexpr int LDS_BYTES = STAGES * STAGE_BYTES;
  static constexpr int EPI_ROWS = 32;  // epilogue staging pass height
  static_assert(EPI_ROWS * (BN + 4) * 4 <= LDS_BYTES, "epilogue staging does not fit");
};

// 16-byte zero page in global memory for out-of-range chunks (glds needs a global source).
__device__ __attribute__((aligned(64))) static const bf16_t g_zero_page[32] = {0};

__device__ __forceinline__ const void* zero_src() { return (const void*)g_zero_page; }

// branch-free select between a real chunk address and the zero page
__device__ __forceinline__ const void* sel(bool ok, const void* p) {
  const uintptr_t a = (uintptr_t)p, z = (uintptr_t)zero_src();
  return (const void*)(ok ? a : z);
}

// swizzle of the 16-B chunk index of an MC row (CH chunks): makes the 8 rows read by one ds_read_b64_tr_b16
// half-wave (rows 8g + q, g in {0, 1}, q in 0..3) hit distinct banks.  A half-wave reads, per row, one aligned
// pair of chunks (c, c + 1) and rows of equal parity share the same 32 banks, so the swizzle's bits [2:1] must
// differ over rows {0, 2, 8, 10} (and {1, 3, 9, 11}).  For 64-row tiles (CH = 8) that takes row bits 1 and 3
// (plus row bit 0 as chunk bit 0, which also spreads the 16-B row reads of a 16-row block over all 8 chunks);
// the wider rows keep the pair-preserving form.  (The earlier CH = 8 form folded row bit 3 away: rows 0 and 8
// read the same banks, a 2-way conflict on every 64-row MC fragment read -- 57 % / 46 % of the attention forward /
// backward's LDS cycles were bank conflicts, profiles/r06_lds_swz.)
template <int CH>
__device__ __forceinline__ int mc_swz(int k) {
  if constexpr (CH == 8) return (((k >> 3) & 1) << 2) | (((k >> 1) & 1) << 1) | (k & 1);
  return ((((k & 3) | (((k >> 3) & 1) << 2)) << 1) & (CH - 1));
}

// ---- dense sources -------------------------------------------------------------------------
// KC: matrix stored [rows][ld] with k contiguous
template <bool GUARD>
struct DenseKC {
  static constexpr bool kGuard = GUARD;
  const bf16_t* p;
  long long ld;
  int rows, K;
  __device__ __forceinline__ const void* chunk(int row, int k) const {
    if constexpr (!GUARD) return p + (long long)row * ld + k;
    const int r = row < rows ? row : rows - 1;
    return sel(k < K, p + (long long)r * ld + k);
  }
};
// MC: matrix stored [K][ld] with the row/col (M or N) index contiguous
template <bool GUARD>
struct DenseMC {
  static constexpr bool kGuard = GUARD;
  const bf16_t* p;
  long long ld;
  int cols, K;
  __device__ __forceinline__ const void* chunk(int krow, int col) const {
    if constexpr (!GUARD) return p + (long long)krow * ld + col;
    const bool ok = krow < K && col < cols;
    const int kr = krow < K ? krow : K - 1;
    const int cc = col < cols ? col : 0;
    return sel(ok, p + (long long)kr * ld + cc);
  }
};

// ---- staging ---------------------------------------------------------------------------------
// KC tile: ROWS x 64 k (128 B rows, chunk XOR (row & 7)); a wave-instruction covers 8 rows; NW waves
// share the tile.  BKT = 32: ROWS x 32 k (64 B rows, 4 chunks, chunk XOR ((row >> 2) & 3): the 16 rows one
// ds_read_b128 lane group touches then hit 16 distinct 16-B slots); a wave-instruction covers 16 rows.
template <int ROWS, class Src, int NW = 4, int BKT = 64>
__device__ __forceinline__ void stage_kc(const Src& src, lds_char* lds_tile, int row0, int k0, int wave, int lane) {
  if constexpr (BKT == 64) {
    constexpr int PER_WAVE = ROWS / (8 * NW);
    static_assert(PER_WAVE >= 1, "tile too small for the wave count");
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int r0 = (wave * PER_WAVE + i) * 8;
      const int r = r0 + (lane >> 3);
      const int cl = lane & 7;           // linear chunk position in LDS
      const int c = cl ^ (r & 7);        // source chunk that belongs there
      const void* g = src.chunk(row0 + r, k0 + c * 8);
      __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_tile + r0 * 128), 16, 0, 0);
    }
  } else {
    constexpr int PER_WAVE = ROWS / (16 * NW);
    static_assert(PER_WAVE >= 1, "tile too small for the wave count");
#pragma unroll
    for (int i = 0; i < PER_WAVE; ++i) {
      const int r0 = (wave * PER_WAVE + i) * 16;
      const int r = r0 + (lane >> 2);
      const int c = (lane & 3) ^ ((r >> 2) & 3);
      const void* g = src.chunk(row0 + r, k0 + c * 8);
      __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_tile + r0 * 64), 16, 0, 0);
    }
  }
}

// MC tile: BKT k-rows x ROWS cols (2*ROWS B rows); a wave-instruction covers 512/ROWS k-rows
template <int ROWS, class Src, int NW = 4, int BKT = 64>
__device__ __forceinline__ void stage_mc(const Src& src, lds_char* lds_tile, int col0, int k0, int wave, int lane) {
  constexpr int CH = ROWS / 8;          // 16-B chunks per k-row
  constexpr int KPI = 64 / CH;          // k-rows per wave-instruction
  constexpr int PER_WAVE = BKT / KPI / NW;
  static_assert(PER_WAVE >= 1, "tile too small for the wave count");
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int kr0 = (wave * PER_WAVE + i) * KPI;
    const int kr = kr0 + lane / CH;
    const int cl = lane % CH;
    const int c = cl ^ mc_swz<CH>(kr);
    const void* g = src.chunk(k0 + kr, col0 + c * 8);
    __builtin_amdgcn_global_load_lds(g, (lds_void*)(lds_tile + kr0 * ROWS * 2), 16, 0, 0);
  }
}

// ---- fragment reads (one 16x32 operand fragment for mfma_f32_16x16x32_bf16) --------------------
// lane l holds X[r0 + (l&15)][ks*32 + 8*(l>>4) + j], j = 0..7
template <int BKT = 64>
__device__ __forceinline__ v8bf frag_kc(const lds_char* lds_tile, int r0, int ks, int lane) {
  const int r = r0 + (lane & 15);
  if constexpr (BKT == 64) {
    const int c = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const lds_v8bf*>(lds_tile + r * 128 + ((c ^ (r & 7)) << 4));
  } else {
    const int c = lane >> 4;
    return *reinterpret_cast<const lds_v8bf*>(lds_tile + r * 64 + ((c ^ ((r >> 2) & 3)) << 4));
  }
}

template <int ROWS>
__device__ __forceinline__ v8bf frag_mc(const lds_char* lds_tile, int r0, int ks, int lane) {
  constexpr int CH = ROWS / 8;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int kA = ks * 32 + 8 * g + q;   // rows for elements 0..3
  const int kB = kA + 4;                // rows for elements 4..7
  const int ch = (r0 >> 3) + (p >> 1);  // 16-B chunk of columns r0+4p .. r0+4p+3
  const int sub = (p & 1) * 8;
  const lds_char* a = lds_tile + kA * ROWS * 2 + ((ch ^ mc_swz<CH>(kA)) << 4) + sub;
  const lds_char* b = lds_tile + kB * ROWS * 2 + ((ch ^ mc_swz<CH>(kB)) << 4) + sub;
  const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(a));
  const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(b));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

template <bool KC, int ROWS, int BKT = 64>
__device__ __forceinline__ v8bf frag(const lds_char* t, int r0, int ks, int lane) {
  if constexpr (KC) return frag_kc<BKT>(t, r0, ks, lane);
  else return frag_mc<ROWS>(t, r0, ks, lane);
}

template <bool KC, int ROWS, class Src, int NW = 4, int BKT = 64>
__device__ __forceinline__ void stage(const Src& s, lds_char* t, int rc0, int k0, int wave, int lane) {
  if constexpr (KC) stage_kc<ROWS, Src, NW, BKT>(s, t, rc0, k0, wave, lane);
  else stage_mc<ROWS, Src, NW, BKT>(s, t, rc0, k0, wave, lane);
}

// LDS-DMA instructions one wave issues to stage one K-step of a ROWS-wide operand
template <int ROWS, int NW, int BKT = 64>
constexpr int stage_loads() { return (ROWS * BKT * 2) / (1024 * NW); }

template <class C, bool AKC, bool BKC>
__device__ __forceinline__ void compute_tile(const lds_char* At, const lds_char* Bt, int wm, int wn, int lane,
                                             f32x4 (&acc)[4][4]) {
#pragma unroll
  for (int ks = 0; ks < C::BK / 32; ++ks) {
    v8bf a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = frag<AKC, C::BM, C::BK>(At, wm * 64 + i * 16, ks, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag<BKC, C::BN, C::BK>(Bt, wn * 64 + j * 16, ks, lane);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
  }
}

// ---- main loop -------------------------------------------------------------------------------
// Accumulates the K range [kbeg, kend) into acc[4][4].  STA(tile, k0) / STB(tile, k0) issue the
// LDS-DMA of one 64-deep K-step of the A / B operand into an LDS tile (generic stagers below,
// or implicit-GEMM gathers in conv.hip).
template <class C, bool AKC, bool BKC, class STA, class STB>
__device__ __forceinline__ void mainloop_st(const STA& sta, const STB& stb, lds_char* smem, int kbeg, int kend,
                                            f32x4 (&acc)[4][4]) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / C::WN, wn = wave % C::WN;
  constexpr int BK = C::BK;
  const int nk = (kend - kbeg + BK - 1) / BK;
  if (nk <= 0) return;
  if constexpr (C::STAGES == 1 && C::RP) {
    constexpr int KS = BK / 32;
    v8bf a[KS][4], b[KS][4];
    auto read_frags = [&]() {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[ks][i] = frag<AKC, C::BM, BK>(smem, wm * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[ks][j] = frag<BKC, C::BN, BK>(smem + C::A_BYTES, wn * 64 + j * 16, ks, lane);
      }
    };
    sta(smem, kbeg);
    stb(smem + C::A_BYTES, kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    read_frags();
    __syncthreads();  // every wave holds its fragments: the LDS buffer is free for the next DMA
    for (int kt = 0; kt < nk; ++kt) {
      const bool more = kt + 1 < nk;
      if (more) {
        sta(smem, kbeg + (kt + 1) * BK);
        stb(smem + C::A_BYTES, kbeg + (kt + 1) * BK);
      }
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks][i], b[ks][j], acc[i][j], 0, 0, 0);
      if (more) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        read_frags();
        __syncthreads();
      }
    }
  } else if constexpr (C::STAGES == 1) {
    for (int kt = 0; kt < nk; ++kt) {
      sta(smem, kbeg + kt * BK);
      stb(smem + C::A_BYTES, kbeg + kt * BK);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      compute_tile<C, AKC, BKC>(smem, smem + C::A_BYTES, wm, wn, lane, acc);
      __syncthreads();
    }
  } else if constexpr (C::STAGES >= 3) {
    // S-slot ring, prefetch distance D = S-1, one barrier per K-step.  At the top of step kt the
    // wave's outstanding LDS-DMA ops are those of tiles kt .. min(kt+D-1, nk-1) (LPS each, issued
    // in order; vmcnt retires in issue order): a counted vmcnt(younger*LPS) retires tile kt only,
    // the barrier publishes it to all waves (and certifies every wave is done reading slot
    // (kt+D)%S = (kt-1)%S), then tile kt+D's DMA is issued and tile kt computed.  Deep rings keep
    // (S-1) stages of operand bytes in flight per workgroup: what the memory-bound short-K GEMMs
    // need (bandwidth = bytes in flight / latency).
    constexpr int S = C::STAGES, D = S - 1;
    constexpr int LPS = stage_loads<C::BM, C::NW, BK>() + stage_loads<C::BN, C::NW, BK>();
#pragma unroll
    for (int i = 0; i < D; ++i)
      if (i < nk) {
        sta(smem + i * C::STAGE_BYTES, kbeg + i * BK);
        stb(smem + i * C::STAGE_BYTES + C::A_BYTES, kbeg + i * BK);
      }
    int slot = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int younger = min(D - 1, nk - 1 - kt);
      if constexpr (D - 1 >= 3) { if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LPS) : "memory"); }
      if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
      else if (younger == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // raw barrier: __syncthreads() would make the compiler drain every in-flight DMA (vmcnt(0)) here,
      // collapsing the ring to one stage of prefetch (cdna_hip_programming.md, glds pipelining rules)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (kt + D < nk) {
        const int sd = slot == 0 ? S - 1 : slot - 1;  // (kt + D) % S
        sta(smem + sd * C::STAGE_BYTES, kbeg + (kt + D) * BK);
        stb(smem + sd * C::STAGE_BYTES + C::A_BYTES, kbeg + (kt + D) * BK);
      }
      compute_tile<C, AKC, BKC>(smem + slot * C::STAGE_BYTES, smem + slot * C::STAGE_BYTES + C::A_BYTES, wm, wn, lane,
                                acc);
      slot = slot == S - 1 ? 0 : slot + 1;
    }
  } else {
    sta(smem, kbeg);
    stb(smem + C::A_BYTES, kbeg);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = (kt & 1) * C::STAGE_BYTES, nxt = C::STAGE_BYTES - cur;
      if (kt + 1 < nk) {
        sta(smem + nxt, kbeg + (kt + 1) * BK);
        stb(smem + nxt + C::A_BYTES, kbeg + (kt + 1) * BK);
      }
      compute_tile<C, AKC, BKC>(smem + cur, smem + cur + C::A_BYTES, wm, wn, lane, acc);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
}

template <class C, bool AKC, bool BKC, class SA, class SB>
__device__ __forceinline__ void mainloop(const SA& sa, const SB& sb, lds_char* smem, int bm0, int bn0, int kbeg,
                                         int kend, f32x4 (&acc)[4][4]) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  mainloop_st<C, AKC, BKC>(
      [&](lds_char* t, int k0) { stage<AKC, C::BM, SA, C::NW, C::BK>(sa, t, bm0, k0, wave, lane); },
      [&](lds_char* t, int k0) { stage<BKC, C::BN, SB, C::NW, C::BK>(sb, t, bn0, k0, wave, lane); },
                           smem, kbeg, kend, acc);
}

// ---- fast integer division by a runtime constant (Granlund-Montgomery), n < 2^31 --------------
struct FastDiv {
  uint32_t d, m, l;
  FastDiv() : d(1), m(1), l(0) {}
  explicit FastDiv(uint32_t dd) : d(dd) {
    l = 0;
    while ((1u << l) < d) ++l;
    m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  }
  __device__ __forceinline__ uint32_t div(uint32_t n) const {
    return (uint32_t)(((uint64_t)__umulhi(n, m) + n) >> l);
  }
  __device__ __forceinline__ void divmod(uint32_t n, uint32_t& q, uint32_t& r) const {
    q = div(n);
    r = n - q * d;
  }
};

// ---- epilogue ----------------------------------------------------------------------------------
// Stages the block's fp32 accumulators through LDS (EPI_ROWS rows at a time) so that every
// global store is a coalesced 16-byte vector; OP(row, col0, float (&v)[8]) finishes 8 consecutive
// columns (bias, residual/beta, activation, dtype) and stores them.
template <class C, class OP, bool FULL = false>
__device__ __forceinline__ void epilogue_staged(lds_char* smem, f32x4 (&acc)[4][4], int bm0, int bn0, int M, int N,
                                                const OP& op) {
  constexpr int LD = C::BN + 4;  // fp32 row pitch (pad breaks bank aliasing of the column writes)
  constexpr int R = C::EPI_ROWS;
  lds_float* st = reinterpret_cast<lds_float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WN, wn = wave % C::WN;
  __syncthreads();  // operand ring no longer read by anyone
#pragma unroll
  for (int pass = 0; pass < C::BM / R; ++pass) {
    // rows [pass*R, pass*R + R) belong to wave-row wm = pass*R/64, i-blocks (pass*R%64)/16 ...
    const int prow0 = pass * R;
    if (wm == prow0 / 64) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rblk = (i * 16) - (prow0 % 64);  // row offset of this i-block inside the pass
        if (rblk >= 0 && rblk < R) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              st[(rblk + (lane >> 4) * 4 + r) * LD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
        }
      }
    }
    __syncthreads();
    constexpr int CPR = C::BN / 8;  // 8-column groups per row
#pragma unroll
    for (int idx = tid; idx < R * CPR; idx += C::NTH) {
      const int rr = idx / CPR, cg = idx % CPR;
      const int m = bm0 + prow0 + rr, n = bn0 + cg * 8;
      if (FULL || (m < M && n < N)) {
        float v[8];
        const lds_float* s = st + rr * LD + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = s[k];
        op(m, n, v);
      }
    }
    __syncthreads();
  }
}

// epilogue_staged with operand prefetch, for epilogues that READ per-element inputs (the BN backward
// modes: the BN input x, the relu mask, the residual gradient).  Each pass first has every thread issue
// the loads of all its GPT groups (PRE(j, m, n, ok) -> the caller's registers), then stages the
// accumulators through LDS and finishes the groups (OP(j, m, n, v)).  The loads of a pass are thus in
// flight together and under the staging, instead of one group's loads per memory round trip: the
// stores of group j may alias the next group's loads (same C array), so the compiler cannot hoist
// them itself.  The barriers are raw s_barrier (LDS counter only): __syncthreads() would also drain
// the prefetch.  R rows per pass (a multiple of 16 dividing BM); GPT = R*BN/8/NTH groups per thread.
template <class C, int R, class PRE, class OP>
__device__ __forceinline__ void epilogue_staged_pf(lds_char* smem, f32x4 (&acc)[4][4], int bm0, int bn0, int M, int N,
                                                   const PRE& pre, const OP& op) {
  constexpr int LD = C::BN + 4;
  constexpr int CPR = C::BN / 8;
  static_assert(R % 16 == 0 && C::BM % R == 0, "pass height");
  static_assert(R * LD * 4 <= C::LDS_BYTES, "epilogue staging does not fit");
  static_assert((R * CPR) % C::NTH == 0, "whole groups per thread");
  constexpr int GPT = R * CPR / C::NTH;
  lds_float* st = reinterpret_cast<lds_float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / C::WN, wn = wave % C::WN;
  __syncthreads();  // operand ring no longer read by anyone
#pragma unroll
  for (int pass = 0; pass < C::BM / R; ++pass) {
    const int prow0 = pass * R;
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
      const int idx = tid + j * C::NTH, rr = idx / CPR, cg = idx % CPR;
      const int m = bm0 + prow0 + rr, n = bn0 + cg * 8;
      pre(j, m, n, m < M && n < N);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rblk = wm * 64 + i * 16 - prow0;  // this i-block's row offset inside the pass
      if (rblk >= 0 && rblk < R) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            st[(rblk + (lane >> 4) * 4 + r) * LD + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][r];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int j = 0; j < GPT; ++j) {
      const int idx = tid + j * C::NTH, rr = idx / CPR, cg = idx % CPR;
      const int m = bm0 + prow0 + rr, n = bn0 + cg * 8;
      if (m < M && n < N) {
        float v[8];
        const lds_float* sp = st + rr * LD + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = sp[k];
        op(j, m, n, v);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // LDS reads done before the next pass overwrites
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
}

// unpack 8 bf16 held as one 16-byte vector
__device__ __forceinline__ void unpack8_bf16(const uint4& v, float (&o)[8]) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  o[4] = __uint_as_float(v.z << 16); o[5] = __uint_as_float(v.z & 0xffff0000u);
  o[6] = __uint_as_float(v.w << 16); o[7] = __uint_as_float(v.w & 0xffff0000u);
}

}  // namespace gemm
}  // namespace dtg
