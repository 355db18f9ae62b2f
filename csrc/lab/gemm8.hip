// 256x256 bf16 GEMM, 8 waves, 8-phase staggered schedule (cdna_hip_programming.md §5 "The 256² 8-phase
// template", T3+T4+T5), for the large GEMMs of ResNet-50 (1x1 convs at batch 256) and BERT.
//
// Wave w = (wr = w>>2, wc = w&3) owns the 128x64 output block rows [128 wr, +128), cols [64 wc, +64)
// = acc[8][4] (16x16 MFMA tiles).  A K-tile (BK = 64) is split into four LDS "halves", each 128 rows x
// 64 k = 16 KB, arranged so that every phase reads exactly one A half and one B half:
//     A_h = rows {128 wr + 64 h + [0, 64)}  (the h-th 64-row quarter of both wave-row slabs)
//     B_h = cols {64 wc + 32 h + [0, 32)}   (the h-th 32-col half of every wave's column block)
// Phases per K-tile compute one (mq, nq) quadrant (64x32 per wave, 16 MFMA) in the order
//     P0 (0,0): ds_read A_0, B_0     P1 (1,0): ds_read A_1     P2 (1,1): ds_read B_1     P3 (0,1): -
// (A_0's fragments stay in registers until P3), so every half of buffer u&1 is read in exactly one
// phase (A_0, B_0 @P0, A_1 @P1, B_1 @P2) and is re-staged (LDS-DMA, 2 glds per thread per half) for
// a later tile at least two phases after that read:
//     tile u issues  P0: A_1(u+1)  P1: B_1(u+1)  P2: A_0(u+2)  P3: B_0(u+2)
// giving every half >= 3 phases of DMA flight.  Each phase = { ds_read; glds; s_barrier; lgkmcnt(0);
// setprio 1; 16 MFMA; setprio 0; counted vmcnt; s_barrier }.  Waves 4-7 run one barrier behind
// waves 0-3 (one extra s_barrier up front), so on every SIMD one wave is in its MFMA section while
// the other is in its load section.  With that stagger a DMA is visible to every reader two phases
// after the issuing waves' vmcnt, and a half can be overwritten two phases after its last read: the
// waits at the end of P0 / P2 / P3 retire exactly the halves read two phases later and leave the
// three newest halves (vmcnt 6) in flight; the tail counts are exact.
// All LDS is one __shared__ array (a second LDS object can make hipcc drain vmcnt each step).
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "lab.h"
#include "dtg/mfma_gemm.cuh"
#include "dtg/gemm_epi.cuh"
#include <type_traits>

namespace dtg {
using namespace gemm;

namespace g8 {

constexpr int BM = 256, BN = 256, NTH = 512, HALF = 16384, BUF = 4 * HALF;  // A0 A1 B0 B1 per buffer
constexpr int LDS = 2 * BUF;                                                  // 128 KB

// Stage half h of a KC operand: LDS [128 rows][64 k] (frag_kc layout), LDS row lr -> operand row
//   A: rc0 + 128 (lr / 64) + 64 h + lr % 64         B: rc0 + 64 (lr / 32) + 32 h + lr % 32
template <bool IS_A, class Src>
__device__ __forceinline__ void stage_half_kc(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = (wave * 2 + i) * 8;
    const int lr = r0 + (lane >> 3);
    const int row = IS_A ? rc0 + 128 * (lr >> 6) + 64 * h + (lr & 63) : rc0 + 64 * (lr >> 5) + 32 * h + (lr & 31);
    const int cl = lane & 7, c = cl ^ (lr & 7);
    __builtin_amdgcn_global_load_lds(src.chunk(row, k0 + c * 8), (lds_void*)(t + r0 * 128), 16, 0, 0);
  }
}

// Stage half h of an MC operand: LDS [64 k][128 cols] (frag_mc<128> layout), LDS col lc -> operand col
// with the same mapping as above
template <bool IS_A, class Src>
__device__ __forceinline__ void stage_half_mc(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
  constexpr int CH = 16, KPI = 4;  // 16 chunks per 256-B k-row, 4 k-rows per wave-instruction
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int kr0 = (wave * 2 + i) * KPI;
    const int kr = kr0 + lane / CH;
    const int cl = lane % CH, c = cl ^ mc_swz<CH>(kr);
    const int lc = c * 8;  // first of the 8 columns of this chunk (a chunk never straddles a run)
    const int col = IS_A ? rc0 + 128 * (lc >> 6) + 64 * h + (lc & 63) : rc0 + 64 * (lc >> 5) + 32 * h + (lc & 31);
    __builtin_amdgcn_global_load_lds(src.chunk(k0 + kr, col), (lds_void*)(t + kr0 * 256), 16, 0, 0);
  }
}

template <bool KC, bool IS_A, class Src>
__device__ __forceinline__ void stage_half(const Src& src, lds_char* t, int rc0, int h, int k0, int wave, int lane) {
  if constexpr (KC) stage_half_kc<IS_A>(src, t, rc0, h, k0, wave, lane);
  else stage_half_mc<IS_A>(src, t, rc0, h, k0, wave, lane);
}

template <bool KC>
__device__ __forceinline__ v8bf hfrag(const lds_char* t, int r0, int ks, int lane) {
  if constexpr (KC) return frag_kc(t, r0, ks, lane);
  else return frag_mc<128>(t, r0, ks, lane);
}

}  // namespace g8

template <bool AKC, bool BKC, class SA, class SB>
__global__ void __launch_bounds__(512, 1) gemm8_kernel(SA sa, SB sb, int M, int N, int K, int tiles_n, int split_k,
                                                       int k_per_split, Epi e, float* __restrict__ ws) {
  using namespace g8;
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BN;
  const int kbeg = blockIdx.y * k_per_split;
  const int kend = min(K, kbeg + k_per_split);
  const int nk = (kend - kbeg + BK - 1) / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half slots: buffer u&1, A_h at h*HALF, B_h at (2+h)*HALF
  auto A_h = [&](int u, int h) { return smem + (u & 1) * BUF + h * HALF; };
  auto B_h = [&](int u, int h) { return smem + (u & 1) * BUF + (2 + h) * HALF; };
  auto stA = [&](int u, int h) { g8::stage_half<AKC, true>(sa, A_h(u, h), bm0, h, kbeg + u * BK, wave, lane); };
  auto stB = [&](int u, int h) { g8::stage_half<BKC, false>(sb, B_h(u, h), bn0, h, kbeg + u * BK, wave, lane); };

  if (nk > 0) {
    // prologue: tile 0 plus the two tile-1 halves steady state issues two phases before tile 0
    // starts; retire A_0, B_0, A_1 of tile 0 (needed by P0/P1), keep 3 halves in flight
    stA(0, 0);
    stB(0, 0);
    stA(0, 1);
    stB(0, 1);
    if (nk > 1) {
      stA(1, 0);
      stB(1, 0);
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // raw barrier: __syncthreads would drain the in-flight DMA
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger: waves 4-7 run one barrier behind

    // A_0 fragments stay in registers from P0 to P3 (a0), A_1 from P1 to P2 (a1), so every half is
    // read from LDS in exactly one phase and can be re-staged early (>= 3 phases of DMA flight)
    v8bf a0[4][2], a1[4][2], b[2][2];
    for (int u = 0; u < nk; ++u) {
      const bool n1 = u + 1 < nk, n2 = u + 2 < nk;
      // ---- P0: quadrant (0,0): read A_0, B_0; issue A_1(u+1); retire B_1(u)
      {
        const lds_char* ta = A_h(u, 0);
        const lds_char* tb = B_h(u, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a0[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::hfrag<BKC>(tb, wc * 32 + j * 16, ks, lane);
        if (n1) stA(u + 1, 1);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i][ks], b[j][ks], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      // ---- P1: quadrant (1,0): read A_1; issue B_1(u+1)
      {
        const lds_char* ta = A_h(u, 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a1[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
        if (n1) stB(u + 1, 1);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i][ks], b[j][ks], acc[4 + i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        __builtin_amdgcn_s_barrier();
      }
      // ---- P2: quadrant (1,1): read B_1; issue A_0(u+2); retire A_0(u+1), B_0(u+1)
      {
        const lds_char* tb = B_h(u, 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::hfrag<BKC>(tb, wc * 32 + j * 16, ks, lane);
        if (n2) stA(u + 2, 0);
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[4 + i][2 + j] =
                  __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[i][ks], b[j][ks], acc[4 + i][2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      // ---- P3: quadrant (0,1): registers only (a0, B_1); issue B_0(u+2); retire A_1(u+1)
      {
        if (n2) stB(u + 2, 0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
              acc[i][2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[i][ks], b[j][ks], acc[i][2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  // ---- epilogue: 8 passes of 32 rows through LDS (fp32, padded rows), 16-B stores
  constexpr int LD = BN + 4, R = 32;
  lds_float* stg = reinterpret_cast<lds_float*>(smem);
  const bool slab = split_k > 1;
  float* slab_p = ws + (long long)blockIdx.y * M * N;
#pragma unroll
  for (int pass = 0; pass < BM / R; ++pass) {  // fully unrolled: acc is indexed with constants only
    if (wr == pass / 4) {
      const int ib = (pass % 4) * 2;  // the two 16-row m-tiles of this pass
#pragma unroll
      for (int ii = 0; ii < 2; ++ii)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            stg[(ii * 16 + (lane >> 4) * 4 + r) * LD + wc * 64 + j * 16 + (lane & 15)] = acc[ib + ii][j][r];
    }
    __syncthreads();
    constexpr int CPR = BN / 8;
    for (int idx = tid; idx < R * CPR; idx += NTH) {
      const int rr = idx / CPR, cg = idx % CPR;
      const int m = bm0 + pass * R + rr, n = bn0 + cg * 8;
      if (m < M && n < N) {
        float v[8];
        const lds_float* s = stg + rr * LD + cg * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = s[k];
        if (slab) {
          float* p = slab_p + (long long)m * N + n;
          if ((N & 3) == 0 && n + 8 <= N) store8_f32(p, v);
          else
            for (int k = 0; k < 8 && n + k < N; ++k) p[k] = v[k];
        } else {
          epi_store8(e, N, m, n, v);
        }
      }
    }
    __syncthreads();
  }
}

// ---- persistent variant (gemm8p) ----------------------------------------------------------------
// The same 8-phase schedule with the K loop flattened over every (tile, K-tile) pair a workgroup owns,
// so the LDS-DMA of the next output tile's first K-tiles is in flight under the current tile's last
// phases and its epilogue: a short reduction (BERT's K = 768, 12 K-tiles per 256x256 tile) no longer
// pays a pipeline fill and drain per tile.  One workgroup per CU (grid 256); workgroup b serves linear
// tiles L = i * 256 + 32 (b % 8) + b / 8, so the 32 tiles an XCD runs at once are consecutive in
// row-major tile order and share their A row slabs and B column slabs in that XCD's L2.
//
// The epilogue needs no LDS and no barrier: the MFMA operands are swapped (N-side fragment as src A), so
// a lane's accumulator holds 4 consecutive output COLUMNS of one row, and the B fragments are read with
// a column permutation that gives each lane 8 consecutive columns per 32-column half:
//     MFMA row q of n-tile jt in half h  ->  column 32 h + 8 (q >> 2) + 4 jt + (q & 3)
// (the B halves use their own chunk swizzles, swz8p_kc / swz8p_mc, under which the permuted reads stay
// bank-conflict free).  Lane l then finishes row (l & 15) of each 16-row m-tile at columns
// [32 h + 8 (l >> 4), +8) straight from registers with 16-byte stores; the four lane groups cover 64
// contiguous bytes of a row per store instruction.  The bias of the tile arrives by LDS-DMA with the last
// K-tile's operands, the first K-tile's MFMAs take a zero accumulator (no register clearing), and the two
// counted waits after an epilogue leave its stores in flight (vmcnt 6 + stores) instead of draining them.
namespace g8 {

// B-half swizzles of the persistent kernel: the permuted fragment read touches LDS rows {8 g + 4 jt + (q & 3)}
// (KC) / column groups {4 c0 + p} of four k-rows (MC), so the chunk XOR is chosen to make the 8 (KC) or 16
// (MC) lanes of one read pass hit distinct 16-B slots:  KC chunk ^ swz8p_kc(row), MC chunk ^ swz8p_mc(k-row)
__device__ __forceinline__ int swz8p_kc(int r) { return (r & 3) | ((r >> 1) & 4); }
__device__ __forceinline__ int swz8p_mc(int k) { return (k & 3) << 2; }

template <bool KC>
__device__ __forceinline__ v8bf bfrag_perm(const lds_char* t, int cb, int jt, int ks, int lane) {
  const int q = lane & 15;
  if constexpr (KC) {
    const int r = cb + (q >> 2) * 8 + jt * 4 + (q & 3);
    const int c = ks * 4 + (lane >> 4);
    return *reinterpret_cast<const lds_v8bf*>(t + r * 128 + ((c ^ swz8p_kc(r)) << 4));
  } else {
    // ds_read_tr16_b64: address lane (k-row qk, column group p) feeds MFMA rows 4p..4p+3 (frag_mc)
    constexpr int ROWS = 128;
    const int qk = q >> 2, p = q & 3;
    const int kA = ks * 32 + 8 * (lane >> 4) + qk, kB = kA + 4;
    const int ch = (cb >> 3) + p, sub = jt * 8;
    const lds_char* a = t + kA * ROWS * 2 + ((ch ^ swz8p_mc(kA)) << 4) + sub;
    const lds_char* b = t + kB * ROWS * 2 + ((ch ^ swz8p_mc(kB)) << 4) + sub;
    // inline asm: hipcc cannot tell the transposed read from a read of the in-flight LDS-DMA destination and
    // puts an s_waitcnt vmcnt(0) before the intrinsic form, draining the pipeline every phase; the kernel's own
    // counted vmcnt + barrier order the DMA, and its lgkmcnt(0) + sched_barrier retire these reads
    v4bf lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"((unsigned)(uintptr_t)a) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"((unsigned)(uintptr_t)b) : "memory");
    return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  }
}

// epilogue modes: 0 plain, 1 + bias, 2 + bias -> GELU with GELU'(pre) saved to aux, 3 x aux (GELU backward)
template <int EM>
__device__ __forceinline__ void epi8p(const Epi& e, int m, int n, float (&v)[8], const float (&bias)[8]) {
  const long long off = (long long)m * e.ldc + n;
  if constexpr (EM == 1 || EM == 2) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += bias[k];
  }
  if constexpr (EM == 2) {
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x = v[k], sg = gelu_sig(x);
      const float du = 0.7978845608028654f * fmaf(3.f * 0.044715f * x, x, 1.f);
      d[k] = fmaf(2.f * x * sg * (1.f - sg), du, sg);
      v[k] = x * sg;
    }
    store8_bf16_nt((bf16_t*)e.aux + off, d);
  }
  store8_bf16((bf16_t*)e.C + off, v);
}

// EM 3's saved GELU' rows: all 16 loads of a lane issued before the first use (one wait behind the in-flight
// DMA instead of one round trip per row)
__device__ __forceinline__ void mul_raw8(float (&v)[8], const u32x4v& w) {
  v[0] *= __uint_as_float(w.x << 16); v[1] *= __uint_as_float(w.x & 0xffff0000u);
  v[2] *= __uint_as_float(w.y << 16); v[3] *= __uint_as_float(w.y & 0xffff0000u);
  v[4] *= __uint_as_float(w.z << 16); v[5] *= __uint_as_float(w.z & 0xffff0000u);
  v[6] *= __uint_as_float(w.w << 16); v[7] *= __uint_as_float(w.w & 0xffff0000u);
}

}  // namespace g8

// ABL (timing ablations for tools/gemm_ab.py only, results are garbage): 1 = no operand DMA after the
// prologue, 2 = no barriers inside the K loop
template <bool BKC, int EM, int ABL = 0>
__global__ void __launch_bounds__(512, 1) gemm8p_kernel(const bf16_t* __restrict__ A, long long lda,
                                                        const bf16_t* __restrict__ B, long long ldb, int K,
                                                        int tiles_n, int tiles, Epi e) {
  using namespace g8;
  constexpr bool AKC = true;
  constexpr bool BIAS = EM == 1 || EM == 2;
  // VM-counter instructions one epilogue issues per lane (16-B stores of C, of aux, loads of aux)
  constexpr int EPI_VM = (EM == 2 || EM == 3) ? 32 : 16;
  constexpr int BIAS_OFF = LDS;  // 8 waves x 2 tile parities x 64 fp32 bias values after the operand ring
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS + 2 * 8 * 256];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int G = gridDim.x;  // a multiple of 8
  const int base = (blockIdx.x & 7) * (G >> 3) + (blockIdx.x >> 3);
  const int my_tiles = base < tiles ? (tiles - base + G - 1) / G : 0;
  const int nk = K / BK;        // >= 2 (host), so positions u+1 and u+2 lie in this tile or the next
  const int U = my_tiles * nk;  // flattened (tile, K-tile) iterations of this workgroup

  f32x4 acc[8][4];
  const f32x4 zero4 = {0.f, 0.f, 0.f, 0.f};

  auto A_h = [&](int u, int h) { return smem + (u & 1) * BUF + h * HALF; };
  auto B_h = [&](int u, int h) { return smem + (u & 1) * BUF + (2 + h) * HALF; };
  auto tile_rc = [&](int ti, int& bm0, int& bn0) {
    const int L = ti * G + base;
    bm0 = (L / tiles_n) * BM;
    bn0 = (L % tiles_n) * BN;
  };
  // Per-lane byte offsets of the staged 16-B chunks relative to the (scalar) tile/K-step base (the chunk
  // maps of stage_half_kc / stage_half_mc, B with the swz8p_* swizzles): tile-invariant, so the loop's
  // address work is one scalar base per stage.
  unsigned offA[2][2], offB[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = (wave * 2 + i) * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (lr & 7);
      offA[h][i] = (unsigned)(((long long)(128 * (lr >> 6) + 64 * h + (lr & 63)) * lda + c * 8) * 2);
      if constexpr (BKC) {
        const int cb = (lane & 7) ^ swz8p_kc(lr);
        offB[h][i] = (unsigned)(((long long)(64 * (lr >> 5) + 32 * h + (lr & 31)) * ldb + cb * 8) * 2);
      } else {
        const int kr = (wave * 2 + i) * 4 + lane / 16;
        const int lc = ((lane % 16) ^ swz8p_mc(kr)) * 8;
        offB[h][i] = (unsigned)(((long long)kr * ldb + 64 * (lc >> 5) + 32 * h + (lc & 31)) * 2);
      }
    }
  // tile coordinates of the current tile and the next one; position u+d (d <= 2) is in one of them
  int kk = 0, ti = 0, cur_bm, cur_bn, nxt_bm, nxt_bn;
  tile_rc(0, cur_bm, cur_bn);
  tile_rc(1, nxt_bm, nxt_bn);
  auto stA = [&](int u, int d, int h) {
    if constexpr (ABL == 1) { if (u > 0) return; }
    const int k = kk + d;
    const int bm = k < nk ? cur_bm : nxt_bm, k0 = (k < nk ? k : k - nk) * BK;
    const char* sb = (const char*)(A + (long long)bm * lda + k0);
    lds_char* t = A_h(u + d, h);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(sb + offA[h][i]), (lds_void*)(t + (wave * 2 + i) * 8 * 128), 16,
                                       0, 0);
  };
  auto stB = [&](int u, int d, int h) {
    if constexpr (ABL == 1) { if (u > 0) return; }
    const int k = kk + d;
    const int bn = k < nk ? cur_bn : nxt_bn, k0 = (k < nk ? k : k - nk) * BK;
    lds_char* t = B_h(u + d, h);
    if constexpr (BKC) {
      const char* sb = (const char*)(B + (long long)bn * ldb + k0);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(sb + offB[h][i]), (lds_void*)(t + (wave * 2 + i) * 8 * 128),
                                         16, 0, 0);
    } else {
      const char* sb = (const char*)(B + (long long)k0 * ldb + bn);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(sb + offB[h][i]), (lds_void*)(t + (wave * 2 + i) * 4 * 256),
                                         16, 0, 0);
    }
  };
  // 16 MFMAs of one quadrant; on a tile's first K-tile the first k-step starts from a zero accumulator
#define DTG_G8P_QUAD(I0, J0, AF)                                                                        \
  if (kk == 0) {                                                                                        \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j) {     \
      acc[I0 + i][J0 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][0], AF[i][0], zero4, 0, 0, 0); \
      acc[I0 + i][J0 + j] =                                                                             \
          __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][1], AF[i][1], acc[I0 + i][J0 + j], 0, 0, 0);     \
    }                                                                                                   \
  } else {                                                                                              \
    _Pragma("unroll") for (int i = 0; i < 4; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)         \
        _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) acc[I0 + i][J0 + j] =                          \
        __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j][ks], AF[i][ks], acc[I0 + i][J0 + j], 0, 0, 0);     \
  }

#define DTG_G8P_BAR()                                   \
  do {                                                  \
    if constexpr (ABL != 2) __builtin_amdgcn_s_barrier(); \
  } while (0)
  if (U > 0) {
    stA(0, 0, 0);
    stB(0, 0, 0);
    stA(0, 0, 1);
    stB(0, 0, 1);
    stA(0, 1, 0);  // U >= nk >= 2
    stB(0, 1, 0);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (wr == 1) __builtin_amdgcn_s_barrier();

    v8bf a0[4][2], a1[4][2], b[2][2];
    bool post = false;  // this iteration follows an epilogue: its P0 / P2 waits also leave those stores in flight
    for (int u = 0; u < U; ++u) {
      const bool n1 = u + 1 < U, n2 = u + 2 < U;
      // ---- P0: quadrant (0,0)
      {
        const lds_char* ta = A_h(u, 0);
        const lds_char* tb = B_h(u, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a0[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::bfrag_perm<BKC>(tb, wc * 32, j, ks, lane);
        if constexpr (BIAS) {
          // the tile's bias (this wave's 64 columns) by LDS-DMA with its last K-tile; retired by the P2 wait
          if (kk == nk - 1)
            __builtin_amdgcn_global_load_lds((const void*)(e.bias + cur_bn + wc * 64 + lane),
                                             (lds_void*)(smem + BIAS_OFF + ((ti & 1) * 8 + wave) * 256), 4, 0, 0);
        }
        if (n1) stA(u, 1, 1);
        DTG_G8P_BAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs below the wait (asm-read operands)
        __builtin_amdgcn_s_setprio(1);
        DTG_G8P_QUAD(0, 0, a0)
        __builtin_amdgcn_s_setprio(0);
        if (!n1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else if (post) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + EPI_VM) : "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        DTG_G8P_BAR();
      }
      // ---- P1: quadrant (1,0)
      {
        const lds_char* ta = A_h(u, 1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) a1[i][ks] = g8::hfrag<AKC>(ta, wr * 64 + i * 16, ks, lane);
        if (n1) stB(u, 1, 1);
        DTG_G8P_BAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs below the wait (asm-read operands)
        __builtin_amdgcn_s_setprio(1);
        DTG_G8P_QUAD(4, 0, a1)
        __builtin_amdgcn_s_setprio(0);
        DTG_G8P_BAR();
      }
      // ---- P2: quadrant (1,1)
      {
        const lds_char* tb = B_h(u, 1);
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) b[j][ks] = g8::bfrag_perm<BKC>(tb, wc * 32, j, ks, lane);
        if (n2) stA(u, 2, 0);
        DTG_G8P_BAR();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs below the wait (asm-read operands)
        __builtin_amdgcn_s_setprio(1);
        DTG_G8P_QUAD(4, 2, a1)
        __builtin_amdgcn_s_setprio(0);
        if (!n2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (post) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 + EPI_VM) : "memory");
        else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        DTG_G8P_BAR();
      }
      // ---- P3: quadrant (0,1)
      {
        if (n2) stB(u, 2, 0);
        DTG_G8P_BAR();
        __builtin_amdgcn_s_setprio(1);
        DTG_G8P_QUAD(0, 2, a0)
        __builtin_amdgcn_s_setprio(0);
        if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        DTG_G8P_BAR();
      }
      post = false;
      // ---- tile finished: epilogue from registers while the next tile's first K-tiles stream in
      if (++kk == nk) {
        const int bm0 = cur_bm, bn0 = cur_bn;
        const int fq = lane >> 4;
        u32x4v pre[2][8];
        if constexpr (EM == 3) {
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int i = 0; i < 8; ++i)
              pre[h][i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(
                  (const bf16_t*)e.aux + (long long)(bm0 + wr * 128 + i * 16 + (lane & 15)) * e.ldc + bn0 + wc * 64 +
                  h * 32 + fq * 8));
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int n = bn0 + wc * 64 + h * 32 + fq * 8;
          float bias[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          if constexpr (BIAS) {
            const lds_float* bl =
                reinterpret_cast<const lds_float*>(smem + BIAS_OFF + ((ti & 1) * 8 + wave) * 256) + h * 32 + fq * 8;
#pragma unroll
            for (int k = 0; k < 8; ++k) bias[k] = bl[k];
          }
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int m = bm0 + wr * 128 + i * 16 + (lane & 15);
            float v[8];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              v[r] = acc[i][2 * h][r];
              v[4 + r] = acc[i][2 * h + 1][r];
            }
            if constexpr (EM == 3) g8::mul_raw8(v, pre[h][i]);
            g8::epi8p<EM>(e, m, n, v, bias);
          }
        }
        kk = 0;
        ++ti;
        cur_bm = nxt_bm;
        cur_bn = nxt_bn;
        tile_rc(ti + 1, nxt_bm, nxt_bn);
        post = true;
      }
    }
#undef DTG_G8P_QUAD
#undef DTG_G8P_BAR
    if (wr == 0) __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---- host ----------------------------------------------------------------------------------------
template <bool BK_, int EM, int ABL = 0>
static void launch8p(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                     const Epi& e, hipStream_t st) {
  const int tiles_n = N / g8::BN, tiles = (M / g8::BM) * tiles_n;
  hipLaunchKernelGGL((gemm8p_kernel<BK_, EM, ABL>), dim3(256), dim3(g8::NTH), 0, st, A, lda, B, ldb, K, tiles_n, tiles, e);
  DTG_LAUNCH_CHECK();
}

template <int EM>
static void launch8p_b(int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K,
                       const Epi& e, hipStream_t st) {
  if (b_kc) launch8p<true, EM>(A, lda, B, ldb, M, N, K, e, st);
  else launch8p<false, EM>(A, lda, B, ldb, M, N, K, e, st);
}

int gemm8p_mode(const Epi& e) {
  if (!e.c_bf16 || e.alpha != 1.f || e.beta != 0.f || (e.ldc & 7)) return -1;
  if (!e.bias && e.act == 0 && e.aux_mode == 0) return 0;
  if (e.bias && e.act == 0 && e.aux_mode == 0) return 1;
  if (e.bias && e.act == 2 && e.aux_mode == 3) return 2;
  if (!e.bias && e.act == 0 && e.aux_mode == 4) return 3;
  return -1;
}

bool gemm8p_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, const Epi& e,
                 int M, int N, int K, hipStream_t st, int abl) {
  const int em = gemm8p_mode(e);
  if (em < 0 || !a_kc || M % g8::BM || N % g8::BN || K % BK || K < 2 * BK || (lda & 7) || (ldb & 7)) return false;
  // per-lane chunk offsets are 32-bit byte offsets from the tile base (at most 256 rows / 64 k-rows of a
  // leading dimension)
  if (256LL * lda * 2 >= (1LL << 31) || 256LL * ldb * 2 >= (1LL << 31)) return false;
  if ((long long)(M / g8::BM) * (N / g8::BN) < 256) return false;  // fewer tiles than CUs: not persistent work
  if (abl) {  // timing ablations: plain epilogue, KC B only
    if (em != 0 || !b_kc) return false;
    if (abl == 1) launch8p<true, 0, 1>(A, lda, B, ldb, M, N, K, e, st);
    else launch8p<true, 0, 2>(A, lda, B, ldb, M, N, K, e, st);
    return true;
  }
  switch (em) {
    case 0: launch8p_b<0>(b_kc, A, lda, B, ldb, M, N, K, e, st); break;
    case 1: launch8p_b<1>(b_kc, A, lda, B, ldb, M, N, K, e, st); break;
    case 2: launch8p_b<2>(b_kc, A, lda, B, ldb, M, N, K, e, st); break;
    default: launch8p_b<3>(b_kc, A, lda, B, ldb, M, N, K, e, st); break;
  }
  return true;
}

template <bool AK, bool BK_, bool GUARD>
static void launch8(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M, int N, int K, int split_k,
                    int kps, const Epi& e, float* ws, hipStream_t st) {
  using SA = std::conditional_t<AK, DenseKC<GUARD>, DenseMC<GUARD>>;
  using SB = std::conditional_t<BK_, DenseKC<GUARD>, DenseMC<GUARD>>;
  SA sa{A, lda, M, K};
  SB sb{B, ldb, N, K};
  const int tiles_m = (M + g8::BM - 1) / g8::BM, tiles_n = (N + g8::BN - 1) / g8::BN;
  dim3 grid(tiles_m * tiles_n, split_k);
  hipLaunchKernelGGL((gemm8_kernel<AK, BK_, SA, SB>), grid, dim3(g8::NTH), 0, st, sa, sb, M, N, K, tiles_n, split_k,
                     kps, e, ws); DTG_LAUNCH_CHECK();
}

template <bool GUARD>
static void launch8_layout(int a_kc, int b_kc, const bf16_t* A, long long lda, const bf16_t* B, long long ldb, int M,
                           int N, int K, int split_k, int kps, const Epi& e, float* ws, hipStream_t st) {
  if (a_kc && b_kc) launch8<true, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else if (a_kc) launch8<true, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else if (b_kc) launch8<false, true, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else launch8<false, false, GUARD>(A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
}

void gemm8_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, const Epi& e,
                int M, int N, int K, int split_k, int kps, float* ws, hipStream_t st) {
  const bool full = (M % g8::BM == 0) && (N % g8::BN == 0) && (K % BK == 0);
  if (full) launch8_layout<false>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  else launch8_layout<true>(a_kc, b_kc, A, lda, B, ldb, M, N, K, split_k, kps, e, ws, st);
  if (split_k > 1) gemm_splitk_reduce(ws, split_k, M, N, e, st);
}

}  // namespace dtg
