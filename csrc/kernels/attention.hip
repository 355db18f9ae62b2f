// Fused multi-head attention for BERT-style encoders (head dim 64, additive key mask,
// attention-probability dropout from the counter hash), forward and backward, on MFMA.
//
// Forward  (grid: [B*nh, ceil(S/128)], 8 waves; a wave owns 16 query rows, a workgroup 128 queries):
//   K and V of the (b, h) are staged once per 128 queries (once per head at S = 128) into LDS by LDS-DMA (K row-major/KC, V as k-major MC
//   tiles read back with ds_read_b64_tr_b16); Q fragments come straight from global memory.  Per
//   64-key chunk, transposed: S^T = K Q^T (8 MFMA; a lane holds one query x 4 consecutive keys per block) ->
//   scale + mask -> online softmax (per-lane running max / sum; two cross-lane steps for the chunk max) ->
//   dropout(P) through a per-wave LDS scratch (one 8-byte store per block) -> O^T += V^T P^T (8 MFMA).  Writes O
//   (bf16, coalesced through LDS) and LSE = m + log(l) per row for the backward.  No [S, S] matrix reaches HBM.
// Backward (grid: [B*nh], 8 waves; a wave owns 16 keys; S in {64, 128}; longer S: two launches, below):
//   recomputes P^T = exp(K Q^T * scale + mask - LSE) per 32-query chunk, then
//   dV += dropout(P)^T dO,  dP^T = V dO^T,  dS^T = P^T (dropout'(dP^T) - D),  dK += dS^T Q * scale;
//   dS is kept whole in LDS, so after one barrier dQ = dS K * scale is a plain MFMA pass per
//   16-query wave (no atomics).  D = rowsum(dO * O) is computed in the prologue.
//   A lane's accumulator elements are 4 consecutive keys of one query, so dropout(P) and dS are
//   stored query-major (one 8-byte LDS store per matrix and 16-query block) and read back as
//   transposed fragments (ds_read_b64_tr_b16) where the key-major operand is needed.
//
// Fragment conventions as in dtg/mfma_gemm.cuh: mfma(a = X_A[m][k], b = X_B[n][k]) accumulates
// C[m][n], lane l holding C[(l>>4)*4 + r][l & 15].
// dbias (optional, fp32 [3 * nh * 64]): the QKV bias gradient, column sums of dQ | dK | dV over all B * S rows,
// added in the backward's epilogue (per-wave sums, combined over the workgroup in LDS, one device atomic per
// column and workgroup) instead of a second pass over the 3H-wide dQKV.
// The dropout element index is ((b*nh + h)*S + q)*S + key, drawn by the pair hash (keep_attn below), identical to
// attn_softmax_fwd and to the PyTorch mirror (dtg/ops/transformer.py attn_dropout_keep) -- the fused and unfused
// paths agree bit-for-bit on which probabilities are dropped.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"

namespace dtg {
using namespace gemm;

namespace {

__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
// Attention-probability dropout: ONE hash per pair of adjacent keys.  Element idx (= ((b*nh + h)*S + q)*S + key)
// is kept iff the low (even idx) / high (odd idx) 16 bits of fmix32((idx >> 1) * golden + seed) are >= th16 =
// floor(p * 2^16): half the hashes of a per-element draw, and the kernels hold 4 consecutive keys per lane.
__device__ __forceinline__ uint32_t pair_hash(uint32_t seed, uint32_t pidx) { return fmix32(pidx * 0x9E3779B1u + seed); }
__device__ __forceinline__ bool keep_attn(uint32_t seed, uint32_t idx, uint32_t th16) {
  const uint32_t h = pair_hash(seed, idx >> 1);
  return ((idx & 1u) ? (h >> 16) : (h & 0xffffu)) >= th16;
}
// keep flags of 4 consecutive keys starting at an even idx
__device__ __forceinline__ void keep4_attn(uint32_t seed, uint32_t idx0, uint32_t th16, bool (&k)[4]) {
  const uint32_t h0 = pair_hash(seed, idx0 >> 1), h1 = pair_hash(seed, (idx0 >> 1) + 1u);
  k[0] = (h0 & 0xffffu) >= th16;
  k[1] = (h0 >> 16) >= th16;
  k[2] = (h1 & 0xffffu) >= th16;
  k[3] = (h1 >> 16) >= th16;
}

// 16 B of a KC row straight from global memory (A/B fragment of a [rows][64] operand)
__device__ __forceinline__ v8bf gfrag(const bf16_t* base, long long ld, int row0, int ks, int lane) {
  const bf16_t* p = base + (long long)(row0 + (lane & 15)) * ld + ks * 32 + 8 * (lane >> 4);
  return *reinterpret_cast<const v8bf*>(p);
}

// byte offset of element (row, k) in a [rows][64] bf16 KC tile with the frag_kc swizzle
__device__ __forceinline__ int kc_off(int row, int k) { return row * 128 + ((((k >> 3) ^ (row & 7))) << 4) + (k & 7) * 2; }

typedef __attribute__((ext_vector_type(2))) uint32_t u32x2v;
// 4 bf16 (8 bytes) into LDS
__device__ __forceinline__ void st4_bf16(lds_char* p, const float (&v)[4]) {
  u32x2v w;
  w.x = pack_bf2(v[0], v[1]);
  w.y = pack_bf2(v[2], v[3]);
  *reinterpret_cast<__attribute__((address_space(3))) u32x2v*>(p) = w;
}

__device__ __forceinline__ void st_bf16(lds_char* base, int off, float v) {
  *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(base + off) = f2bf(v);
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Column sums of a wave's 16 C-layout rows x 64 columns (v * scale): the lane's 4 rows, then the 4 lane groups
// that share a column (xor 16, 32).  Lanes 0-15 hold columns j * 16 + lane.
__device__ __forceinline__ void colsum16(const f32x4 (&v)[4], float scale, float (&s)[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float t = (v[j][0] + v[j][1]) + (v[j][2] + v[j][3]);
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    s[j] = t * scale;
  }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
constexpr int kFwdWaves = 8;  // 128 queries per workgroup: K/V of a head staged once at S <= 128

template <int SMAX>
__global__ void __launch_bounds__(64 * kFwdWaves) attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
                                                       bf16_t* __restrict__ out, float* __restrict__ lse, int S, int nh,
                                                       float scale, uint32_t th, float dscale, uint32_t seed) {
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int H = nh * 64;
  const long long ld = 3LL * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bf16_t* Qg = qkv + (long long)b * S * ld + h * 64;
  const bf16_t* Kg = Qg + H;
  const bf16_t* Vg = Qg + 2 * H;
  lds_char* Kt = smem;                      // [S][64] KC
  lds_char* Vt = smem + S * 128;            // S/64 MC tiles [64 keys][64 d]
  lds_char* scr = smem + 2 * S * 128 + wave * 2048;  // per-wave [16][64] bf16
  const int nkc = S / 64;
  {
    DenseKC<false> ks_{Kg, ld, S, 64};
    DenseMC<false> vs_{Vg, ld, 64, S};
    for (int c = 0; c < nkc; ++c) {
      stage_kc<64, DenseKC<false>, kFwdWaves>(ks_, Kt + c * 8192, c * 64, 0, wave, lane);
      stage_mc<64, DenseMC<false>, kFwdWaves>(vs_, Vt + c * 8192, 0, c * 64, wave, lane);
    }
  }
  const int q0 = blockIdx.y * (16 * kFwdWaves) + wave * 16;
  const bool active = q0 < S;  // S % 64 == 0: the last workgroup of S = 64 * odd has 4 idle waves
  v8bf qa[2];
  if (active) {
    qa[0] = gfrag(Qg, ld, q0, 0, lane);
    qa[1] = gfrag(Qg, ld, q0, 1, lane);
  }
  // the additive key mask of batch b, staged once (was one global load per 16-key block and chunk,
  // each on the critical path of the softmax)
  lds_float* Mk = reinterpret_cast<lds_float*>(smem + 2 * S * 128 + kFwdWaves * 2048);
  for (int i = threadIdx.x; i < S; i += 64 * kFwdWaves) Mk[i] = mask ? mask[(long long)b * S + i] : 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!active) return;  // (no barrier below this point)
  // Transposed form: S^T = K Q^T and O^T = V^T P^T, so lane (q = lane & 15, g = lane >> 4) holds, per 16-key block
  // j, the scores of ONE query q0 + q against 4 consecutive keys j * 16 + 4g + [0, 4): the softmax statistics are
  // per lane (running max / sum need 2 cross-lane steps per chunk for the max and one final sum, not 4 rows x 4
  // steps each), the dropout pairs are in-lane (2 hashes per 4 keys), P leaves as one 8-byte LDS store per block,
  // and O^T's accumulators (4 consecutive d per block) rescale by the lane's own alpha.
  float m = -INFINITY, l = 0.f;  // l: this lane's partial sum (its 16 of every 64 keys), combined at the end
  f32x4 o[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qi = lane & 15, g = lane >> 4;
  const uint32_t qrow = ((uint32_t)bh * (uint32_t)S + (uint32_t)(q0 + qi)) * (uint32_t)S;  // dropout index base
  for (int kc = 0; kc < nkc; ++kc) {
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        s[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_kc(Kt + kc * 8192, j * 16, ks, lane), qa[ks], s[j], 0, 0, 0);
    }
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 madd = *reinterpret_cast<const __attribute__((address_space(3))) f32x4*>(Mk + kc * 64 + j * 16 + 4 * g);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[j][r] = fmaf(s[j][r], scale, madd[r]);
        mx = fmaxf(mx, s[j][r]);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = __expf(m - mn);
    m = mn;
    float rs = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key0 = kc * 64 + j * 16 + 4 * g;
      float pd[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pd[r] = __expf(s[j][r] - mn);
        rs += pd[r];
      }
      if (th) {
        const uint32_t pidx = (qrow + (uint32_t)key0) >> 1;
        const uint32_t h0 = pair_hash(seed, pidx), h1 = pair_hash(seed, pidx + 1u);
        pd[0] = (h0 & 0xffffu) >= th ? pd[0] * dscale : 0.f;
        pd[1] = (h0 >> 16) >= th ? pd[1] * dscale : 0.f;
        pd[2] = (h1 & 0xffffu) >= th ? pd[2] * dscale : 0.f;
        pd[3] = (h1 >> 16) >= th ? pd[3] * dscale : 0.f;
      }
      st4_bf16(scr + kc_off(qi, j * 16 + 4 * g), pd);  // P [16 q][64 keys] KC: 4 keys in one 16-B chunk
    }
    l = l * alpha + rs;
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= alpha;
    lds_fence();
    const v8bf pb0 = frag_kc(scr, 0, 0, lane), pb1 = frag_kc(scr, 0, 1, lane);  // X_B[q][key]
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_mc<64>(Vt + kc * 8192, j * 16, 0, lane), pb0, o[j], 0, 0, 0);
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_mc<64>(Vt + kc * 8192, j * 16, 1, lane), pb1, o[j], 0, 0, 0);
    }
    lds_fence();  // the scratch is rewritten by the next chunk
  }
  // finalize: O^T / l -> scratch ([16 q][64 d], 4 consecutive d per lane and block; 16-B chunks XOR-swizzled by the
  // row, so the 16 rows of a store do not all hit the same banks) -> 16-B global stores
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float il = 1.f / l;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float v[4] = {o[j][0] * il, o[j][1] * il, o[j][2] * il, o[j][3] * il};
    st4_bf16(scr + qi * 128 + (((2 * j + (g >> 1)) ^ (qi & 7)) << 4) + (g & 1) * 8, v);
  }
  if (g == 0) lse[(long long)bh * S + q0 + qi] = m + __logf(l);
  lds_fence();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;  // 128 chunks of 16 B: row c/8, chunk c%8
    const int row = c >> 3, ch = c & 7;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(scr + row * 128 + ((ch ^ (row & 7)) << 4));
    *reinterpret_cast<v8bf*>(out + ((long long)b * S + q0 + row) * H + h * 64 + ch * 8) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Backward, S in {64, 128}: one workgroup (8 waves) per (b, h); wave w owns keys [16w, 16w+16).
// LDS (S = 128: 74 KB, so two workgroups share a CU): Q and dO as MC tiles (ds_read_b64_tr_b16
// B-operands), the whole dS [S q][S keys] bf16 (written by the key-waves; dK reads it transposed, dQ
// = dS K row-wise -- no atomics), D / LSE / mask rows, and per-wave [32 q][16 keys] scratch for
// dropout(P).  K is only read by phase 2, so it is staged into the Q tile after phase 1 (its DMA
// overlaps the dK / dV stores, which stage through the dO tile).
//   phase 1 (per 32-query chunk): S^T = K Q^T, dP^T = V dO^T (16 MFMA) -> P^T, dropout, dS^T
//            -> dV += Pd^T dO, dK += dS^T Q (8 MFMA)
//   phase 2 (after a barrier): wave w computes dQ for query rows [16w, 16w+16) over all keys.
// Gradients leave through LDS staging as 16-byte row stores.
// rows [row0, row0+16) x 64 bf16 of a wave's C-layout accumulators -> global (16-B stores) via a
// 2 KB per-wave LDS staging area
__device__ __forceinline__ void store_rows16(lds_char* stg, const f32x4 (&v)[4], float scale, bf16_t* g, long long ldg,
                                             int lane) {
  const int rbase = (lane >> 4) * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) st_bf16(stg, (rbase + r) * 128 + (j * 16 + (lane & 15)) * 2, v[j][r] * scale);
  lds_fence();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i, row = c >> 3, ch = c & 7;
    const v8bf x = *reinterpret_cast<const lds_v8bf*>(stg + row * 128 + ch * 16);
    *reinterpret_cast<v8bf*>(g + row * ldg + ch * 8) = x;
  }
  lds_fence();
}

template <int S_>
__global__ void __launch_bounds__(512) attn_bwd_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                       const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                       const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                       int nh, float scale, uint32_t th, float dscale, uint32_t seed,
                                                       float* __restrict__ dbias) {
  constexpr int S = S_, NW = 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int H = nh * 64;
  const long long ld = 3LL * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bf16_t* Qg = qkv + (long long)b * S * ld + h * 64;
  const bf16_t* Kg = Qg + H;
  const bf16_t* Vg = Qg + 2 * H;
  const bf16_t* Og = o + (long long)b * S * H + h * 64;
  const bf16_t* dOg = dout + (long long)b * S * H + h * 64;
  lds_char* Qt = smem;                         // MC [q][d]; phase 2: K as MC [key][d]
  lds_char* dOt = Qt + S * 128;                // MC [q][d]; phase 2: per-wave output staging
  lds_char* Kt = Qt;
  lds_char* dSq = dOt + S * 128;               // dS [S q][S key] bf16, MC-swizzled rows
  lds_float* Ds = reinterpret_cast<lds_float*>(dSq + S * S * 2);
  lds_float* Ls = Ds + S;
  lds_float* Ms = Ls + S;
  lds_char* scr = reinterpret_cast<lds_char*>(Ms + S) + wave * 1024;  // [32 q][16 keys]
  {
    DenseMC<false> qs_{Qg, ld, 64, S};
    DenseMC<false> ds_{dOg, (long long)H, 64, S};
#pragma unroll
    for (int c = 0; c < S / 64; ++c) {
      stage_mc<64, DenseMC<false>, NW>(qs_, Qt + c * 8192, 0, c * 64, wave, lane);
      stage_mc<64, DenseMC<false>, NW>(ds_, dOt + c * 8192, 0, c * 64, wave, lane);
    }
  }
  if (tid < 2 * S) {  // D[q] = sum_d dO[q, d] * O[q, d]: two threads per row
    const int q = tid >> 1, half = tid & 1;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a[8], bb[8];
      load8_bf16(dOg + (long long)q * H + half * 32 + c * 8, a);
      load8_bf16(Og + (long long)q * H + half * 32 + c * 8, bb);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += a[k] * bb[k];
    }
    acc += __shfl_xor(acc, 1, 64);
    if (half == 0) Ds[q] = acc;
  }
  if (tid < S) {
    Ls[tid] = lse[(long long)bh * S + tid];
    Ms[tid] = mask ? mask[(long long)b * S + tid] : 0.f;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int rbase = (lane >> 4) * 4;
  const int kb = wave * 16;
  const bool has_keys = kb < S;
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dk[j] = dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (has_keys) {
    constexpr float kLog2e = 1.4426950408889634f;
    // the lane's 4 keys are fixed for the whole pass: their mask terms (base-2 units) live in registers
    float msl[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) msl[r] = Ms[kb + rbase + r] * kLog2e;
    const float sl2 = scale * kLog2e;
    const v8bf ka0 = gfrag(Kg, ld, kb, 0, lane), ka1 = gfrag(Kg, ld, kb, 1, lane);
    const v8bf va0 = gfrag(Vg, ld, kb, 0, lane), va1 = gfrag(Vg, ld, kb, 1, lane);
#pragma unroll 1
    for (int qc = 0; qc < S; qc += 32) {
      const int tq = qc >> 6, kq = (qc & 63) >> 5;
      f32x4 st[2], dpt[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        // B fragments (16 queries x 32 d) read row-wise out of the staged MC tiles (undoing their swizzle)
        // instead of from global memory
        const int qrow = (qc & 63) + ni * 16 + (lane & 15), cb = lane >> 4;
        const int sw = mc_swz<8>(qrow);
        const lds_char* qt = Qt + tq * 8192 + qrow * 128;
        const lds_char* dt = dOt + tq * 8192 + qrow * 128;
        const v8bf qb0 = *reinterpret_cast<const lds_v8bf*>(qt + ((cb ^ sw) << 4));
        const v8bf qb1 = *reinterpret_cast<const lds_v8bf*>(qt + (((4 + cb) ^ sw) << 4));
        const v8bf db0 = *reinterpret_cast<const lds_v8bf*>(dt + ((cb ^ sw) << 4));
        const v8bf db1 = *reinterpret_cast<const lds_v8bf*>(dt + (((4 + cb) ^ sw) << 4));
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka0, qb0, z, 0, 0, 0);
        st[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka1, qb1, z, 0, 0, 0);
        z = f32x4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va0, db0, z, 0, 0, 0);
        dpt[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va1, db1, z, 0, 0, 0);
      }
      // lane: one query q, 4 consecutive keys -> one 8-byte store per matrix into q-major tiles
      // (dropout(P) into the wave's [32 q][16 key] scratch, dS into dS [S q][S key]); both are
      // read back as transposed (MC) fragments
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int ql = ni * 16 + (lane & 15), q = qc + ql;
        const float lq = Ls[q] * kLog2e, dq = Ds[q];
        const uint32_t ib = ((uint32_t)bh * (uint32_t)S + (uint32_t)q) * (uint32_t)S + (uint32_t)(kb + rbase);
        float pd[4], dsv[4];
        bool kp[4] = {true, true, true, true};
        if (th) keep4_attn(seed, ib, th, kp);  // ib even: kb + rbase is a multiple of 4
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[ni][r], sl2, msl[r] - lq));
          float pv = p, dp = dpt[ni][r];
          if (th) {
            pv = kp[r] ? p * dscale : 0.f;
            dp = kp[r] ? dp * dscale : 0.f;
          }
          pd[r] = pv;
          dsv[r] = p * (dp - dq);
        }
        st4_bf16(scr + ql * 32 + rbase * 2, pd);
        const int key0 = kb + rbase;
        st4_bf16(dSq + q * (S * 2) + ((((key0 >> 3) ^ mc_swz<S / 8>(q))) << 4) + (key0 & 7) * 2, dsv);
      }
      lds_fence();
      const v8bf pa = frag_mc<16>(scr, 0, 0, lane);        // dropout(P)^T [16 keys][32 q]
      const v8bf sa = frag_mc<S>(dSq, kb, qc >> 5, lane);   // dS^T [16 keys][32 q]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dv[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, frag_mc<64>(dOt + tq * 8192, j * 16, kq, lane), dv[j], 0,
                                                        0, 0);
        dk[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, frag_mc<64>(Qt + tq * 8192, j * 16, kq, lane), dk[j], 0,
                                                        0, 0);
      }
      lds_fence();  // scratch rewritten by the next chunk
    }
  }
  __syncthreads();  // dS complete; the Q / dO tiles are free
  {  // K for dQ = dS K into the Q tile: its DMA is in flight while dK / dV are stored
    DenseMC<false> kss{Kg, ld, 64, S};
#pragma unroll
    for (int c = 0; c < S / 64; ++c) stage_mc<64, DenseMC<false>, NW>(kss, Kt + c * 8192, 0, c * 64, wave, lane);
  }
  lds_char* stg = dOt + wave * 2048;  // per-wave output staging inside the dO tile (16 or 32 KB)
  // bias-gradient partials: the wave's [dQ | dK | dV] column sums in its (now idle) P scratch
  lds_float* bsum = reinterpret_cast<lds_float*>(scr);
  if (dbias) {
    float sk[4] = {0.f, 0.f, 0.f, 0.f}, sv[4] = {0.f, 0.f, 0.f, 0.f};
    if (has_keys) {
      colsum16(dk, scale, sk);
      colsum16(dv, 1.f, sv);
    }
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bsum[64 + j * 16 + lane] = sk[j];
        bsum[128 + j * 16 + lane] = sv[j];
      }
    }
  }
  if (has_keys) {
    bf16_t* gk = dqkv + ((long long)b * S + kb) * ld + H + h * 64;
    store_rows16(stg, dk, scale, gk, ld, lane);
    store_rows16(stg, dv, 1.f, gk + H, ld, lane);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // K staged by every wave
  const int qr = wave * 16;
  if (qr < S) {
    f32x4 dq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int qa_ = qr + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < S / 32; ++kk) {
      // X_A[q][key] = dS: row q of the q-major tile, 8 consecutive keys (its MC swizzle undone)
      const int c = kk * 4 + (lane >> 4);
      const v8bf a = *reinterpret_cast<const lds_v8bf*>(dSq + qa_ * (S * 2) + ((c ^ mc_swz<S / 8>(qa_)) << 4));
#pragma unroll
      for (int j = 0; j < 4; ++j)
        dq[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, frag_mc<64>(Kt + (kk >> 1) * 8192, j * 16, kk & 1, lane),
                                                        dq[j], 0, 0, 0);
    }
    store_rows16(stg, dq, scale, dqkv + ((long long)b * S + qr) * ld + h * 64, ld, lane);
    if (dbias) {
      float sq[4];
      colsum16(dq, scale, sq);
      if (lane < 16)
#pragma unroll
        for (int j = 0; j < 4; ++j) bsum[j * 16 + lane] = sq[j];
    }
  } else if (dbias && lane < 16) {
#pragma unroll
    for (int j = 0; j < 4; ++j) bsum[j * 16 + lane] = 0.f;
  }
  if (dbias) {  // (kernel argument: uniform) 8 wave partials -> one atomic per column
    __syncthreads();
    if (tid < 192) {
      const int part = tid >> 6, c = tid & 63;
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) t += reinterpret_cast<lds_float*>(Ms + S)[w * 256 + tid];
      atomicAdd(dbias + part * H + h * 64 + c, t);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Backward at 128 < S <= 512: the whole dS of a head no longer fits LDS (S = 512: 512 KB), so the
// backward is split in two launches that each recompute P (flash-attention style, no [S, S] tensor
// in HBM and no atomics):
//   dKV (grid [B*nh, S/128], 8 waves, wave w owns keys 128*y + 16w + [0, 16)): phase 1 of the
//       kernel above over all S queries in 32-query chunks; dropout(P)^T and dS^T go through two
//       per-wave [32 q][16 key] scratches instead of the head's dS matrix.
//   dQ  (grid [B*nh, S/128], 8 waves, wave w owns queries 128*y + 16w + [0, 16)): K and V of the
//       head staged once as KC tiles (the forward's layout); per 64-key chunk S = Q K^T and
//       dP = dO V^T (16 MFMA), dS = P (dropout'(dP) - D) into the wave's [16 q][64 key] KC scratch,
//       dQ += dS K (8 MFMA) with K read TRANSPOSED out of its KC image (frag_tr_kc).
// LDS at S = 512: dKV 148 KB (Q, dO MC tiles), dQ 146 KB (K, V KC tiles): one workgroup per CU.

// B fragment X_B[n][k] = T[k][n] of a KC image T [rows = k][64 cols = n] (frag_kc's swizzle): the
// MC-orientation read of a tile that was staged row-wise (ds_read_b64_tr_b16, 4 rows x 4 cols per lane
// address; the chunk XOR moves whole 16-B chunks, so each 8-byte half stays contiguous)
__device__ __forceinline__ v8bf frag_tr_kc(const lds_char* t, int n0, int ks, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int kA = ks * 32 + 8 * g + q, kB = kA + 4;
  const int ch = (n0 + 4 * p) >> 3, sub = (p & 1) * 8;
  const lds_char* a = t + kA * 128 + ((ch ^ (kA & 7)) << 4) + sub;
  const lds_char* b = t + kB * 128 + ((ch ^ (kB & 7)) << 4) + sub;
  const v4bf lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(a));
  const v4bf hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_v4bf*)(b));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

constexpr int kLongKeys = 128;  // keys (dKV) / queries (dQ) per workgroup of the long backward

__global__ void __launch_bounds__(512) attn_bwd_dkv_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                           const bf16_t* __restrict__ dout,
                                                           const float* __restrict__ lse,
                                                           const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                           int S, int nh, float scale, uint32_t th, float dscale,
                                                           uint32_t seed, float* __restrict__ dbias) {
  constexpr int NW = 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int H = nh * 64;
  const long long ld = 3LL * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bf16_t* Qg = qkv + (long long)b * S * ld + h * 64;
  const bf16_t* Kg = Qg + H;
  const bf16_t* Vg = Qg + 2 * H;
  const bf16_t* Og = o + (long long)b * S * H + h * 64;
  const bf16_t* dOg = dout + (long long)b * S * H + h * 64;
  lds_char* Qt = smem;                          // S/64 MC tiles [64 q][64 d]
  lds_char* dOt = Qt + S * 128;                 // same for dO; after the loop: per-wave output staging
  lds_float* Ds = reinterpret_cast<lds_float*>(dOt + S * 128);
  lds_float* Ls = Ds + S;
  lds_char* scr = reinterpret_cast<lds_char*>(Ls + S) + wave * 2048;  // [32 q][16 keys] x {P, dS}
  const int kb = blockIdx.y * kLongKeys + wave * 16;
  const bool has_keys = kb < S;  // wave-uniform
  const int rbase = (lane >> 4) * 4;
  constexpr float kLog2e = 1.4426950408889634f;
  float msl[4] = {0.f, 0.f, 0.f, 0.f};
  if (has_keys && mask) {
#pragma unroll
    for (int r = 0; r < 4; ++r) msl[r] = mask[(long long)b * S + kb + rbase + r] * kLog2e;
  }
  {
    DenseMC<false> qs_{Qg, ld, 64, S};
    DenseMC<false> ds_{dOg, (long long)H, 64, S};
    for (int c = 0; c < S / 64; ++c) {
      stage_mc<64, DenseMC<false>, NW>(qs_, Qt + c * 8192, 0, c * 64, wave, lane);
      stage_mc<64, DenseMC<false>, NW>(ds_, dOt + c * 8192, 0, c * 64, wave, lane);
    }
  }
  for (int i = tid; i < 2 * S; i += 64 * NW) {  // D[q] = sum_d dO[q, d] * O[q, d]: two threads per row
    const int q = i >> 1, half = i & 1;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float a[8], bb[8];
      load8_bf16(dOg + (long long)q * H + half * 32 + c * 8, a);
      load8_bf16(Og + (long long)q * H + half * 32 + c * 8, bb);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += a[k] * bb[k];
    }
    acc += __shfl_xor(acc, 1, 64);
    if (half == 0) Ds[q] = acc;
  }
  for (int i = tid; i < S; i += 64 * NW) Ls[i] = lse[(long long)bh * S + i];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 dk[4], dv[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dk[j] = dv[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (has_keys) {
    const float sl2 = scale * kLog2e;
    const v8bf ka0 = gfrag(Kg, ld, kb, 0, lane), ka1 = gfrag(Kg, ld, kb, 1, lane);
    const v8bf va0 = gfrag(Vg, ld, kb, 0, lane), va1 = gfrag(Vg, ld, kb, 1, lane);
    lds_char* scp = scr;
    lds_char* scs = scr + 1024;
#pragma unroll 1
    for (int qc = 0; qc < S; qc += 32) {
      const int tq = qc >> 6, kq = (qc & 63) >> 5;
      f32x4 st[2], dpt[2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int qrow = (qc & 63) + ni * 16 + (lane & 15), cb = lane >> 4;
        const int sw = mc_swz<8>(qrow);
        const lds_char* qt = Qt + tq * 8192 + qrow * 128;
        const lds_char* dt = dOt + tq * 8192 + qrow * 128;
        const v8bf qb0 = *reinterpret_cast<const lds_v8bf*>(qt + ((cb ^ sw) << 4));
        const v8bf qb1 = *reinterpret_cast<const lds_v8bf*>(qt + (((4 + cb) ^ sw) << 4));
        const v8bf db0 = *reinterpret_cast<const lds_v8bf*>(dt + ((cb ^ sw) << 4));
        const v8bf db1 = *reinterpret_cast<const lds_v8bf*>(dt + (((4 + cb) ^ sw) << 4));
        f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka0, qb0, z, 0, 0, 0);
        st[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka1, qb1, z, 0, 0, 0);
        z = f32x4{0.f, 0.f, 0.f, 0.f};
        z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va0, db0, z, 0, 0, 0);
        dpt[ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va1, db1, z, 0, 0, 0);
      }
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        const int ql = ni * 16 + (lane & 15), q = qc + ql;
        const float lq = Ls[q] * kLog2e, dq = Ds[q];
        const uint32_t ib = ((uint32_t)bh * (uint32_t)S + (uint32_t)q) * (uint32_t)S + (uint32_t)(kb + rbase);
        float pd[4], dsv[4];
        bool kp[4] = {true, true, true, true};
        if (th) keep4_attn(seed, ib, th, kp);  // ib even: kb + rbase is a multiple of 4
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = __builtin_amdgcn_exp2f(fmaf(st[ni][r], sl2, msl[r] - lq));
          float pv = p, dp = dpt[ni][r];
          if (th) {
            pv = kp[r] ? p * dscale : 0.f;
            dp = kp[r] ? dp * dscale : 0.f;
          }
          pd[r] = pv;
          dsv[r] = p * (dp - dq);
        }
        st4_bf16(scp + ql * 32 + rbase * 2, pd);
        st4_bf16(scs + ql * 32 + rbase * 2, dsv);
      }
      lds_fence();
      const v8bf pa = frag_mc<16>(scp, 0, 0, lane);  // dropout(P)^T [16 keys][32 q]
      const v8bf sa = frag_mc<16>(scs, 0, 0, lane);  // dS^T [16 keys][32 q]
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dv[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, frag_mc<64>(dOt + tq * 8192, j * 16, kq, lane), dv[j], 0,
                                                        0, 0);
        dk[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, frag_mc<64>(Qt + tq * 8192, j * 16, kq, lane), dk[j], 0,
                                                        0, 0);
      }
      lds_fence();  // scratches rewritten by the next chunk
    }
  }
  __syncthreads();  // every wave is done with the Q / dO tiles
  if (has_keys) {
    lds_char* stg = dOt + wave * 2048;
    bf16_t* gk = dqkv + ((long long)b * S + kb) * ld + H + h * 64;
    store_rows16(stg, dk, scale, gk, ld, lane);
    store_rows16(stg, dv, 1.f, gk + H, ld, lane);
    if (dbias) {  // (long sequences: one device atomic per column and wave)
      float sk[4], sv[4];
      colsum16(dk, scale, sk);
      colsum16(dv, 1.f, sv);
      if (lane < 16)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          atomicAdd(dbias + H + h * 64 + j * 16 + lane, sk[j]);
          atomicAdd(dbias + 2 * H + h * 64 + j * 16 + lane, sv[j]);
        }
    }
  }
}

__global__ void __launch_bounds__(512) attn_bwd_dq_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                          const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                          const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                          int S, int nh, float scale, uint32_t th, float dscale,
                                                          uint32_t seed, float* __restrict__ dbias) {
  constexpr int NW = 8;
  extern __shared__ __attribute__((aligned(16))) char smem_raw[];
  lds_char* smem = (lds_char*)smem_raw;
  const int H = nh * 64;
  const long long ld = 3LL * H;
  const int bh = blockIdx.x, b = bh / nh, h = bh % nh;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bf16_t* Qg = qkv + (long long)b * S * ld + h * 64;
  const bf16_t* Kg = Qg + H;
  const bf16_t* Vg = Qg + 2 * H;
  const bf16_t* Og = o + (long long)b * S * H + h * 64;
  const bf16_t* dOg = dout + (long long)b * S * H + h * 64;
  lds_char* Kt = smem;                        // S/64 KC tiles [64 keys][64 d]
  lds_char* Vt = smem + S * 128;              // same for V
  lds_float* Mk = reinterpret_cast<lds_float*>(smem + 2 * S * 128);
  lds_char* scr = reinterpret_cast<lds_char*>(Mk + S) + wave * 2048;  // dS [16 q][64 keys] KC
  {
    DenseKC<false> ks_{Kg, ld, S, 64};
    DenseKC<false> vs_{Vg, ld, S, 64};
    for (int c = 0; c < S / 64; ++c) {
      stage_kc<64, DenseKC<false>, NW>(ks_, Kt + c * 8192, c * 64, 0, wave, lane);
      stage_kc<64, DenseKC<false>, NW>(vs_, Vt + c * 8192, c * 64, 0, wave, lane);
    }
  }
  constexpr float kLog2e = 1.4426950408889634f;
  for (int i = tid; i < S; i += 64 * NW) Mk[i] = mask ? mask[(long long)b * S + i] * kLog2e : 0.f;
  const int q0 = blockIdx.y * kLongKeys + wave * 16;
  const bool active = q0 < S;  // wave-uniform
  const int rbase = (lane >> 4) * 4;
  v8bf qa[2], da[2];
  float lq[4], dd[4];
  if (active) {
    qa[0] = gfrag(Qg, ld, q0, 0, lane);
    qa[1] = gfrag(Qg, ld, q0, 1, lane);
    da[0] = gfrag(dOg, (long long)H, q0, 0, lane);
    da[1] = gfrag(dOg, (long long)H, q0, 1, lane);
    // D of the wave's 16 rows: 4 lanes per row, 16 d each
    const int row = lane >> 2, part = lane & 3;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float a[8], bb[8];
      load8_bf16(dOg + (long long)(q0 + row) * H + part * 16 + c * 8, a);
      load8_bf16(Og + (long long)(q0 + row) * H + part * 16 + c * 8, bb);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += a[k] * bb[k];
    }
    acc += __shfl_xor(acc, 1, 64);
    acc += __shfl_xor(acc, 2, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      dd[r] = __shfl(acc, (rbase + r) * 4, 64);
      lq[r] = lse[(long long)bh * S + q0 + rbase + r] * kLog2e;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!active) return;  // (no barrier below this point)
  const float sl2 = scale * kLog2e;
  f32x4 dq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int kc = 0; kc < S / 64; ++kc) {
    const lds_char* kt = Kt + kc * 8192;
    const lds_char* vt = Vt + kc * 8192;
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        s[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], frag_kc(kt, j * 16, ks, lane), s[j], 0, 0, 0);
        dp[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[ks], frag_kc(vt, j * 16, ks, lane), dp[j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kc * 64 + j * 16 + (lane & 15);
      const float mk = Mk[key];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __builtin_amdgcn_exp2f(fmaf(s[j][r], sl2, mk - lq[r]));
        float dpv = dp[j][r];
        if (th) {
          const uint32_t idx = ((uint32_t)bh * (uint32_t)S + (uint32_t)(q0 + rbase + r)) * (uint32_t)S + (uint32_t)key;
          dpv = keep_attn(seed, idx, th) ? dpv * dscale : 0.f;
        }
        st_bf16(scr, kc_off(rbase + r, j * 16 + (lane & 15)), p * (dpv - dd[r]));
      }
    }
    lds_fence();
    const v8bf a0 = frag_kc(scr, 0, 0, lane), a1 = frag_kc(scr, 0, 1, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dq[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, frag_tr_kc(kt, j * 16, 0, lane), dq[j], 0, 0, 0);
      dq[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, frag_tr_kc(kt, j * 16, 1, lane), dq[j], 0, 0, 0);
    }
    lds_fence();  // the scratch is rewritten by the next chunk
  }
  store_rows16(scr, dq, scale, dqkv + ((long long)b * S + q0) * ld + h * 64, ld, lane);
  if (dbias) {
    float sq[4];
    colsum16(dq, scale, sq);
    if (lane < 16)
#pragma unroll
      for (int j = 0; j < 4; ++j) atomicAdd(dbias + h * 64 + j * 16 + lane, sq[j]);
  }
}

// 16-bit threshold of the pair-hash dropout (keep_attn); 0 = no dropout
static uint32_t drop_th(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 65536.0;
  return t >= 65535.0 ? 0xffffu : (t < 1.0 ? 1u : (uint32_t)t);
}

int attn_fused_supported(int S, int dh, int backward) {
  if (dh != 64 || S % 64 != 0 || S <= 0) return 0;
  return S <= 512;  // backward: the one-launch kernel at S <= 128, the dKV + dQ pair above that
}

static size_t fwd_lds(int S) { return (size_t)2 * S * 128 + kFwdWaves * 2048 + (size_t)S * 4; }
static size_t bwd_lds(int S) { return (size_t)2 * S * 128 + (size_t)S * S * 2 + 3 * S * 4 + 8 * 1024; }
static size_t dkv_lds(int S) { return (size_t)2 * S * 128 + (size_t)2 * S * 4 + 8 * 2048; }
static size_t dq_lds(int S) { return (size_t)2 * S * 128 + (size_t)S * 4 + 8 * 2048; }

void attn_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse, int B, int S, int nh, float p,
              uint32_t seed, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_kernel<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)fwd_lds(512)));
    attr = true;
  }
  const uint32_t th = drop_th(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  dim3 grid(B * nh, (S + 16 * kFwdWaves - 1) / (16 * kFwdWaves));
  hipLaunchKernelGGL(attn_fwd_kernel<512>, grid, dim3(64 * kFwdWaves), fwd_lds(S), st, qkv, mask, out, lse, S, nh, 0.125f, th,
                     ds, seed); DTG_LAUNCH_CHECK();
}

void attn_bwd(const bf16_t* qkv, const bf16_t* o, const bf16_t* dout, const float* lse, const float* mask,
              bf16_t* dqkv, int B, int S, int nh, float p, uint32_t seed, float* dbias, hipStream_t st) {
  const uint32_t th = drop_th(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  static bool attr = false;
  if (!attr) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_kernel<128>,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)bwd_lds(128)));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_dkv_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)dkv_lds(512)));
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_dq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)dq_lds(512)));
    attr = true;
  }
  if (S > 128) {
    const dim3 grid(B * nh, (S + kLongKeys - 1) / kLongKeys);
    hipLaunchKernelGGL(attn_bwd_dkv_kernel, grid, dim3(512), dkv_lds(S), st, qkv, o, dout, lse, mask, dqkv, S, nh,
                       0.125f, th, ds, seed, dbias); DTG_LAUNCH_CHECK();
    hipLaunchKernelGGL(attn_bwd_dq_kernel, grid, dim3(512), dq_lds(S), st, qkv, o, dout, lse, mask, dqkv, S, nh,
                       0.125f, th, ds, seed, dbias); DTG_LAUNCH_CHECK();
  } else if (S == 64) {
    hipLaunchKernelGGL(attn_bwd_kernel<64>, dim3(B * nh), dim3(512), bwd_lds(64), st, qkv, o, dout, lse, mask, dqkv,
                       nh, 0.125f, th, ds, seed, dbias); DTG_LAUNCH_CHECK();
  } else {
    hipLaunchKernelGGL(attn_bwd_kernel<128>, dim3(B * nh), dim3(512), bwd_lds(128), st, qkv, o, dout, lse, mask,
                       dqkv, nh, 0.125f, th, ds, seed, dbias); DTG_LAUNCH_CHECK();
  }
}

}  // namespace dtg
