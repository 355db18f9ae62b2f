// Fused multi-head attention for BERT-style encoders (head dim 64, additive key mask,
// attention-probability dropout from the counter hash), forward and backward, on MFMA.
//
// Forward  (grid: [B*nh, S/64], 4 waves; a wave owns 16 query rows):
//   K and V of the (b, h) are staged once into LDS by LDS-DMA (K row-major/KC, V as k-major MC
//   tiles read back with ds_read_b64_tr_b16); Q fragments come straight from global memory.  Per
//   64-key chunk: S = Q K^T (8 MFMA) -> scale + mask -> online softmax (running max / sum per row,
//   reductions across the 16 lanes that share a row) -> dropout(P) through a per-wave LDS
//   scratch into A-fragment layout -> O += P V (8 MFMA).  Writes O (bf16, coalesced through LDS) and
//   LSE = m + log(l) per row for the backward.  No [S, S] matrix ever reaches HBM.
// Backward (grid: [B*nh], 4 waves; a wave owns 32 keys; S <= 128):
//   recomputes P^T = exp(K Q^T * scale + mask - LSE) per 32-query chunk, then
//   dV += dropout(P)^T dO,  dP^T = V dO^T,  dS^T = P^T (dropout'(dP^T) - D),  dK += dS^T Q * scale,
//   dQ += dS K * scale (LDS fp32 accumulator shared by the 4 key-waves, ds_add),
//   with D = rowsum(dO * O) computed in the prologue.  40 MFMA per wave per chunk.
//
// Fragment conventions as in dtg/mfma_gemm.cuh: mfma(a = X_A[m][k], b = X_B[n][k]) accumulates
// C[m][n], lane l holding C[(l>>4)*4 + r][l & 15].
// The dropout element index is ((b*nh + h)*S + q)*S + key, identical to attn_softmax_fwd and to
// the PyTorch mirror (dtg/ops/transformer.py) -- the fused and unfused paths agree bit-for-bit on
// which probabilities are dropped.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/mfma_gemm.cuh"
#include <stdlib.h>

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
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t idx, uint32_t thresh) {
  return fmix32(idx * 0x9E3779B1u + seed) >= thresh;
}

// 16 B of a KC row straight from global memory (A/B fragment of a [rows][64] operand)
__device__ __forceinline__ v8bf gfrag(const bf16_t* base, long long ld, int row0, int ks, int lane) {
  const bf16_t* p = base + (long long)(row0 + (lane & 15)) * ld + ks * 32 + 8 * (lane >> 4);
  return *reinterpret_cast<const v8bf*>(p);
}

// byte offset of element (row, k) in a [rows][64] bf16 KC tile with the frag_kc swizzle
__device__ __forceinline__ int kc_off(int row, int k) { return row * 128 + ((((k >> 3) ^ (row & 7))) << 4) + (k & 7) * 2; }

// byte offset of element (k, col) in a [k][32] bf16 MC tile with the frag_mc<32> swizzle
__device__ __forceinline__ int mc32_off(int k, int col) {
  return k * 64 + ((((col >> 3) ^ mc_swz<4>(k))) << 4) + (col & 7) * 2;
}

__device__ __forceinline__ void st_bf16(lds_char* base, int off, float v) {
  *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(base + off) = f2bf(v);
}

__device__ __forceinline__ void lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace

// ---------------------------------------------------------------------------------------------
template <int SMAX>
__global__ void __launch_bounds__(256) attn_fwd_kernel(const bf16_t* __restrict__ qkv, const float* __restrict__ mask,
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
      stage_kc<64>(ks_, Kt + c * 8192, c * 64, 0, wave, lane);
      stage_mc<64>(vs_, Vt + c * 8192, 0, c * 64, wave, lane);
    }
  }
  const int q0 = blockIdx.y * 64 + wave * 16;
  v8bf qa[2];
  qa[0] = gfrag(Qg, ld, q0, 0, lane);
  qa[1] = gfrag(Qg, ld, q0, 1, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const float* mk = mask ? mask + (long long)b * S : nullptr;
  float m[4], l[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m[r] = -INFINITY;
    l[r] = 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rbase = (lane >> 4) * 4;  // this lane's 4 C rows
  for (int kc = 0; kc < nkc; ++kc) {
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
        s[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[ks], frag_kc(Kt + kc * 8192, j * 16, ks, lane), s[j], 0, 0, 0);
    }
    float mx[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mx[r] = -INFINITY;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float madd = mk ? mk[kc * 64 + j * 16 + (lane & 15)] : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[j][r] = s[j][r] * scale + madd;
        mx[r] = fmaxf(mx[r], s[j][r]);
      }
    }
    float alpha[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o_ = 1; o_ < 16; o_ <<= 1) mx[r] = fmaxf(mx[r], __shfl_xor(mx[r], o_, 64));
      const float mn = fmaxf(m[r], mx[r]);
      alpha[r] = __expf(m[r] - mn);
      m[r] = mn;
      rs[r] = 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kc * 64 + j * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[j][r] - m[r]);
        rs[r] += p;
        float pd = p;
        if (th) {
          const uint32_t idx = (uint32_t)(((long long)bh * S + q0 + rbase + r) * S + key);
          pd = keep_elem(seed, idx, th) ? p * dscale : 0.f;
        }
        st_bf16(scr, kc_off(rbase + r, j * 16 + (lane & 15)), pd);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o_ = 1; o_ < 16; o_ <<= 1) rs[r] += __shfl_xor(rs[r], o_, 64);
      l[r] = l[r] * alpha[r] + rs[r];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[j][r] *= alpha[r];
    lds_fence();
    v8bf pa0 = frag_kc(scr, 0, 0, lane), pa1 = frag_kc(scr, 0, 1, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa0, frag_mc<64>(Vt + kc * 8192, j * 16, 0, lane), o[j], 0, 0, 0);
      o[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa1, frag_mc<64>(Vt + kc * 8192, j * 16, 1, lane), o[j], 0, 0, 0);
    }
    lds_fence();  // the scratch is rewritten by the next chunk
  }
  // finalize: O / l -> scratch (plain row-major [16][64]) -> 16-B global stores
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) st_bf16(scr, (rbase + r) * 128 + (j * 16 + (lane & 15)) * 2, o[j][r] / l[r]);
  if ((lane & 15) == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) lse[(long long)bh * S + q0 + rbase + r] = m[r] + __logf(l[r]);
  }
  lds_fence();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i;  // 128 chunks of 16 B: row c/8, chunk c%8
    const int row = c >> 3, ch = c & 7;
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(scr + row * 128 + ch * 16);
    *reinterpret_cast<v8bf*>(out + ((long long)b * S + q0 + row) * H + h * 64 + ch * 8) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Backward, S <= 128 (one workgroup holds a whole (b, h)).  LDS: Q, dO, K as MC tiles (S/64 x 8 KB
// each), dQ fp32 [S][64], D and LSE [S], per-wave scratch 2 x [32][32] bf16.
__global__ void __launch_bounds__(256) attn_bwd_kernel(const bf16_t* __restrict__ qkv, const bf16_t* __restrict__ o,
                                                       const bf16_t* __restrict__ dout, const float* __restrict__ lse,
                                                       const float* __restrict__ mask, bf16_t* __restrict__ dqkv,
                                                       int S, int nh, float scale, uint32_t th, float dscale,
                                                       uint32_t seed, int abl) {
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
  const int nc64 = S / 64;
  lds_char* Qt = smem;                        // MC [q][d]
  lds_char* dOt = Qt + S * 128;               // MC [q][d]
  lds_char* Kt = dOt + S * 128;               // MC [key][d]
  lds_float* dQs = reinterpret_cast<lds_float*>(Kt + S * 128);  // [S][64] fp32
  lds_float* Ds = dQs + S * 64;               // [S]
  lds_float* Ls = Ds + S;                     // [S]
  lds_float* Ms = Ls + S;                     // [S] key mask
  lds_char* scrP = reinterpret_cast<lds_char*>(Ms + S) + wave * 4096;  // [32 keys][32 q] MC-swizzled
  lds_char* scrS = scrP + 2048;
  {
    DenseMC<false> qs_{Qg, ld, 64, S};
    DenseMC<false> ds_{dOg, (long long)H, 64, S};
    DenseMC<false> kss{Kg, ld, 64, S};
    for (int c = 0; c < nc64; ++c) {
      stage_mc<64>(qs_, Qt + c * 8192, 0, c * 64, wave, lane);
      stage_mc<64>(ds_, dOt + c * 8192, 0, c * 64, wave, lane);
      stage_mc<64>(kss, Kt + c * 8192, 0, c * 64, wave, lane);
    }
  }
  // D[q] = sum_d dO[q, d] * O[q, d]  (two threads per row, 32 columns each), LSE, key mask, dQ = 0
  for (int i = tid; i < ((abl & 1) ? 0 : 2 * S); i += 256) {
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
  if (abl & 1)
    for (int i = tid; i < S; i += 256) Ds[i] = 0.f;
  for (int i = tid; i < S; i += 256) {
    Ls[i] = lse[(long long)bh * S + i];
    Ms[i] = mask ? mask[(long long)b * S + i] : 0.f;
  }
  for (int i = tid; i < S * 64; i += 256) dQs[i] = 0.f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int rbase = (lane >> 4) * 4;
  for (int kb = wave * 32; kb < S; kb += 128) {  // this wave's 32-key block(s)
    v8bf ka[2][2], va[2][2];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        ka[mi][ks] = gfrag(Kg, ld, kb + mi * 16, ks, lane);
        va[mi][ks] = gfrag(Vg, ld, kb + mi * 16, ks, lane);
      }
    f32x4 dk[2][4], dv[2][4];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j) dk[mi][j] = dv[mi][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int qc = 0; qc < S; qc += 32) {
      const int tq = qc >> 6, kq = (qc & 63) >> 5;  // 64-row MC tile and its 32-row half
      // sT[key][q] = K Q^T ; dPdT[key][q] = V dO^T
      f32x4 st[2][2], dpt[2][2];
#pragma unroll
      for (int ni = 0; ni < 2; ++ni) {
        v8bf qb0, qb1, db0, db1;
        if (abl & 8) {
          qb0 = ka[0][0]; qb1 = ka[0][1]; db0 = va[0][0]; db1 = va[0][1];
        } else {
          qb0 = gfrag(Qg, ld, qc + ni * 16, 0, lane); qb1 = gfrag(Qg, ld, qc + ni * 16, 1, lane);
          db0 = gfrag(dOg, (long long)H, qc + ni * 16, 0, lane); db1 = gfrag(dOg, (long long)H, qc + ni * 16, 1, lane);
        }
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          f32x4 z = f32x4{0.f, 0.f, 0.f, 0.f};
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[mi][0], qb0, z, 0, 0, 0);
          st[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[mi][1], qb1, z, 0, 0, 0);
          z = f32x4{0.f, 0.f, 0.f, 0.f};
          z = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[mi][0], db0, z, 0, 0, 0);
          dpt[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va[mi][1], db1, z, 0, 0, 0);
        }
      }
      // P^T, dropout, dS^T  (C layout: row = key, col = q)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const int qcol = ni * 16 + (lane & 15);
          const int q = qc + qcol;
          const float lq = Ls[q], dq = Ds[q];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int krow = mi * 16 + rbase + r;
            const int key = kb + krow;
            const float p = __expf(st[mi][ni][r] * scale + Ms[key] - lq);
            float pd = p, dp = dpt[mi][ni][r];
            if (th) {
              const bool kp = keep_elem(seed, (uint32_t)(((long long)bh * S + q) * S + key), th);
              pd = kp ? p * dscale : 0.f;
              dp = kp ? dp * dscale : 0.f;
            }
            st_bf16(scrP, mc32_off(krow, qcol), pd);
            st_bf16(scrS, mc32_off(krow, qcol), p * (dp - dq));
          }
        }
      lds_fence();
      // A fragments [key][q] (one 16-B chunk per lane) and the transposed dS [q][key] (tr reads)
      v8bf pa[2], sa[2], sta[2];
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) {
        const int krow = mi * 16 + (lane & 15), ch = lane >> 4;
        const int off = krow * 64 + ((ch ^ mc_swz<4>(krow)) << 4);
        pa[mi] = *reinterpret_cast<const lds_v8bf*>(scrP + off);
        sa[mi] = *reinterpret_cast<const lds_v8bf*>(scrS + off);
        sta[mi] = frag_mc<32>(scrS, mi * 16, 0, lane);  // X_A[q][key] = dS
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const v8bf dob = frag_mc<64>(dOt + tq * 8192, j * 16, kq, lane);  // X_B[d][q] = dO
        const v8bf qbm = frag_mc<64>(Qt + tq * 8192, j * 16, kq, lane);   // X_B[d][q] = Q
        const v8bf kbm = frag_mc<64>(Kt + (kb >> 6) * 8192, j * 16, (kb & 63) >> 5, lane);  // X_B[d][key] = K
#pragma unroll
        for (int mi = 0; mi < 2; ++mi) {
          dv[mi][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[mi], dob, dv[mi][j], 0, 0, 0);
          dk[mi][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa[mi], qbm, dk[mi][j], 0, 0, 0);
          f32x4 dq = f32x4{0.f, 0.f, 0.f, 0.f};
          dq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sta[mi], kbm, dq, 0, 0, 0);
          if (abl & 2) {
            asm volatile("" ::"v"(dq[0]), "v"(dq[1]), "v"(dq[2]), "v"(dq[3]));
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              __builtin_amdgcn_ds_faddf(dQs + (qc + mi * 16 + rbase + r) * 64 + j * 16 + (lane & 15), dq[r], 0, 0,
                                        false);
          }
        }
      }
      lds_fence();  // scratch reuse by the next chunk
    }
    // dK (scaled), dV -> dqkv
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long row = (long long)b * S + kb + mi * 16 + rbase + r;
          const int col = h * 64 + j * 16 + (lane & 15);
          if (abl & 4) {
            asm volatile("" ::"v"(dk[mi][j][r]), "v"(dv[mi][j][r]));
          } else {
            dqkv[row * ld + H + col] = f2bf(dk[mi][j][r] * scale);
            dqkv[row * ld + 2 * H + col] = f2bf(dv[mi][j][r]);
          }
        }
  }
  __syncthreads();
  for (int i = tid; i < S * 8; i += 256) {  // dQ: 8 x 16-B chunks per row
    const int q = i >> 3, ch = i & 7;
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = dQs[q * 64 + ch * 8 + k] * scale;
    store8_bf16(dqkv + ((long long)b * S + q) * ld + h * 64 + ch * 8, v);
  }
}

static uint32_t drop_th(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

int attn_fused_supported(int S, int dh, int backward) {
  if (dh != 64 || S % 64 != 0 || S <= 0) return 0;
  return backward ? (S <= 128) : (S <= 512);
}

static size_t fwd_lds(int S) { return (size_t)2 * S * 128 + 4 * 2048; }
static size_t bwd_lds(int S) { return (size_t)3 * S * 128 + (size_t)S * 64 * 4 + 3 * S * 4 + 4 * 4096; }

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
  dim3 grid(B * nh, S / 64);
  hipLaunchKernelGGL(attn_fwd_kernel<512>, grid, dim3(256), fwd_lds(S), st, qkv, mask, out, lse, S, nh, 0.125f, th,
                     ds, seed);
}

void attn_bwd(const bf16_t* qkv, const bf16_t* o, const bf16_t* dout, const float* lse, const float* mask,
              bf16_t* dqkv, int B, int S, int nh, float p, uint32_t seed, hipStream_t st) {
  static const int abl = getenv("DTG_ATTN_ABL") ? atoi(getenv("DTG_ATTN_ABL")) : 0;  // perf ablation only
  const uint32_t th = drop_th(p);
  const float ds = p > 0.f ? 1.f / (1.f - p) : 1.f;
  hipLaunchKernelGGL(attn_bwd_kernel, dim3(B * nh), dim3(256), bwd_lds(S), st, qkv, o, dout, lse, mask, dqkv, S, nh,
                     0.125f, th, ds, seed, abl);
}

}  // namespace dtg
