// BatchNorm statistics fused into the MFMA GEMM / implicit-GEMM epilogue (see BnEpi in kernels.h).
//
// ResNet's BN layers read every conv output once more just to reduce it per channel (forward: sum,
// sum of squares; backward: sum(dp), sum(dp*xhat)).  The epilogue already holds each output tile in
// registers, so it reduces its tile column-wise on the way out and adds one partial per column into
// a small slot buffer: the separate statistics pass (one full read of an M x C activation per BN)
// disappears.  In backward the ReLU mask is recomputed from the BN input and the saved per-channel
// statistics (gamma*xhat + beta > 0, the same fp32 expression the forward apply evaluates), so the
// BN output need not be re-read, and the stored gradient is already masked: the dx pass then reads
// dp and x only.
//
// Thread -> column mapping: epilogue_staged hands thread `tid` the 8-column group tid % (BN/8) in
// every pass (NTH is a multiple of BN/8), so each thread accumulates 8 columns in registers over all
// its rows; the block then reduces over the NTH/(BN/8) threads sharing a group through LDS.
#pragma once
#include "dtg/common.h"
#include "dtg/kernels.h"
#include "dtg/gemm_epi.cuh"
#include "dtg/mfma_gemm.cuh"

namespace dtg {
namespace gemm {

// BnEpi::old_sub2: does output row `row` = (n, h, w) carry a residual gradient (h and w even)?
__device__ __forceinline__ bool bn_row_has_old(const BnEpi& bn, int row) {
  if (!bn.old_sub2) return true;
  const uint32_t r = (uint32_t)row;
  const uint32_t n = (uint32_t)(((uint64_t)__umulhi(r, bn.hw_m) + r) >> bn.hw_l);
  const uint32_t hw = r - n * bn.old_hw;
  const uint32_t h = (uint32_t)(((uint64_t)__umulhi(hw, bn.w_m) + hw) >> bn.w_l);
  const uint32_t w = hw - h * bn.old_w;
  return ((h | w) & 1u) == 0;
}

struct RowId {  // identity row map (dense GEMMs)
  __device__ __forceinline__ int operator()(int m) const { return m; }
};

// pass height of the prefetching backward epilogue: the tallest of 128 / 64 / 32 rows whose fp32 staging
// fits the tile's LDS with at most 4 prefetched 8-column groups per thread
template <class C>
constexpr int bn_pf_rows() {
  for (int r = 128; r >= 32; r /= 2)
    if (r <= C::BM && C::BM % r == 0 && r * (C::BN + 4) * 4 <= C::LDS_BYTES && (r * (C::BN / 8)) % C::NTH == 0 &&
        r * (C::BN / 8) / C::NTH <= 4)
      return r;
  return 32;
}

// PF: the backward modes prefetch their per-element inputs (epilogue_staged_pf).  That pays where the
// epilogue's streaming dominates (short reductions, wide outputs: -6 to -11 % on ResNet's 1x1 dgrads) and
// costs where the extra prefetch registers lower the occupancy of a long main loop (+4 to +28 % on the 3x3
// dgrads), so the launcher chooses (gemm_bn_dispatch; profiles/r02_epi_pf).
// Per-thread column statistics of an epilogue (s: sum, q: raw moment, q2: the second BN's raw moment),
// streamed by epilogue_bn_stream and reduced once per workgroup by epilogue_bn_reduce.
struct BnAcc {
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q[8] = {0, 0, 0, 0, 0, 0, 0, 0}, q2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
};

template <class C, int MODE, class ROWMAP, bool PF = false>
__device__ __forceinline__ void epilogue_bn_stream(lds_char* smem, f32x4 (&acc)[4][4], int bm0, int bn0, int M, int N,
                                                   const Epi& e, const BnEpi& bn, const ROWMAP& rowmap, BnAcc& st) {
  // 4 = mode 3 + a second BN (x2); 5 = not a BN: the GEMM's own bias/activation/aux epilogue
  // (epi_store8_fast_act) plus the column sums of the stored output added into bn.part[N] (fp32) --
  // the bias gradient of the layer whose output gradient this GEMM produces, without a re-read
  static_assert(MODE >= 1 && MODE <= 5, "BN epilogue mode");
  constexpr int CPR = C::BN / 8, RW = C::NTH / CPR;
  static_assert(C::NTH % CPR == 0, "fixed column group per thread");
  static_assert((MODE == 4 ? 3 : 2) * RW * C::BN * 4 <= C::LDS_BYTES, "reduction scratch does not fit the LDS ring");
  const int tid = threadIdx.x, cg = tid % CPR, n0 = bn0 + cg * 8;
  // Backward modes accumulate the raw moment sum(d * x) and convert it once per column after the
  // block reduction: sum(d * xhat) = invstd * (sum(d * x) - mean * sum(d)).  Keeping mean/invstd out of
  // the row loop saves 16 VGPRs (32 in mode 4), which is what puts the 128x128 backward epilogues
  // under the 128-VGPR line of 4 workgroups per CU.
  float (&s)[8] = st.s;
  float (&q)[8] = st.q;
  float sc[8], sf[8];
  // mode 3 with a second BN on the same gradient (x2: the projection shortcut's BN input): sum(dp*x2)
  float (&q2)[8] = st.q2;
  constexpr bool two = MODE == 4;  // a separate instantiation: mode 3 keeps its register budget
  if constexpr (MODE == 2) {  // the relu mask is recomputed from x: gamma*xhat + beta > 0
    if (n0 < N) {
      float mu[8], is[8], g[8], b[8];
      load8_f32(bn.mean + n0, mu);
      load8_f32(bn.invstd + n0, is);
      load8_f32(bn.gamma + n0, g);
      load8_f32(bn.beta + n0, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sc[k] = g[k] * is[k];          // = bn_finalize's coef (scale)
        sf[k] = b[k] - mu[k] * sc[k];  // = bn_finalize's coef (shift)
      }
    }
  }
  if constexpr (MODE == 1 || MODE == 5) {
    epilogue_staged<C>(smem, acc, bm0, bn0, M, N, [&](int m, int n, float (&v)[8]) {
      const int row = rowmap(m);
      if constexpr (MODE == 5) {
        epi_store8_fast_act(e, row, n, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += bf2f(f2bf(v[k]));  // sum of what was stored
      } else {
        epi_store8_fast(e, row, n, v);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float r = bf2f(f2bf(v[k]));  // statistics of what the apply pass will read
          s[k] += r;
          q[k] += r * r;
        }
      }
    });
  } else if constexpr (!PF) {
    epilogue_staged<C>(smem, acc, bm0, bn0, M, N, [&](int m, int n, float (&v)[8]) {
      const int row = rowmap(m);
      const long long off = (long long)row * e.ldc + n;
      float xv[8];
      load8_bf16(bn.x + off, xv);
      if constexpr (MODE == 2) {  // the relu mask is recomputed from x
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = fmaf(xv[k], sc[k], sf[k]) > 0.f ? v[k] * e.alpha : 0.f;
          v[k] = d;
          s[k] += d;
          q[k] += d * xv[k];
        }
      } else {
        float mk[8], old[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (bn.maskbits) {
          const uint32_t byte = bn.maskbits[(long long)row * (N >> 3) + (n >> 3)];
#pragma unroll
          for (int k = 0; k < 8; ++k) mk[k] = (float)((byte >> k) & 1u);
        } else {
          load8_bf16(bn.mask + off, mk);
        }
        if (e.beta != 0.f && bn_row_has_old(bn, row)) load8_bf16((const bf16_t*)e.C + off, old);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = mk[k] > 0.f ? fmaf(v[k], e.alpha, e.beta * old[k]) : 0.f;
          v[k] = d;
          s[k] += d;
          q[k] += d * xv[k];
        }
        if constexpr (two) {
          float x2v[8];
          load8_bf16(bn.x2 + off, x2v);
#pragma unroll
          for (int k = 0; k < 8; ++k) q2[k] += v[k] * x2v[k];
        }
      }
      store8_bf16((bf16_t*)e.C + off, v);
    });
  } else {
    // backward modes read x (+ mask, residual gradient, x2) per element: prefetched a pass ahead of the
    // accumulator staging (epilogue_staged_pf), held as raw 16-B vectors until the group is finished
    constexpr int R = bn_pf_rows<C>();
    constexpr int GPT = R * CPR / C::NTH;
    uint4 px[GPT], po[GPT], px2[GPT];
    uint32_t pm[GPT];
    bool ho[GPT];
    const bool has_old = MODE != 2 && e.beta != 0.f;
    const bool bits = MODE != 2 && bn.maskbits != nullptr;
    auto pre = [&](int j, int m, int n, bool ok) {
      if (!ok) return;
      const int row = rowmap(m);
      const long long off = (long long)row * e.ldc + n;
      px[j] = *reinterpret_cast<const uint4*>(bn.x + off);
      if constexpr (MODE != 2) {
        if (bits) pm[j] = bn.maskbits[(long long)row * (N >> 3) + (n >> 3)];
        ho[j] = has_old && bn_row_has_old(bn, row);
        if (ho[j]) po[j] = *reinterpret_cast<const uint4*>((const bf16_t*)e.C + off);
        if constexpr (two) px2[j] = *reinterpret_cast<const uint4*>(bn.x2 + off);
      }
    };
    auto op = [&](int j, int m, int n, float (&v)[8]) {
      const int row = rowmap(m);
      const long long off = (long long)row * e.ldc + n;
      float xv[8];
      unpack8_bf16(px[j], xv);
      if constexpr (MODE == 2) {  // the relu mask is recomputed from x
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = fmaf(xv[k], sc[k], sf[k]) > 0.f ? v[k] * e.alpha : 0.f;
          v[k] = d;
          s[k] += d;
          q[k] += d * xv[k];
        }
      } else {
        float mk[8], old[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (bits) {
#pragma unroll
          for (int k = 0; k < 8; ++k) mk[k] = (float)((pm[j] >> k) & 1u);
        } else {
          load8_bf16(bn.mask + off, mk);
        }
        if (ho[j]) unpack8_bf16(po[j], old);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float d = mk[k] > 0.f ? fmaf(v[k], e.alpha, e.beta * old[k]) : 0.f;
          v[k] = d;
          s[k] += d;
          q[k] += d * xv[k];
        }
        if constexpr (two) {
          float x2v[8];
          unpack8_bf16(px2[j], x2v);
#pragma unroll
          for (int k = 0; k < 8; ++k) q2[k] += v[k] * x2v[k];
        }
      }
      store8_bf16((bf16_t*)e.C + off, v);
    };
    epilogue_staged_pf<C, R>(smem, acc, bm0, bn0, M, N, pre, op);
  }
}

// Block reduction of the BnAcc column statistics + one atomic add per column into the partial slot
// slot_id % kBnStatSlots (mode 5: straight into bn.part[N]).  The LDS ring must be free (every
// epilogue_bn_stream ends with a barrier).
template <class C, int MODE>
__device__ __forceinline__ void epilogue_bn_reduce(lds_char* smem, int bn0, int N, const BnEpi& bn, int slot_id,
                                                   const BnAcc& st) {
  constexpr int CPR = C::BN / 8, RW = C::NTH / CPR;
  constexpr bool two = MODE == 4;
  const int tid = threadIdx.x, cg = tid % CPR;
  const float (&s)[8] = st.s;
  const float (&q)[8] = st.q;
  const float (&q2)[8] = st.q2;
  const int tile_id = slot_id;
  lds_float* red = reinterpret_cast<lds_float*>(smem);
  const int r = tid / CPR;
  if constexpr (MODE == 5) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[r * C::BN + cg * 8 + k] = s[k];
    __syncthreads();
    for (int c = tid; c < C::BN; c += C::NTH) {
      if (bn0 + c < N) {
        float ts = 0.f;
#pragma unroll 8
        for (int j = 0; j < RW; ++j) ts += red[j * C::BN + c];
        atomicAdd(bn.part + bn0 + c, ts);
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[r * C::BN + cg * 8 + k] = s[k];
    red[(RW + r) * C::BN + cg * 8 + k] = q[k];
    if constexpr (two) red[(2 * RW + r) * C::BN + cg * 8 + k] = q2[k];
  }
  __syncthreads();
  const long long slot = (long long)(tile_id % kBnStatSlots) * 2 * N;
  float* part = bn.part + slot;
  for (int c = tid; c < C::BN; c += C::NTH) {
    if (bn0 + c < N) {
      float ts = 0.f, tq = 0.f;
#pragma unroll 8
      for (int j = 0; j < RW; ++j) {
        ts += red[j * C::BN + c];
        tq += red[(RW + j) * C::BN + c];
      }
      if constexpr (MODE >= 2) tq = bn.invstd[bn0 + c] * (tq - bn.mean[bn0 + c] * ts);  // raw -> centred
      atomicAdd(part + bn0 + c, ts);
      atomicAdd(part + N + bn0 + c, tq);
      if constexpr (two) {  // the second BN's partials: (sum dp, sum dp*xhat2), same finalize layout
        float tq2 = 0.f;
#pragma unroll 8
        for (int j = 0; j < RW; ++j) tq2 += red[(2 * RW + j) * C::BN + c];
        tq2 = bn.invstd2[bn0 + c] * (tq2 - bn.mean2[bn0 + c] * ts);
        atomicAdd(bn.part2 + slot + bn0 + c, ts);
        atomicAdd(bn.part2 + slot + N + bn0 + c, tq2);
      }
    }
  }
}

// stream + reduce for one tile (every BN-epilogue GEMM / conv workgroup owns exactly one output tile)
template <class C, int MODE, class ROWMAP, bool PF = false>
__device__ __forceinline__ void epilogue_bn(lds_char* smem, f32x4 (&acc)[4][4], int bm0, int bn0, int M, int N,
                                            const Epi& e, const BnEpi& bn, int tile_id, const ROWMAP& rowmap) {
  BnAcc st;
  epilogue_bn_stream<C, MODE, ROWMAP, PF>(smem, acc, bm0, bn0, M, N, e, bn, rowmap, st);
  epilogue_bn_reduce<C, MODE>(smem, bn0, N, bn, tile_id, st);
}

}  // namespace gemm
}  // namespace dtg
