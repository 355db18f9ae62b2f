// Shared GEMM epilogue: C = act(alpha * acc + beta * C + bias), fp32 or bf16 output, 8 columns
// at a time (16-byte vectors when aligned).  Used by gemm.hip and conv.hip.
#pragma once
#include "dtg/common.h"

namespace dtg {

struct Epi {
  void* C;
  long long ldc;
  int c_bf16;
  float alpha, beta;
  const float* bias;  // per column (N), may be null
  int act;            // 0 none, 1 relu, 2 gelu(tanh), 3 tanh (BERT pooler)
  void* aux = nullptr;  // bf16 [M, ldc] side buffer (see aux_mode)
  // 0 none; 1 store the pre-activation to aux; 2 multiply by act'(aux) (act backward from the saved
  // pre-activation); 3 store act'(pre-activation) to aux (forward: the derivative while the
  // activation's exp is in registers); 4 multiply by aux (act backward from the saved derivative)
  int aux_mode = 0;
};

// GELU (tanh form) through its sigmoid identity 0.5 * (1 + tanh(u)) = sigmoid(2u): one v_exp_f32 and
// one v_rcp_f32 instead of libm tanhf (range reduction and branches), which made the GELU GEMM
// epilogues issue-bound.  exp overflow is benign: sigmoid -> 0 or 1.
__device__ __forceinline__ float gelu_sig(float x) {  // sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x * x, x);
  return __builtin_amdgcn_rcpf(1.f + __expf(-u2));
}

// tanh(x) = 2 sigmoid(2x) - 1: one v_exp_f32 + one v_rcp_f32 (saturates cleanly to +-1)
__device__ __forceinline__ float tanh_fast(float x) {
  return fmaf(2.f, __builtin_amdgcn_rcpf(1.f + __expf(-2.f * x)), -1.f);
}

__device__ __forceinline__ float apply_act(float v, int act) {
  if (act == 1) return fmaxf(v, 0.f);
  if (act == 2) return v * gelu_sig(v);
  if (act == 3) return tanh_fast(v);
  return v;
}

// d act(x) / dx;  GELU: s + x * (1 - t^2)/2 * u' with t = 2s - 1, (1 - t^2) = 4 s (1 - s)
__device__ __forceinline__ float act_grad(float x, int act) {
  if (act == 1) return x > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float s = gelu_sig(x);
    const float du = 0.7978845608028654f * fmaf(3.f * 0.044715f * x, x, 1.f);
    return fmaf(2.f * x * s * (1.f - s), du, s);
  }
  if (act == 3) {
    const float t = tanh_fast(x);
    return fmaf(-t, t, 1.f);
  }
  return 1.f;
}

// finish 8 consecutive columns [n, n+8) of row m (n < N; the tail is masked element-wise)
__device__ __forceinline__ void epi_store8(const Epi& e, int N, int m, int n, float (&v)[8]) {
  const long long off = (long long)m * e.ldc + n;
  const int cnt = N - n < 8 ? N - n : 8;
  const bool vec = cnt == 8 && ((e.ldc & 7) == 0);
  float old[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (e.beta != 0.f) {
    if (vec) {
      if (e.c_bf16) load8_bf16((const bf16_t*)e.C + off, old);
      else load8_f32((const float*)e.C + off, old);
    } else {
      for (int k = 0; k < cnt; ++k)
        old[k] = e.c_bf16 ? bf2f(((const bf16_t*)e.C)[off + k]) : ((const float*)e.C)[off + k];
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    float x = v[k] * e.alpha + e.beta * old[k];
    if (e.bias && k < cnt) x += e.bias[n + k];
    v[k] = x;
  }
  if (e.aux_mode == 1 || e.aux_mode == 3) {
    float t[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) t[k] = e.aux_mode == 3 ? act_grad(v[k], e.act) : v[k];
    if (vec) store8_bf16((bf16_t*)e.aux + off, t);
    else
      for (int k = 0; k < cnt; ++k) ((bf16_t*)e.aux)[off + k] = f2bf(t[k]);
  }
  if (e.aux_mode == 2 || e.aux_mode == 4) {
    float pre[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (vec) load8_bf16((const bf16_t*)e.aux + off, pre);
    else
      for (int k = 0; k < cnt; ++k) pre[k] = bf2f(((const bf16_t*)e.aux)[off + k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= e.aux_mode == 4 ? pre[k] : act_grad(pre[k], e.act);
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = apply_act(v[k], e.act);
  }
  if (vec) {
    if (e.c_bf16) store8_bf16((bf16_t*)e.C + off, v);
    else store8_f32((float*)e.C + off, v);
  } else {
    for (int k = 0; k < cnt; ++k) {
      if (e.c_bf16) ((bf16_t*)e.C)[off + k] = f2bf(v[k]);
      else ((float*)e.C)[off + k] = v[k];
    }
  }
}

// Fast path of epi_store8 for the common case: bf16 output, 8 full aligned columns, no bias /
// activation / aux; C = alpha*acc (+ beta*C).  The generic version's per-group runtime switches cost
// more VALU/SALU than the data movement in the memory-bound GEMMs (issue-bound epilogue, see
// profiles/r01_pmc).
__device__ __forceinline__ void epi_store8_fast(const Epi& e, int m, int n, float (&v)[8]) {
  bf16_t* p = (bf16_t*)e.C + (long long)m * e.ldc + n;
  if (e.beta != 0.f) {
    float old[8];
    load8_bf16(p, old);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], e.alpha, e.beta * old[k]);
  } else if (e.alpha != 1.f) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= e.alpha;
  }
  store8_bf16(p, v);
}

// epi_store8_fast plus bias / activation / aux (bf16, full aligned groups): the switches are
// wave-uniform branches around whole 8-column loops, not per-element tests as in epi_store8.
// PB: the bias of these 8 columns is already in registers (pb) -- a thread of the staged epilogue keeps one
// column group for the whole tile, so the caller loads it once instead of once per group: loaded here, every
// group waited for its own bias load (BERT FFN1 forward 155 -> 178 us with the bias, tools/epi_decomp.py)
template <bool PB = false>
__device__ __forceinline__ void epi_store8_fast_act(const Epi& e, int m, int n, float (&v)[8],
                                                    const float* pb = nullptr) {
  const long long off = (long long)m * e.ldc + n;
  bf16_t* p = (bf16_t*)e.C + off;
  if (e.beta != 0.f) {
    float old[8];
    load8_bf16(p, old);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], e.alpha, e.beta * old[k]);
  } else if (e.alpha != 1.f) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= e.alpha;
  }
  if (e.bias) {
    float b[8];
    if constexpr (PB) {
#pragma unroll
      for (int k = 0; k < 8; ++k) b[k] = pb[k];
    } else {
      load8_f32(e.bias + n, b);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += b[k];
  }
  if (e.aux_mode == 1) store8_bf16((bf16_t*)e.aux + off, v);
  if (e.aux_mode == 2 || e.aux_mode == 4) {
    float pre[8];
    load8_bf16_nt((const bf16_t*)e.aux + off, pre);  // saved in forward, last use
    if (e.aux_mode == 4) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= pre[k];
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= act_grad(pre[k], e.act);
    }
  } else if (e.aux_mode == 3 && e.act == 2) {  // GELU and its derivative from one sigmoid
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x = v[k], sg = gelu_sig(x);
      const float du = 0.7978845608028654f * fmaf(3.f * 0.044715f * x, x, 1.f);
      d[k] = fmaf(2.f * x * sg * (1.f - sg), du, sg);
      v[k] = x * sg;
    }
    // GELU'(pre) is read again only in the backward pass: a non-temporal store keeps it from evicting
    // the activation the next GEMM reads at once from the Infinity Cache
    store8_bf16_nt((bf16_t*)e.aux + off, d);
  } else if (e.act == 1) {
    if (e.aux_mode == 3) {
      float d[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) d[k] = v[k] > 0.f ? 1.f : 0.f;
      store8_bf16((bf16_t*)e.aux + off, d);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
  } else if (e.act == 2) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= gelu_sig(v[k]);
  } else if (e.act == 3) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = tanh_fast(v[k]);
  }
  store8_bf16(p, v);
}

// split-K reduction of fp32 slabs [split][M][N] + the epilogue (gemm.hip)
void gemm_splitk_reduce(const float* ws, int split_k, int M, int N, const Epi& e, hipStream_t st);

}  // namespace dtg
