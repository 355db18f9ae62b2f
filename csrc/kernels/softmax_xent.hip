// Softmax cross-entropy over the rows of a [B, V] logit matrix (ResNet's 1000-way classifier, BERT's
// 30528-way masked-LM decoder).
//   forward   loss[r] = logsumexp(x[r,:]) - x[r, label[r]],  lse[r] saved
//   backward  dlogits[r,j] = (exp(x[r,j] - lse[r]) - [j == label[r]]) * scale * g
// label < 0 is ignored (loss 0, grad 0): used by the BERT MLM head.
//
// The backward reads the upstream gradient g from DEVICE memory (a 0-d tensor), so the autograd node
// needs no host read of it and no separate rescale pass over the [B, V] gradient (which for the MLM
// head is 312 MB at 5120 x 30528 bf16).  The forward can still emit the gradient for a known g = 1
// (want_grad) in the same pass.
// One 256-thread block per row; bf16 rows with V % 8 == 0 move as 16-byte vectors (8 logits per
// lane-access), other rows element-wise.  Online max / sum in fp32, per-lane then across the block.
#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long long i);
template <>
__device__ __forceinline__ float ld<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }

template <typename T>
__device__ __forceinline__ void st(T* p, long long i, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, long long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void st<bf16_t>(bf16_t* p, long long i, float v) { p[i] = f2bf(v); }

// online (max, sum) update with one value / with 8 values
__device__ __forceinline__ void ms_add(float& m, float& s, float v) {
  if (v > m) {
    s = s * __expf(m - v) + 1.f;
    m = v;
  } else {
    s += __expf(v - m);
  }
}
__device__ __forceinline__ void ms_add8(float& m, float& s, const float (&v)[8]) {
  float mx = v[0];
#pragma unroll
  for (int k = 1; k < 8; ++k) mx = fmaxf(mx, v[k]);
  if (mx == -INFINITY) return;  // all eight masked out
  if (mx > m) {
    s = (m == -INFINITY ? 0.f : s * __expf(m - mx));
    m = mx;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) s += __expf(v[k] - m);
}

// block-wide logsumexp of the per-thread (m, s) pairs (256 threads = 4 waves)
__device__ __forceinline__ float block_lse(float m, float s, float (*red)[4]) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  if (lane == 0) {
    red[0][wid] = m;
    red[1][wid] = s;
  }
  __syncthreads();
  float M = red[0][0];
#pragma unroll
  for (int w = 1; w < 4; ++w) M = fmaxf(M, red[0][w]);
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) S += red[1][w] * __expf(red[0][w] - M);
  return M + __logf(S);
}

// VEC: bf16 rows with V % 8 == 0 (16-B aligned rows), 8 logits per access
template <typename T, bool VEC>
__global__ void __launch_bounds__(256) softmax_xent_kernel(const T* __restrict__ x, const long long* __restrict__ label,
                                                           int V, float scale, float* __restrict__ loss,
                                                           T* __restrict__ dx, float* __restrict__ lse_out) {
  __shared__ float red[2][4];
  const int row = blockIdx.x;
  const T* xr = x + (long long)row * V;
  const int tid = threadIdx.x;
  float m = -INFINITY, s = 0.f;
  if constexpr (VEC) {
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(xr);
    for (int c = tid; c < (V >> 3); c += 256) {
      float v[8];
      load8_bf16(xb + c * 8, v);
      ms_add8(m, s, v);
    }
  } else {
    for (int j = tid; j < V; j += 256) ms_add(m, s, ld<T>(xr, j));
  }
  const float lse = block_lse(m, s, red);
  const long long lab = label[row];
  if (tid == 0) {
    loss[row] = lab >= 0 ? lse - ld<T>(xr, lab) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (!dx) return;
  T* dr = dx + (long long)row * V;
  if constexpr (VEC) {
    bf16_t* db = reinterpret_cast<bf16_t*>(dr);
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(xr);
    for (int c = tid; c < (V >> 3); c += 256) {
      float v[8];
      load8_bf16(xb + c * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        v[k] = lab < 0 ? 0.f : (__expf(v[k] - lse) - (c * 8 + k == lab ? 1.f : 0.f)) * scale;
      store8_bf16(db + c * 8, v);
    }
  } else {
    for (int j = tid; j < V; j += 256)
      st<T>(dr, j, lab < 0 ? 0.f : (__expf(ld<T>(xr, j) - lse) - (j == lab ? 1.f : 0.f)) * scale);
  }
}

// backward from the saved lse: dx = (softmax - onehot) * scale * (*g)
template <typename T, bool VEC>
__global__ void __launch_bounds__(256) softmax_xent_bwd_kernel(const T* __restrict__ x,
                                                               const long long* __restrict__ label,
                                                               const float* __restrict__ lse, int V, float scale,
                                                               const float* __restrict__ g, T* __restrict__ dx) {
  const int row = blockIdx.x;
  const long long lab = label[row];
  const float sc = scale * (g ? *g : 1.f), l = lse[row];
  const T* xr = x + (long long)row * V;
  T* dr = dx + (long long)row * V;
  if constexpr (VEC) {
    const bf16_t* xb = reinterpret_cast<const bf16_t*>(xr);
    bf16_t* db = reinterpret_cast<bf16_t*>(dr);
    for (int c = threadIdx.x; c < (V >> 3); c += 256) {
      float v[8];
      load8_bf16(xb + c * 8, v);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = lab < 0 ? 0.f : (__expf(v[k] - l) - (c * 8 + k == lab ? 1.f : 0.f)) * sc;
      store8_bf16(db + c * 8, v);
    }
  } else {
    for (int j = threadIdx.x; j < V; j += 256)
      st<T>(dr, j, lab < 0 ? 0.f : (__expf(ld<T>(xr, j) - l) - (j == lab ? 1.f : 0.f)) * sc);
  }
}

static bool vec_ok(const void* x, int x_bf16, int V, const void* dx) {
  return x_bf16 && (V % 8) == 0 && ((uintptr_t)x % 16) == 0 && ((uintptr_t)dx % 16) == 0;
}

void softmax_xent(const void* x, int x_bf16, const long long* label, long long B, int V, float scale, float* loss,
                  void* dx, float* lse, hipStream_t st) {
  if (vec_ok(x, x_bf16, V, dx))
    softmax_xent_kernel<bf16_t, true><<<(unsigned)B, 256, 0, st>>>((const bf16_t*)x, label, V, scale, loss, (bf16_t*)dx,
                                                                  lse);
  else if (x_bf16)
    softmax_xent_kernel<bf16_t, false><<<(unsigned)B, 256, 0, st>>>((const bf16_t*)x, label, V, scale, loss,
                                                                   (bf16_t*)dx, lse);
  else
    softmax_xent_kernel<float, false><<<(unsigned)B, 256, 0, st>>>((const float*)x, label, V, scale, loss, (float*)dx,
                                                                  lse);
  DTG_LAUNCH_CHECK();
}

void softmax_xent_bwd(const void* x, int x_bf16, const long long* label, const float* lse, long long B, int V,
                      float scale, const float* g, void* dx, hipStream_t st) {
  if (vec_ok(x, x_bf16, V, dx))
    softmax_xent_bwd_kernel<bf16_t, true><<<(unsigned)B, 256, 0, st>>>((const bf16_t*)x, label, lse, V, scale, g,
                                                                      (bf16_t*)dx);
  else if (x_bf16)
    softmax_xent_bwd_kernel<bf16_t, false><<<(unsigned)B, 256, 0, st>>>((const bf16_t*)x, label, lse, V, scale, g,
                                                                       (bf16_t*)dx);
  else
    softmax_xent_bwd_kernel<float, false><<<(unsigned)B, 256, 0, st>>>((const float*)x, label, lse, V, scale, g,
                                                                      (float*)dx);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
