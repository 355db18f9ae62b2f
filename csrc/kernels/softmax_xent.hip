// Fused softmax + cross-entropy forward AND backward in one pass over the logits.
//   loss[r]      = logsumexp(x[r,:]) - x[r, label[r]]
//   dlogits[r,j] = (softmax(x[r,:])_j - [j == label[r]]) * scale
// Training always needs both, so the gradient is produced while the row is hot (one read of the
// logits for max/sum, one read + one write for the gradient); the autograd wrapper only rescales
// it if the incoming grad_output is not 1.  label < 0 is ignored (loss 0, grad 0): used by the
// BERT MLM head.  One 256-thread block (4 waves) per row; online max/sum in fp32.
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

template <typename T>
__global__ void __launch_bounds__(256) softmax_xent_kernel(const T* __restrict__ x, const long long* __restrict__ label,
                                                           int V, float scale, float* __restrict__ loss,
                                                           T* __restrict__ dx, float* __restrict__ lse_out) {
  __shared__ float red[2][4];
  const int row = blockIdx.x;
  const T* xr = x + (long long)row * V;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // online max / sum-exp per lane
  float m = -INFINITY, s = 0.f;
  for (int j = tid; j < V; j += 256) {
    const float v = ld<T>(xr, j);
    if (v > m) { s = s * __expf(m - v) + 1.f; m = v; }
    else s += __expf(v - m);
  }
  // combine lanes: (m, s) pairs
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (m == -INFINITY ? 0.f : s * __expf(m - mn)) + (mo == -INFINITY ? 0.f : so * __expf(mo - mn));
    m = mn;
  }
  if (lane == 0) { red[0][wid] = m; red[1][wid] = s; }
  __syncthreads();
  float M = red[0][0];
#pragma unroll
  for (int w = 1; w < 4; ++w) M = fmaxf(M, red[0][w]);
  float S = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) S += red[1][w] * __expf(red[0][w] - M);
  const float lse = M + __logf(S);
  const long long lab = label[row];
  if (tid == 0) {
    loss[row] = lab >= 0 ? lse - ld<T>(xr, lab) : 0.f;
    if (lse_out) lse_out[row] = lse;
  }
  if (dx) {
    T* dr = dx + (long long)row * V;
    if (lab < 0) {
      for (int j = tid; j < V; j += 256) st<T>(dr, j, 0.f);
    } else {
      for (int j = tid; j < V; j += 256) {
        const float p = __expf(ld<T>(xr, j) - lse);
        st<T>(dr, j, (p - (j == lab ? 1.f : 0.f)) * scale);
      }
    }
  }
}

void softmax_xent(const void* x, int x_bf16, const long long* label, long long B, int V, float scale, float* loss,
                  void* dx, float* lse, hipStream_t st) {
  if (x_bf16)
    softmax_xent_kernel<bf16_t><<<(unsigned)B, 256, 0, st>>>((const bf16_t*)x, label, V, scale, loss, (bf16_t*)dx, lse);
  else
    softmax_xent_kernel<float><<<(unsigned)B, 256, 0, st>>>((const float*)x, label, V, scale, loss, (float*)dx, lse);
}

}  // namespace dtg
