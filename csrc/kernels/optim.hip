// Fused optimizer applies over FLAT parameter buffers (one launch updates every parameter of the
// model).  dtg keeps parameters, gradients and optimizer state in single contiguous HBM buffers
// (parallel/flat.py), so the "multi-tensor" apply of other frameworks is a plain vectorised stream:
// 8 elements / lane / iteration, 16-byte loads for bf16, grid capped at 2048 WGs (grid-stride).
//
// Semantics mirror the TF-1.x apply kernels the reference exercises:
//   ApplyGradientDescent  w -= lr*g                       (Hogwild/Hogwild.py:44, ADAG/ADAG.py:62-63)
//   ApplyAdagrad          acc += g^2 ; w -= lr*g/sqrt(acc) (DOWNPOUR/DOWNPOUR.py:57, :92)
// plus momentum-SGD (ResNet-50) and AdamW (BERT) for the north-star models.
//
// Every apply optionally (a) scales the incoming gradient (1/world for all-reduce averaging),
// (b) writes a bf16 mirror of the fp32 master weights (the compute copy the model reads), and
// (c) zeroes the gradient buffer in the same pass (saves a memset before the next backward).
// lr / step live on the device so the apply can be captured in a hipGraph and replayed.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include <type_traits>

namespace dtg {

template <bool GBF16>
__device__ __forceinline__ void load_grad8(const void* g, long long i, float (&o)[8]) {
  if constexpr (GBF16) load8_bf16(reinterpret_cast<const bf16_t*>(g) + i, o);
  else load8_f32(reinterpret_cast<const float*>(g) + i, o);
}

template <bool GBF16>
__device__ __forceinline__ void zero_grad8(void* g, long long i) {
  if constexpr (GBF16) *reinterpret_cast<uint4*>(reinterpret_cast<bf16_t*>(g) + i) = make_uint4(0, 0, 0, 0);
  else {
    float* p = reinterpret_cast<float*>(g) + i;
    *reinterpret_cast<float4*>(p) = make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(p + 4) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <bool GBF16>
__device__ __forceinline__ float load_grad1(const void* g, long long i) {
  if constexpr (GBF16) return bf2f(reinterpret_cast<const bf16_t*>(g)[i]);
  else return reinterpret_cast<const float*>(g)[i];
}

template <bool GBF16>
__device__ __forceinline__ void zero_grad1(void* g, long long i) {
  if constexpr (GBF16) reinterpret_cast<bf16_t*>(g)[i] = 0;
  else reinterpret_cast<float*>(g)[i] = 0.f;
}

// ---------------------------------------------------------------------------------------------
// Generic driver: OP is a functor with  void operator()(float& w, float g, float& st0, float& st1)
// applied per element; the vector path handles 8 elements, the tail path the remainder.
// ---------------------------------------------------------------------------------------------
struct SgdOp {
  float lr, wd;
  __device__ __forceinline__ void operator()(float& w, float g, float&, float&) const { w -= lr * (g + wd * w); }
};

struct MomentumOp {
  float lr, mu, wd;
  int nesterov;
  __device__ __forceinline__ void operator()(float& w, float g, float& m, float&) const {
    g += wd * w;
    m = mu * m + g;
    w -= lr * (nesterov ? g + mu * m : m);
  }
};

struct AdagradOp {
  float lr, eps;
  __device__ __forceinline__ void operator()(float& w, float g, float& acc, float&) const {
    acc += g * g;
    w -= lr * g * __frsqrt_rn(acc + eps);
  }
};

struct AdamOp {
  float lr, b1, b2, eps, wd, bc1, bc2;  // bc = 1/(1-beta^t)
  __device__ __forceinline__ void operator()(float& w, float g, float& m, float& v) const {
    m = b1 * m + (1.f - b1) * g;
    v = b2 * v + (1.f - b2) * g * g;
    const float mh = m * bc1, vh = v * bc2;
    w -= lr * (mh / (sqrtf(vh) + eps) + wd * w);
  }
};

// Device-resident hyper-parameters: the kernels below read lr (and the Adam step) through a
// pointer so a captured graph picks up a new schedule value each replay.
template <class OP, bool GBF16, bool MIRROR, int NST>
__global__ void __launch_bounds__(256) apply_kernel_dev(float* __restrict__ w, bf16_t* __restrict__ mirror,
                                                        void* __restrict__ grad, float* __restrict__ s0,
                                                        float* __restrict__ s1, long long n, float gscale,
                                                        int zero_grad, OP op, const float* __restrict__ hyper) {
  // hyper[0] = lr, hyper[1] = step (Adam only)
  OP o = op;
  o.lr = hyper[0];
  if constexpr (std::is_same<OP, AdamOp>::value) {
    const float t = hyper[1];
    o.bc1 = 1.f / (1.f - __powf(op.b1, t));
    o.bc2 = 1.f / (1.f - __powf(op.b2, t));
  }
  const long long nvec = n >> 3;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const long long i = v << 3;
    float wv[8], gv[8], a[8], b[8];
    load8_f32(w + i, wv);
    load_grad8<GBF16>(grad, i, gv);
    if constexpr (NST >= 1) load8_f32(s0 + i, a);
    if constexpr (NST >= 2) load8_f32(s1 + i, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) o(wv[k], gv[k] * gscale, a[k], b[k]);
    store8_f32(w + i, wv);
    if constexpr (NST >= 1) store8_f32(s0 + i, a);
    if constexpr (NST >= 2) store8_f32(s1 + i, b);
    if constexpr (MIRROR) store8_bf16(mirror + i, wv);
    if (zero_grad) zero_grad8<GBF16>(grad, i);
  }
  if (blockIdx.x == 0) {
    for (long long i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) {
      float wv = w[i], a = 0.f, b = 0.f;
      if constexpr (NST >= 1) a = s0[i];
      if constexpr (NST >= 2) b = s1[i];
      o(wv, load_grad1<GBF16>(grad, i) * gscale, a, b);
      w[i] = wv;
      if constexpr (NST >= 1) s0[i] = a;
      if constexpr (NST >= 2) s1[i] = b;
      if constexpr (MIRROR) mirror[i] = f2bf(wv);
      if (zero_grad) zero_grad1<GBF16>(grad, i);
    }
  }
}

template <class OP, int NST>
static void launch_apply_dev(const OP& op, float* w, bf16_t* mirror, void* grad, int grad_bf16, float* s0,
                             float* s1, long long n, float gscale, int zero_grad, const float* hyper,
                             hipStream_t st) {
  const int block = 256;
  const int grid = grid_for((n >> 3) + 1, block, 2048);
#define DTG_L(G, M)                                                                                              \
  do {                                                                                                          \
    apply_kernel_dev<OP, G, M, NST><<<grid, block, 0, st>>>(w, mirror, grad, s0, s1, n, gscale, zero_grad, op, hyper); \
    DTG_LAUNCH_CHECK();                                                                                          \
  } while (0)
  if (grad_bf16) { if (mirror) DTG_L(true, true); else DTG_L(true, false); }
  else { if (mirror) DTG_L(false, true); else DTG_L(false, false); }
#undef DTG_L
}

void sgd_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, long long n, const float* hyper, float wd,
               float gscale, int zero_grad, hipStream_t st) {
  launch_apply_dev<SgdOp, 0>(SgdOp{0.f, wd}, w, mirror, grad, grad_bf16, nullptr, nullptr, n, gscale, zero_grad,
                             hyper, st);
}

void momentum_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* mom, long long n,
                    const float* hyper, float mu, float wd, int nesterov, float gscale, int zero_grad,
                    hipStream_t st) {
  launch_apply_dev<MomentumOp, 1>(MomentumOp{0.f, mu, wd, nesterov}, w, mirror, grad, grad_bf16, mom, nullptr, n,
                                  gscale, zero_grad, hyper, st);
}

void adagrad_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* acc, long long n,
                   const float* hyper, float eps, float gscale, int zero_grad, hipStream_t st) {
  launch_apply_dev<AdagradOp, 1>(AdagradOp{0.f, eps}, w, mirror, grad, grad_bf16, acc, nullptr, n, gscale,
                                 zero_grad, hyper, st);
}

void adam_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* m, float* v, long long n,
                const float* hyper, float b1, float b2, float eps, float wd, float gscale, int zero_grad,
                hipStream_t st) {
  launch_apply_dev<AdamOp, 2>(AdamOp{0.f, b1, b2, eps, wd, 1.f, 1.f}, w, mirror, grad, grad_bf16, m, v, n, gscale,
                              zero_grad, hyper, st);
}

// ---------------------------------------------------------------------------------------------
// acc = alpha*acc + beta*g   (DOWNPOUR/ADAG/SDAG window accumulate: DOWNPOUR/DOWNPOUR.py:77,
// ADAG/ADAG.py:82).  g may be bf16 or fp32; acc is fp32.
// ---------------------------------------------------------------------------------------------
template <bool GBF16>
__global__ void __launch_bounds__(256) axpby_kernel(float* __restrict__ acc, const void* __restrict__ g, long long n,
                                                    float alpha, float beta) {
  const long long nvec = n >> 3;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    const long long i = v << 3;
    float a[8], gv[8];
    load8_f32(acc + i, a);
    load_grad8<GBF16>(g, i, gv);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = alpha * a[k] + beta * gv[k];
    store8_f32(acc + i, a);
  }
  if (blockIdx.x == 0)
    for (long long i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x)
      acc[i] = alpha * acc[i] + beta * load_grad1<GBF16>(g, i);
}

void axpby(float* acc, const void* g, int g_bf16, long long n, float alpha, float beta, hipStream_t st) {
  const int grid = grid_for((n >> 3) + 1, 256, 2048);
  if (g_bf16) { axpby_kernel<true><<<grid, 256, 0, st>>>(acc, g, n, alpha, beta); DTG_LAUNCH_CHECK(); }
  else { axpby_kernel<false><<<grid, 256, 0, st>>>(acc, g, n, alpha, beta); DTG_LAUNCH_CHECK(); }
}

// fp32 -> bf16 mirror refresh (after a PS pull / checkpoint restore)
__global__ void __launch_bounds__(256) f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                          long long n) {
  const long long nvec = n >> 3;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float a[8];
    load8_f32(x + (v << 3), a);
    store8_bf16(y + (v << 3), a);
  }
  if (blockIdx.x == 0)
    for (long long i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) y[i] = f2bf(x[i]);
}

void f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t st) {
  f32_to_bf16_kernel<<<grid_for((n >> 3) + 1, 256, 2048), 256, 0, st>>>(x, y, n); DTG_LAUNCH_CHECK();
}

// Stream-ordered zero fill with vector stores (instead of hipMemsetAsync, which launches the runtime's own
// fill kernel): 16 B per lane, then the byte tail.
__global__ void __launch_bounds__(256) fill_zero_kernel(unsigned char* __restrict__ p, long long bytes) {
  const long long nvec = bytes >> 4;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride)
    reinterpret_cast<uint4*>(p)[v] = make_uint4(0u, 0u, 0u, 0u);
  if (blockIdx.x == 0)
    for (long long i = (nvec << 4) + threadIdx.x; i < bytes; i += blockDim.x) p[i] = 0;
}

void fill_zero(void* p, long long bytes, hipStream_t st) {
  if (bytes <= 0) return;
  fill_zero_kernel<<<grid_for((bytes >> 4) + 1, 256, 4096), 256, 0, st>>>(reinterpret_cast<unsigned char*>(p), bytes);
  DTG_LAUNCH_CHECK();
}

// hyper[1] += 1: the step counter the applies read (device-resident so a captured step replays with a fresh
// value); one lane, one vector store, stream-ordered before the step's apply kernels
__global__ void hyper_tick_kernel(float* hyper) {
  if (threadIdx.x == 0) hyper[1] = hyper[1] + 1.f;
}

void hyper_tick(float* hyper, hipStream_t st) {
  hyper_tick_kernel<<<1, 64, 0, st>>>(hyper); DTG_LAUNCH_CHECK();
}

}  // namespace dtg
