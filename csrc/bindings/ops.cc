// PyTorch bindings for dtg's HIP kernels (module dtg._C).
// Each wrapper validates shapes/dtypes/devices on the host (a kernel never sees an operand whose
// shape disagrees with its grid), allocates outputs with the caching allocator and launches on the
// current HIP stream, so everything composes with torch streams and hipGraph capture.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "dtg/kernels.h"

namespace {

using at::Tensor;
using dtg::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

// fp32 zeros on like's device, filled by a dtg kernel on the current stream
at::Tensor zeros_f32(long long n, const at::Tensor& like) {
  c10::DeviceGuard dg(like.device());  // the fill runs on like's device's current stream
  at::Tensor t = at::empty({n}, like.options().dtype(at::kFloat));
  dtg::fill_zero(t.data_ptr(), n * 4, cur_stream());
  return t;
}

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_DT(x, dt) TORCH_CHECK((x).scalar_type() == (dt), #x " must be " #dt)
#define CHECK_IN(x) \
  CHECK_CUDA(x);    \
  CHECK_CONTIG(x)

bf16_t* bfp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
const bf16_t* cbfp(const Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
template <class T>
T* opt_ptr(const c10::optional<Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

void check_flat(const Tensor& w, const Tensor& g, const c10::optional<Tensor>& mirror) {
  CHECK_IN(w);
  CHECK_IN(g);
  CHECK_DT(w, at::kFloat);
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "grad must be fp32 or bf16");
  TORCH_CHECK(g.numel() == w.numel(), "grad/param size mismatch");
  if (mirror.has_value() && mirror->defined()) {
    CHECK_IN(*mirror);
    CHECK_DT(*mirror, at::kBFloat16);
    TORCH_CHECK(mirror->numel() == w.numel(), "mirror size mismatch");
  }
}

void check_state(const Tensor& s, const Tensor& w) {
  CHECK_IN(s);
  CHECK_DT(s, at::kFloat);
  TORCH_CHECK(s.numel() == w.numel(), "optimizer state size mismatch");
}

void check_hyper(const Tensor& h) {
  CHECK_IN(h);
  CHECK_DT(h, at::kFloat);
  TORCH_CHECK(h.numel() >= 2, "hyper must hold {lr, step}");
}

// ---- optimizers ----------------------------------------------------------------------------
void sgd_apply(Tensor w, c10::optional<Tensor> mirror, Tensor g, Tensor hyper, double wd, double gscale,
               bool zero_grad) {
  check_flat(w, g, mirror);
  check_hyper(hyper);
  c10::DeviceGuard dg(w.device());
  dtg::sgd_apply(w.data_ptr<float>(), opt_ptr<bf16_t>(mirror), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                 w.numel(), hyper.data_ptr<float>(), (float)wd, (float)gscale, zero_grad, cur_stream());
}

void momentum_apply(Tensor w, c10::optional<Tensor> mirror, Tensor g, Tensor mom, Tensor hyper, double mu, double wd,
                    bool nesterov, double gscale, bool zero_grad) {
  check_flat(w, g, mirror);
  check_state(mom, w);
  check_hyper(hyper);
  c10::DeviceGuard dg(w.device());
  dtg::momentum_apply(w.data_ptr<float>(), opt_ptr<bf16_t>(mirror), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                      mom.data_ptr<float>(), w.numel(), hyper.data_ptr<float>(), (float)mu, (float)wd, nesterov,
                      (float)gscale, zero_grad, cur_stream());
}

void adagrad_apply(Tensor w, c10::optional<Tensor> mirror, Tensor g, Tensor acc, Tensor hyper, double eps,
                   double gscale, bool zero_grad) {
  check_flat(w, g, mirror);
  check_state(acc, w);
  check_hyper(hyper);
  c10::DeviceGuard dg(w.device());
  dtg::adagrad_apply(w.data_ptr<float>(), opt_ptr<bf16_t>(mirror), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                     acc.data_ptr<float>(), w.numel(), hyper.data_ptr<float>(), (float)eps, (float)gscale, zero_grad,
                     cur_stream());
}

void adam_apply(Tensor w, c10::optional<Tensor> mirror, Tensor g, Tensor m, Tensor v, Tensor hyper, double b1,
                double b2, double eps, double wd, double gscale, bool zero_grad) {
  check_flat(w, g, mirror);
  check_state(m, w);
  check_state(v, w);
  check_hyper(hyper);
  c10::DeviceGuard dg(w.device());
  dtg::adam_apply(w.data_ptr<float>(), opt_ptr<bf16_t>(mirror), g.data_ptr(), g.scalar_type() == at::kBFloat16,
                  m.data_ptr<float>(), v.data_ptr<float>(), w.numel(), hyper.data_ptr<float>(), (float)b1, (float)b2,
                  (float)eps, (float)wd, (float)gscale, zero_grad, cur_stream());
}

void axpby(Tensor acc, Tensor g, double alpha, double beta) {
  CHECK_IN(acc);
  CHECK_IN(g);
  CHECK_DT(acc, at::kFloat);
  TORCH_CHECK(g.scalar_type() == at::kFloat || g.scalar_type() == at::kBFloat16, "g must be fp32 or bf16");
  TORCH_CHECK(acc.numel() == g.numel(), "size mismatch");
  c10::DeviceGuard dg(acc.device());
  dtg::axpby(acc.data_ptr<float>(), g.data_ptr(), g.scalar_type() == at::kBFloat16, acc.numel(), (float)alpha,
             (float)beta, cur_stream());
}

void f32_to_bf16(Tensor x, Tensor y) {
  CHECK_IN(x);
  CHECK_IN(y);
  CHECK_DT(x, at::kFloat);
  CHECK_DT(y, at::kBFloat16);
  TORCH_CHECK(x.numel() == y.numel(), "size mismatch");
  c10::DeviceGuard dg(x.device());
  dtg::f32_to_bf16(x.data_ptr<float>(), bfp(y), x.numel(), cur_stream());
}

// ---- batchnorm -------------------------------------------------------------------------------
// x: NHWC-contiguous bf16 viewed as [M, C] (the caller passes channels_last tensors flattened).
std::tuple<Tensor, Tensor, Tensor> bn_fwd_train(Tensor x, c10::optional<Tensor> res, Tensor gamma, Tensor beta,
                                                Tensor rmean, Tensor rvar, double momentum, double eps, bool relu) {
  CHECK_IN(x);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2, "x must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  for (const Tensor* t : {&gamma, &beta, &rmean, &rvar}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  if (res.has_value() && res->defined()) {
    CHECK_IN(*res);
    CHECK_DT(*res, at::kBFloat16);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto smean = at::empty({C}, fopt), sinv = at::empty({C}, fopt);
  auto ws = at::empty({dtg::bn_workspace_floats(M, C)}, fopt);
  dtg::bn_fwd_train(cbfp(x), res.has_value() && res->defined() ? cbfp(*res) : nullptr, bfp(y),
                    gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                    smean.data_ptr<float>(), sinv.data_ptr<float>(), ws.data_ptr<float>(), M, C, (float)momentum,
                    (float)eps, relu, cur_stream());
  return {y, smean, sinv};
}

Tensor bn_fwd_infer(Tensor x, c10::optional<Tensor> res, Tensor gamma, Tensor beta, Tensor rmean, Tensor rvar,
                    double eps, bool relu) {
  CHECK_IN(x);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2, "x must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  for (const Tensor* t : {&gamma, &beta, &rmean, &rvar}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  if (res.has_value() && res->defined()) {
    CHECK_IN(*res);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto y = at::empty_like(x);
  auto ws = at::empty({2LL * C}, x.options().dtype(at::kFloat));
  dtg::bn_fwd_infer(cbfp(x), res.has_value() && res->defined() ? cbfp(*res) : nullptr, bfp(y),
                    gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                    ws.data_ptr<float>(), M, C, (float)eps, relu, cur_stream());
  return y;
}

// dgamma_acc / dbeta_acc given: the parameter gradients are ACCUMULATED into them (flat grads)
std::tuple<Tensor, c10::optional<Tensor>, Tensor, Tensor> bn_bwd(Tensor dy, c10::optional<Tensor> y, Tensor x,
                                                                  Tensor gamma, Tensor smean, Tensor sinv, bool relu,
                                                                  bool want_dres, c10::optional<Tensor> dgamma_acc,
                                                                  c10::optional<Tensor> dbeta_acc) {
  CHECK_IN(dy);
  CHECK_IN(x);
  CHECK_DT(dy, at::kBFloat16);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(dy.sizes() == x.sizes() && x.dim() == 2, "dy/x must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  if (relu) {
    TORCH_CHECK(y.has_value() && y->defined(), "relu backward needs the saved output");
    CHECK_IN(*y);
    TORCH_CHECK(y->sizes() == x.sizes(), "y shape mismatch");
  }
  for (const Tensor* t : {&gamma, &smean, &sinv}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto dx = at::empty_like(x);
  c10::optional<Tensor> dres;
  if (want_dres) dres = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined() && dbeta_acc.has_value() && dbeta_acc->defined();
  Tensor dgamma, dbeta;
  if (acc) {
    dgamma = *dgamma_acc;
    dbeta = *dbeta_acc;
    for (const Tensor* t : {&dgamma, &dbeta}) {
      CHECK_IN(*t);
      CHECK_DT(*t, at::kFloat);
      TORCH_CHECK(t->numel() == C, "gradient accumulator size mismatch");
    }
  } else {
    dgamma = at::empty({C}, fopt);
    dbeta = at::empty({C}, fopt);
  }
  auto ws = at::empty({dtg::bn_workspace_floats(M, C) + C}, fopt);
  dtg::bn_bwd(cbfp(dy), relu ? cbfp(*y) : nullptr, cbfp(x), gamma.data_ptr<float>(), smean.data_ptr<float>(),
              sinv.data_ptr<float>(), bfp(dx), want_dres ? bfp(*dres) : nullptr, dgamma.data_ptr<float>(),
              dbeta.data_ptr<float>(), ws.data_ptr<float>(), M, C, relu, acc, cur_stream());
  return {dx, dres, dgamma, dbeta};
}

// ---- softmax cross entropy -----------------------------------------------------------------
std::tuple<Tensor, c10::optional<Tensor>, Tensor> softmax_xent(Tensor logits, Tensor labels, double scale,
                                                                bool want_grad) {
  CHECK_IN(logits);
  CHECK_IN(labels);
  TORCH_CHECK(logits.dim() == 2, "logits must be [B, V]");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16/fp32");
  CHECK_DT(labels, at::kLong);
  TORCH_CHECK(labels.numel() == logits.size(0), "labels size mismatch");
  c10::DeviceGuard dg(logits.device());
  const long long B = logits.size(0);
  const int V = (int)logits.size(1);
  auto fopt = logits.options().dtype(at::kFloat);
  auto loss = at::empty({B}, fopt), lse = at::empty({B}, fopt);
  c10::optional<Tensor> dx;
  if (want_grad) dx = at::empty_like(logits);
  if (B > 0)
    dtg::softmax_xent(logits.data_ptr(), logits.scalar_type() == at::kBFloat16, reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), B, V,
                      (float)scale, loss.data_ptr<float>(), want_grad ? dx->data_ptr() : nullptr,
                      lse.data_ptr<float>(), cur_stream());
  return {loss, dx, lse};
}

// dlogits = (softmax(logits) - onehot(labels)) * scale * g, g a 0-d/1-element fp32 GPU tensor (the
// upstream gradient, read on the device: no host sync, no separate rescale pass)
Tensor softmax_xent_bwd(Tensor logits, Tensor labels, Tensor lse, Tensor g, double scale) {
  CHECK_IN(logits);
  CHECK_IN(labels);
  CHECK_IN(lse);
  TORCH_CHECK(logits.dim() == 2, "logits must be [B, V]");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat, "logits bf16/fp32");
  CHECK_DT(labels, at::kLong);
  CHECK_DT(lse, at::kFloat);
  const long long B = logits.size(0);
  const int V = (int)logits.size(1);
  TORCH_CHECK(labels.numel() == B && lse.numel() == B, "labels / lse size mismatch");
  CHECK_CUDA(g);
  TORCH_CHECK(g.numel() == 1, "g must hold one element");
  Tensor gf = g.scalar_type() == at::kFloat ? g.contiguous() : g.to(at::kFloat);
  c10::DeviceGuard dg(logits.device());
  auto dx = at::empty_like(logits);
  if (B > 0)
    dtg::softmax_xent_bwd(logits.data_ptr(), logits.scalar_type() == at::kBFloat16,
                          reinterpret_cast<const long long*>(labels.data_ptr<int64_t>()), lse.data_ptr<float>(), B, V,
                          (float)scale, gf.data_ptr<float>(), dx.data_ptr(), cur_stream());
  return dx;
}

// ---- GEMM ----------------------------------------------------------------------------------
// out[M,N] = act(alpha * op(A) op(B) + beta*out + bias).  a_kc: A stored [M,K] (else [K,M]);
// b_kc: B stored [N,K] (else [K,N]).  Row strides are taken from the 2-D tensors.
void gemm(Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor out, double alpha, double beta,
          c10::optional<Tensor> bias, int64_t act, int64_t split_k, c10::optional<Tensor> aux, int64_t aux_mode,
          c10::optional<Tensor> colsum) {
  CHECK_CUDA(A);
  CHECK_CUDA(B);
  CHECK_CUDA(out);
  CHECK_DT(A, at::kBFloat16);
  CHECK_DT(B, at::kBFloat16);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && out.dim() == 2, "gemm operands must be 2-D");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && out.stride(1) == 1, "inner dim must be contiguous");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out fp32/bf16");
  const int M = (int)(a_kc ? A.size(0) : A.size(1));
  const int K = (int)(a_kc ? A.size(1) : A.size(0));
  const int N = (int)(b_kc ? B.size(0) : B.size(1));
  const int Kb = (int)(b_kc ? B.size(1) : B.size(0));
  TORCH_CHECK(K == Kb, "gemm K mismatch: ", K, " vs ", Kb);
  TORCH_CHECK(out.size(0) == M && out.size(1) == N, "gemm out shape mismatch");
  TORCH_CHECK(K % 8 == 0 || (!a_kc && !b_kc), "K-contiguous operands need K % 8 == 0 (pad the reduction dim)");
  TORCH_CHECK(a_kc || M % 8 == 0, "K-major A needs M % 8 == 0");
  TORCH_CHECK(b_kc || N % 8 == 0, "K-major B needs N % 8 == 0");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "row strides must be 16-byte multiples");
  TORCH_CHECK(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0, "16-byte alignment");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    CHECK_IN(*bias);
    CHECK_DT(*bias, at::kFloat);
    TORCH_CHECK(bias->numel() == N, "bias size mismatch");
    bptr = bias->data_ptr<float>();
  }
  void* auxp = nullptr;
  if (aux_mode != 0) {
    TORCH_CHECK(aux_mode >= 1 && aux_mode <= 4, "aux_mode in {0, 1, 2, 3, 4}");
    TORCH_CHECK(aux_mode != 3 || act != 0, "aux_mode 3 stores act'(pre): needs an activation");
    TORCH_CHECK(aux.has_value() && aux->defined(), "aux_mode needs an aux tensor");
    TORCH_CHECK(aux->is_cuda() && aux->scalar_type() == at::kBFloat16 && aux->dim() == 2, "aux must be bf16 2-D");
    TORCH_CHECK(aux->size(0) == M && aux->size(1) == N && aux->stride(0) == out.stride(0) && aux->stride(1) == 1,
                "aux must match out's shape and row stride");
    auxp = aux->data_ptr();
  }
  c10::DeviceGuard dg(A.device());
  if (colsum.has_value() && colsum->defined()) {
    // fused bias gradient: colsum[n] += sum_m out[m, n] (dgrad layout, bf16 out, plain alpha/beta)
    CHECK_IN(*colsum);
    CHECK_DT(*colsum, at::kFloat);
    TORCH_CHECK(colsum->numel() == N, "colsum must hold N floats");
    TORCH_CHECK(a_kc && !b_kc && out.scalar_type() == at::kBFloat16 && alpha == 1.0 && beta == 0.0,
                "colsum epilogue: A [M,K], B [K,N], bf16 out, alpha 1, beta 0");
    TORCH_CHECK(out.stride(0) % 8 == 0 && N % 8 == 0 && ((uintptr_t)out.data_ptr() % 16) == 0 &&
                    (bptr == nullptr || ((uintptr_t)bptr % 16) == 0) && (auxp == nullptr || ((uintptr_t)auxp % 16) == 0),
                "colsum epilogue needs 16-byte aligned rows");
    dtg::gemm_bf16_colsum(cbfp(A), A.stride(0), cbfp(B), B.stride(0), bfp(out), out.stride(0), M, N, K, bptr, (int)act,
                          auxp, (int)aux_mode, colsum->data_ptr<float>(), cur_stream());
    return;
  }
  int sk = split_k > 0 ? (int)split_k : dtg::gemm_pick_split(M, N, K, a_kc ? 1 : 0);
  Tensor ws;
  float* wsp = nullptr;
  if (sk > 1) {
    ws = at::empty({dtg::gemm_workspace_floats(M, N, K, sk)}, A.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  dtg::gemm_bf16(cbfp(A), A.stride(0), a_kc, cbfp(B), B.stride(0), b_kc, out.data_ptr(), out.stride(0),
                 out.scalar_type() == at::kBFloat16, M, N, K, (float)alpha, (float)beta, bptr, (int)act, sk, wsp,
                 cur_stream(), dtg::GemmBatch(), auxp, (int)aux_mode);
}

// ---- implicit-GEMM convolution -----------------------------------------------------------------
// Activations are NHWC-contiguous ("channels_last") bf16 tensors given as [N, H, W, C] views;
// the weight is [K, R, S, C] contiguous (a channels_last [K, C, R, S] parameter viewed as such).
void check_nhwc(const Tensor& t, const char* what) {
  CHECK_CUDA(t);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, what, " must be bf16");
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(), what, " must be a contiguous [N,H,W,C] tensor");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0, what, " must be 16-byte aligned");
}

bool conv_supported(int64_t C, int64_t K, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t which) {
  return dtg::conv_supported((int)C, (int)K, (int)R, (int)S, (int)stride, (int)pad, (int)which) != 0;
}

Tensor conv_fwd(Tensor x, Tensor w, int64_t stride, int64_t pad) {
  check_nhwc(x, "x");
  check_nhwc(w, "w");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(w.size(3) == C, "weight channels mismatch");
  TORCH_CHECK(dtg::conv_supported(C, K, R, S, stride, pad, 0), "conv shape not supported by the HIP kernel");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty output");
  TORCH_CHECK((long long)N * H * W * C < (1LL << 31) && (long long)N * P * Q * K < (1LL << 31), "tensor too large");
  c10::DeviceGuard dg(x.device());
  auto y = at::empty({N, P, Q, K}, x.options());
  dtg::conv_fwd(cbfp(x), cbfp(w), bfp(y), N, H, W, C, K, R, S, stride, pad, cur_stream());
  return y;
}

// (a stride-1 dgrad that read the weight transposed to [C][(r,s,k)] measured equal within +-5 % on the
// ResNet-50 3x3 layers and was retired; conv_dgrad's wT argument stays for the kernel's K-contiguous form)

// dx (= or +=, beta) dgrad; `out` (optional, [N,H,W,C] bf16) receives it in place.  zero_rest=False: a
// strided dgrad leaves the rows no filter tap reaches unwritten (see gemm_bn's sub2_hw)
Tensor conv_dgrad(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t stride, int64_t pad, c10::optional<Tensor> out,
                  double beta, bool zero_rest) {
  check_nhwc(dy, "dy");
  check_nhwc(w, "w");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  const int R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(w.size(0) == K, "weight/dy channel mismatch");
  TORCH_CHECK(dtg::conv_supported(C, K, R, S, stride, pad, 1), "dgrad shape not supported by the HIP kernel");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == P && (W + 2 * pad - S) / stride + 1 == Q, "dgrad geometry mismatch");
  c10::DeviceGuard dg(dy.device());
  Tensor dx;
  if (out.has_value()) {
    dx = *out;
    check_nhwc(dx, "out");
    TORCH_CHECK(dx.size(0) == N && dx.size(1) == H && dx.size(2) == W && dx.size(3) == C, "out shape mismatch");
  } else {
    TORCH_CHECK(beta == 0.0, "beta != 0 needs out");
    dx = at::empty({N, H, W, C}, dy.options());
  }
  Tensor wT;
  TORCH_CHECK(zero_rest || (stride == 2 && R == 1 && S == 1 && pad == 0 && beta == 0.0),
              "zero_rest=False is for a stride-2 1x1 dgrad (beta 0)");
  dtg::conv_dgrad(cbfp(dy), cbfp(w), bfp(dx), N, H, W, C, K, R, S, stride, pad, (float)beta, cur_stream(),
                  dtg::BnEpi(), wT.defined() ? cbfp(wT) : nullptr, zero_rest ? 1 : 0);
  return dx;
}

// 8-channel input conv (the stem): x [N,H,W,8] NHWC, w [K, Kp] with Kp = ceil64(R*S*8), (r,s,c) columns.
// with_stats: also the forward BN statistics of y (returned partials, else an empty tensor).
// stride_w (0 = stride): a separate W stride -- the stem's pixel-pair form is a stride (2, 1) conv.
std::tuple<Tensor, Tensor> conv_fwd_c8(Tensor x, Tensor w, int64_t R, int64_t S, int64_t stride, int64_t pad,
                                       bool with_stats, int64_t stride_w) {
  check_nhwc(x, "x");
  CHECK_IN(w);
  CHECK_DT(w, at::kBFloat16);
  const int sw = stride_w > 0 ? (int)stride_w : (int)stride;
  const int N = x.size(0), H = x.size(1), W = x.size(2), K = w.size(0);
  TORCH_CHECK(x.size(3) == 8, "conv_fwd_c8 needs 8 input channels");
  TORCH_CHECK(w.dim() == 2 && w.size(1) == (R * S * 8 + 63) / 64 * 64, "w must be [K, ceil64(R*S*8)]");
  TORCH_CHECK(K % 64 == 0, "K % 64");
  TORCH_CHECK(stride > 0 && sw > 0 && pad >= 0, "bad stride / pad");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / sw + 1;
  TORCH_CHECK(P > 0 && Q > 0 && (long long)N * P * Q * K < (1LL << 31), "bad geometry");
  c10::DeviceGuard dg(x.device());
  auto y = at::empty({N, P, Q, K}, x.options());
  Tensor part;
  dtg::BnEpi bn;
  if (with_stats) {
    part = zeros_f32((long long)dtg::kBnStatSlots * 2 * K, x);
    bn.part = part.data_ptr<float>();
    bn.mode = 1;
  } else {
    part = at::empty({0}, x.options().dtype(at::kFloat));
  }
  dtg::conv_fwd_c8(cbfp(x), cbfp(w), bfp(y), N, H, W, K, (int)R, (int)S, (int)stride, (int)pad, cur_stream(), bn, sw);
  return {y, part};
}

// ---- BN statistics fused into the producing GEMM / conv (dtg/bn_epi.cuh) ----------------------
// Statistics slots.  pooled: a buffer from a per-device ring of zeroed buffers which the consuming
// finalize (bn_*_part) zeroes again after reading -- no fill kernel per BN.  The caller must consume
// (or zero) every pooled buffer before kPartRing more are handed out; the fused ResNet bottleneck
// does (its producer -> consumer distance is at most 2).  Unpooled: a fresh zeroed tensor.
constexpr int kPartRing = 16;
constexpr long long kPartCap = (long long)dtg::kBnStatSlots * 2 * 2048;
Tensor bn_part(const Tensor& like, int64_t C, bool pooled = false) {
  if (!pooled || C > 2048) return zeros_f32((long long)dtg::kBnStatSlots * 2 * C, like);
  static Tensor* ring = new Tensor[64];  // per device; leaked on purpose (no teardown-order issues)
  static int next[64] = {0};
  const int dev = like.get_device();
  TORCH_CHECK(dev >= 0 && dev < 64, "device index");
  if (!ring[dev].defined()) ring[dev] = zeros_f32((long long)kPartRing * kPartCap, like);
  const int i = next[dev]++ % kPartRing;
  return ring[dev].narrow(0, i * kPartCap, (long long)dtg::kBnStatSlots * 2 * C);
}

dtg::BnEpi bn_bwd_epi(Tensor& part, const Tensor& x, const Tensor& mean, const Tensor& invstd, const Tensor& gamma,
                      const Tensor& beta, long long M, int C) {
  CHECK_IN(x);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.numel() == M * C, "BN input shape mismatch");
  for (const Tensor* t : {&mean, &invstd, &gamma, &beta}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  dtg::BnEpi bn;
  bn.part = part.data_ptr<float>();
  bn.mode = 2;
  bn.x = cbfp(x);
  bn.mean = mean.data_ptr<float>();
  bn.invstd = invstd.data_ptr<float>();
  bn.gamma = gamma.data_ptr<float>();
  bn.beta = beta.data_ptr<float>();
  return bn;
}

// mode 1: out = A W^T (W [N,K]) + forward BN statistics of out.
// mode 2: dp = (dY W) * relu'(bn(x)) (W [K,N]) + backward BN partials (x, mean, invstd, gamma, beta given).
// mode 3: dp = [mask > 0] * (dY W + beta*out) written into `out` (beta = 1 when out is given), partials
//         with xhat from x (the BN input of the layer whose relu output `mask` is).
std::tuple<Tensor, Tensor> gemm_bn(Tensor A, Tensor B, int64_t mode, c10::optional<Tensor> x,
                                   c10::optional<Tensor> mean, c10::optional<Tensor> invstd,
                                   c10::optional<Tensor> gamma, c10::optional<Tensor> beta,
                                   c10::optional<Tensor> mask, c10::optional<Tensor> out, bool pooled,
                                   c10::optional<Tensor> x2, c10::optional<Tensor> mean2,
                                   c10::optional<Tensor> invstd2, c10::optional<Tensor> part2,
                                   c10::optional<std::tuple<int64_t, int64_t>> sub2_hw) {
  CHECK_IN(A);
  CHECK_DT(A, at::kBFloat16);
  CHECK_CUDA(B);
  CHECK_DT(B, at::kBFloat16);
  TORCH_CHECK(mode >= 1 && mode <= 3, "mode in {1, 2, 3}");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && B.stride(1) == 1, "2-D operands, contiguous rows");
  const int M = (int)A.size(0), K = (int)A.size(1);
  const int N = (int)(mode == 1 ? B.size(0) : B.size(1));
  TORCH_CHECK((mode == 1 ? B.size(1) : B.size(0)) == K, "gemm_bn K mismatch");
  TORCH_CHECK(K % 8 == 0 && N % 8 == 0 && B.stride(0) % 8 == 0, "K, N and row strides must be multiples of 8");
  TORCH_CHECK(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0, "16-byte alignment");
  c10::DeviceGuard dg(A.device());
  Tensor o;
  float bt = 0.f;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(mode == 3, "accumulating into `out` is mode 3 only");
    o = *out;
    CHECK_IN(o);
    CHECK_DT(o, at::kBFloat16);
    TORCH_CHECK(o.numel() == (long long)M * N, "out shape mismatch");
    bt = 1.f;
  } else {
    o = at::empty({M, N}, A.options());
  }
  auto part = bn_part(A, N, pooled);
  dtg::BnEpi bn;
  if (mode >= 2) {
    TORCH_CHECK(x && mean && invstd && gamma && beta, "modes 2/3 need x, mean, invstd, gamma, beta");
    bn = bn_bwd_epi(part, *x, *mean, *invstd, *gamma, *beta, M, N);
    if (mode == 3) {
      TORCH_CHECK(mask.has_value() && mask->defined(), "mode 3 needs the mask tensor");
      CHECK_IN(*mask);
      bn.mode = 3;
      if (x2.has_value() && x2->defined()) {  // second BN on the same gradient (projection shortcut)
        TORCH_CHECK(mean2 && invstd2 && part2, "x2 needs mean2, invstd2 and part2");
        CHECK_IN(*x2);
        CHECK_DT(*x2, at::kBFloat16);
        TORCH_CHECK(x2->numel() == (long long)M * N, "x2 shape mismatch");
        for (const Tensor* t : {&*mean2, &*invstd2}) {
          CHECK_IN(*t);
          CHECK_DT(*t, at::kFloat);
          TORCH_CHECK(t->numel() == N, "per-channel tensor size mismatch");
        }
        CHECK_IN(*part2);
        CHECK_DT(*part2, at::kFloat);
        TORCH_CHECK(part2->numel() == (long long)dtg::kBnStatSlots * 2 * N, "part2 size mismatch");
        bn.x2 = cbfp(*x2);
        bn.mean2 = mean2->data_ptr<float>();
        bn.invstd2 = invstd2->data_ptr<float>();
        bn.part2 = part2->data_ptr<float>();
      }
      if (sub2_hw.has_value()) {  // `out` holds a stride-2 projection dgrad: only its even (h, w) rows are valid
        const auto [sh, sw] = *sub2_hw;
        TORCH_CHECK(bt != 0.f && sh > 0 && sw > 0 && (long long)M % (sh * sw) == 0, "sub2_hw needs out and M = N*H*W");
        dtg::bn_sub2_rows(bn, (int)sh, (int)sw);
      }
      if (mask->scalar_type() == at::kByte) {  // packed bits [M, N/8]
        TORCH_CHECK(mask->numel() == (long long)M * (N / 8), "mask bits shape mismatch");
        bn.maskbits = mask->data_ptr<uint8_t>();
      } else {
        CHECK_DT(*mask, at::kBFloat16);
        TORCH_CHECK(mask->numel() == (long long)M * N, "mask shape mismatch");
        bn.mask = cbfp(*mask);
      }
    }
  } else {
    bn.part = part.data_ptr<float>();
    bn.mode = 1;
  }
  dtg::gemm_bf16_bn(cbfp(A), A.stride(0), cbfp(B), B.stride(0), bfp(o), N, M, N, K, bt, bn, cur_stream());
  return {o, part};
}

std::tuple<Tensor, Tensor> conv_fwd_bn(Tensor x, Tensor w, int64_t stride, int64_t pad, bool pooled) {
  check_nhwc(x, "x");
  check_nhwc(w, "w");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = w.size(0), R = w.size(1), S = w.size(2);
  TORCH_CHECK(w.size(3) == C, "weight channels mismatch");
  TORCH_CHECK(dtg::conv_supported(C, K, R, S, stride, pad, 0), "conv shape not supported by the HIP kernel");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty output");
  TORCH_CHECK((long long)N * H * W * C < (1LL << 31) && (long long)N * P * Q * K < (1LL << 31), "tensor too large");
  c10::DeviceGuard dg(x.device());
  auto y = at::empty({N, P, Q, K}, x.options());
  auto part = bn_part(x, K, pooled);
  // (3x3 / s1 / p1, 64 -> 64: conv_fwd takes the direct halo-tile conv, csrc/kernels/conv_halo.hip)
  dtg::BnEpi bn;
  bn.part = part.data_ptr<float>();
  bn.mode = 1;
  dtg::conv_fwd(cbfp(x), cbfp(w), bfp(y), N, H, W, C, K, R, S, stride, pad, cur_stream(), bn);
  return {y, part};
}

// dp = dgrad(dy, w) * relu'(bn(x)) with backward BN partials; x is the BN input [N,H,W,C]
uint8_t* bits_ptr(const c10::optional<Tensor>& bits, long long M, int C) {
  if (!bits.has_value() || !bits->defined()) return nullptr;
  CHECK_IN(*bits);
  TORCH_CHECK(bits->scalar_type() == at::kByte && bits->numel() == M * (C / 8), "bits must be uint8 [M, C/8]");
  return bits->data_ptr<uint8_t>();
}

std::tuple<Tensor, Tensor> conv_dgrad_bn(Tensor dy, Tensor w, int64_t H, int64_t W, int64_t stride, int64_t pad,
                                         Tensor x, Tensor mean, Tensor invstd, Tensor gamma, Tensor beta,
                                         bool pooled, c10::optional<Tensor> bits) {
  check_nhwc(dy, "dy");
  check_nhwc(w, "w");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), K = dy.size(3);
  const int R = w.size(1), S = w.size(2), C = w.size(3);
  TORCH_CHECK(w.size(0) == K, "weight/dy channel mismatch");
  TORCH_CHECK(dtg::conv_supported(C, K, R, S, stride, pad, 1), "dgrad shape not supported by the HIP kernel");
  TORCH_CHECK((H + 2 * pad - R) / stride + 1 == P && (W + 2 * pad - S) / stride + 1 == Q, "dgrad geometry mismatch");
  c10::DeviceGuard dg(dy.device());
  auto dx = at::empty({N, H, W, C}, dy.options());
  auto part = bn_part(dy, C, pooled);
  dtg::BnEpi bn = bn_bwd_epi(part, x, mean, invstd, gamma, beta, (long long)N * H * W, C);
  if (uint8_t* mb = bits_ptr(bits, (long long)N * H * W, C)) {  // the forward's packed relu mask: mode 3, beta 0
    bn.mode = 3;
    bn.maskbits = mb;
  }
  // stride 1: the kernel reads the weight transposed to [C][(r,s,k)] (K-contiguous; ~1 MB, one small copy)
  Tensor wT;
  TORCH_CHECK(dtg::conv_dgrad(cbfp(dy), cbfp(w), bfp(dx), N, H, W, C, K, R, S, stride, pad, 0.f, cur_stream(), bn,
                              wT.defined() ? cbfp(wT) : nullptr),
              "conv_dgrad_bn: geometry leaves rows unwritten (use conv_dgrad + bn_bwd)");
  return {dx, part};
}

// bits (optional uint8 [M, C/8]) receives the packed (out > 0) relu mask
std::tuple<Tensor, Tensor, Tensor> bn_fwd_part(Tensor x, Tensor part, c10::optional<Tensor> res, Tensor gamma,
                                               Tensor beta, Tensor rmean, Tensor rvar, double momentum, double eps,
                                               bool relu, c10::optional<Tensor> bits) {
  CHECK_IN(x);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2, "x must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  CHECK_IN(part);
  CHECK_DT(part, at::kFloat);
  TORCH_CHECK(part.numel() == (long long)dtg::kBnStatSlots * 2 * C, "partials size mismatch");
  for (const Tensor* t : {&gamma, &beta, &rmean, &rvar}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  const bool has_res = res.has_value() && res->defined();
  if (has_res) {
    CHECK_IN(*res);
    CHECK_DT(*res, at::kBFloat16);
    TORCH_CHECK(res->sizes() == x.sizes(), "residual shape mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto smean = at::empty({C}, fopt), sinv = at::empty({C}, fopt), ws = at::empty({2LL * C}, fopt);
  dtg::bn_fwd_from_part(cbfp(x), has_res ? cbfp(*res) : nullptr, bfp(y), gamma.data_ptr<float>(),
                        beta.data_ptr<float>(), rmean.data_ptr<float>(), rvar.data_ptr<float>(),
                        smean.data_ptr<float>(), sinv.data_ptr<float>(), part.data_ptr<float>(), ws.data_ptr<float>(),
                        M, C, (float)momentum, (float)eps, relu, cur_stream(), bits_ptr(bits, M, C));
  return {y, smean, sinv};
}

// out = relu(bn(x) + bn2(r)), both from epilogue partials -> (out, mean, invstd, mean2, invstd2)
std::tuple<Tensor, Tensor, Tensor, Tensor, Tensor> bn_fwd2_part(Tensor x, Tensor part, Tensor gamma, Tensor beta,
                                                                Tensor rmean, Tensor rvar, Tensor r, Tensor part2,
                                                                Tensor gamma2, Tensor beta2, Tensor rmean2,
                                                                Tensor rvar2, double momentum, double eps,
                                                                c10::optional<Tensor> bits) {
  CHECK_IN(x);
  CHECK_IN(r);
  CHECK_DT(x, at::kBFloat16);
  CHECK_DT(r, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && r.sizes() == x.sizes(), "x/r must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  for (const Tensor* t : {&part, &part2}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == (long long)dtg::kBnStatSlots * 2 * C, "partials size mismatch");
  }
  for (const Tensor* t : {&gamma, &beta, &rmean, &rvar, &gamma2, &beta2, &rmean2, &rvar2}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto y = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  auto m1 = at::empty({C}, fopt), i1 = at::empty({C}, fopt), m2 = at::empty({C}, fopt), i2 = at::empty({C}, fopt);
  auto ws = at::empty({4LL * C}, fopt);
  dtg::bn_fwd2_from_part(cbfp(x), cbfp(r), bfp(y), part.data_ptr<float>(), part2.data_ptr<float>(),
                         gamma.data_ptr<float>(), beta.data_ptr<float>(), rmean.data_ptr<float>(),
                         rvar.data_ptr<float>(), m1.data_ptr<float>(), i1.data_ptr<float>(), gamma2.data_ptr<float>(),
                         beta2.data_ptr<float>(), rmean2.data_ptr<float>(), rvar2.data_ptr<float>(),
                         m2.data_ptr<float>(), i2.data_ptr<float>(), ws.data_ptr<float>(), M, C, (float)momentum,
                         (float)eps, cur_stream(), bits_ptr(bits, M, C));
  return {y, m1, i1, m2, i2};
}

// dx, dx2 of two BNs fed by the same masked gradient dp (BN3 + projection BN), parameter gradients
// accumulated into the given fp32 accumulators
// fused weight gradient (both bn_bwd*_part): with `wact` [M, CI] (the input of the conv whose output is x) and
// `wgrad` [C, CI] fp32, wgrad += dx^T wact inside the dx pass (bn_dx_wgrad.hip) -- check bn_dx_wgrad_ok first
static void check_wgrad_fuse(const Tensor& x, const c10::optional<Tensor>& wact, const c10::optional<Tensor>& wgrad) {
  TORCH_CHECK(wact.has_value() && wgrad.has_value() && wact->defined() && wgrad->defined(), "wact needs wgrad");
  CHECK_CUDA(*wact);
  CHECK_DT(*wact, at::kBFloat16);
  CHECK_IN(*wgrad);
  TORCH_CHECK(wgrad->scalar_type() == at::kFloat || wgrad->scalar_type() == at::kBFloat16, "wgrad fp32/bf16");
  const long long M = x.size(0);
  const int C = (int)x.size(1), CI = (int)wact->size(1);
  TORCH_CHECK(wact->dim() == 2 && wact->size(0) == M && wact->stride(1) == 1 && wact->stride(0) % 8 == 0 &&
                  ((uintptr_t)wact->data_ptr() % 16) == 0,
              "wact must be [M, CI] with 16-byte aligned rows");
  TORCH_CHECK(wgrad->numel() == (long long)C * CI, "wgrad must be [C, CI]");
  TORCH_CHECK(dtg::bn_dx_wgrad_ok(M, C, CI), "fused dx + wgrad: unsupported shape (see bn_dx_wgrad_ok)");
}

std::tuple<Tensor, Tensor> bn_bwd2_part(Tensor dp, Tensor x, Tensor part, Tensor gamma, Tensor smean, Tensor sinv,
                                        Tensor dgamma, Tensor dbeta, Tensor x2, Tensor part2, Tensor gamma2,
                                        Tensor smean2, Tensor sinv2, Tensor dgamma2, Tensor dbeta2,
                                        c10::optional<Tensor> wact, c10::optional<Tensor> wgrad,
                                        c10::optional<Tensor> wact2, c10::optional<Tensor> wgrad2) {
  for (const Tensor* t : {&dp, &x, &x2}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kBFloat16);
  }
  TORCH_CHECK(x.dim() == 2 && dp.numel() == x.numel() && x2.sizes() == x.sizes(), "dp/x/x2 must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  for (const Tensor* t : {&part, &part2}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == (long long)dtg::kBnStatSlots * 2 * C, "partials size mismatch");
  }
  for (const Tensor* t : {&gamma, &smean, &sinv, &dgamma, &dbeta, &gamma2, &smean2, &sinv2, &dgamma2, &dbeta2}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto dx = at::empty_like(x), dx2 = at::empty_like(x);
  auto ws = at::empty({6LL * C}, x.options().dtype(at::kFloat));
  if (wact.has_value() && wact->defined()) {
    check_wgrad_fuse(x, wact, wgrad);
    const int CI = (int)wact->size(1);
    const bool w2 = wact2.has_value() && wact2->defined();
    if (w2) {  // the projection shortcut's weight gradient too: dW2 += dx2^T wact2 (256 x 64 only)
      check_wgrad_fuse(x2, wact2, wgrad2);
      TORCH_CHECK(C == 256 && CI == 64 && wact2->size(1) == CI && wgrad2->scalar_type() == wgrad->scalar_type(),
                  "wact2: 256 x 64 only, wgrad2 of wgrad's dtype");
    }
    const long long ns = (long long)dtg::bn_dx_wgrad_slabs(C, CI, w2) * C * CI;
    auto slabs = at::empty({w2 ? 2 * ns : ns}, x.options().dtype(at::kFloat));
    float* w = ws.data_ptr<float>();
    dtg::bn_bwd_coef_from_part(part.data_ptr<float>(), gamma.data_ptr<float>(), smean.data_ptr<float>(),
                               sinv.data_ptr<float>(), w, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), M, C, 1,
                               cur_stream());
    dtg::bn_bwd_coef_from_part(part2.data_ptr<float>(), gamma2.data_ptr<float>(), smean2.data_ptr<float>(),
                               sinv2.data_ptr<float>(), w + 3LL * C, dgamma2.data_ptr<float>(),
                               dbeta2.data_ptr<float>(), M, C, 1, cur_stream());
    dtg::bn_dx_wgrad(cbfp(dp), cbfp(x), w, cbfp(x2), w + 3LL * C, bfp(dx), bfp(dx2), cbfp(*wact), wact->stride(0),
                     wgrad->data_ptr(), wgrad->scalar_type() == at::kBFloat16, slabs.data_ptr<float>(), M, C, CI,
                     cur_stream(), w2 ? cbfp(*wact2) : nullptr, w2 ? wact2->stride(0) : 0,
                     w2 ? wgrad2->data_ptr() : nullptr, w2 ? slabs.data_ptr<float>() + ns : nullptr);
    return {dx, dx2};
  }
  dtg::bn_bwd2_from_part(cbfp(dp), cbfp(x), cbfp(x2), part.data_ptr<float>(), part2.data_ptr<float>(),
                         gamma.data_ptr<float>(), smean.data_ptr<float>(), sinv.data_ptr<float>(),
                         gamma2.data_ptr<float>(), smean2.data_ptr<float>(), sinv2.data_ptr<float>(), bfp(dx),
                         bfp(dx2), dgamma.data_ptr<float>(), dbeta.data_ptr<float>(), dgamma2.data_ptr<float>(),
                         dbeta2.data_ptr<float>(), ws.data_ptr<float>(), M, C, 1, cur_stream());
  return {dx, dx2};
}

std::tuple<Tensor, c10::optional<Tensor>, Tensor, Tensor> bn_bwd_part(Tensor dp, Tensor x, Tensor part, Tensor gamma,
                                                                       Tensor smean, Tensor sinv, bool want_dres,
                                                                       c10::optional<Tensor> dgamma_acc,
                                                                       c10::optional<Tensor> dbeta_acc,
                                                                       c10::optional<Tensor> wact,
                                                                       c10::optional<Tensor> wgrad) {
  CHECK_IN(dp);
  CHECK_IN(x);
  CHECK_DT(dp, at::kBFloat16);
  CHECK_DT(x, at::kBFloat16);
  TORCH_CHECK(x.dim() == 2 && dp.numel() == x.numel(), "dp/x must be [M, C]");
  const long long M = x.size(0);
  const int C = (int)x.size(1);
  TORCH_CHECK(C % 8 == 0, "C must be a multiple of 8");
  CHECK_IN(part);
  CHECK_DT(part, at::kFloat);
  TORCH_CHECK(part.numel() == (long long)dtg::kBnStatSlots * 2 * C, "partials size mismatch");
  for (const Tensor* t : {&gamma, &smean, &sinv}) {
    CHECK_IN(*t);
    CHECK_DT(*t, at::kFloat);
    TORCH_CHECK(t->numel() == C, "per-channel tensor size mismatch");
  }
  c10::DeviceGuard dg(x.device());
  auto dx = at::empty_like(x);
  c10::optional<Tensor> dres;
  if (want_dres) dres = at::empty_like(x);
  auto fopt = x.options().dtype(at::kFloat);
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined() && dbeta_acc.has_value() && dbeta_acc->defined();
  Tensor dgamma, dbeta;
  if (acc) {
    dgamma = *dgamma_acc;
    dbeta = *dbeta_acc;
    for (const Tensor* t : {&dgamma, &dbeta}) {
      CHECK_IN(*t);
      CHECK_DT(*t, at::kFloat);
      TORCH_CHECK(t->numel() == C, "gradient accumulator size mismatch");
    }
  } else {
    dgamma = at::empty({C}, fopt);
    dbeta = at::empty({C}, fopt);
  }
  auto ws = at::empty({3LL * C}, fopt);
  if (wact.has_value() && wact->defined()) {
    TORCH_CHECK(!want_dres, "fused dx + wgrad: no dres");
    check_wgrad_fuse(x, wact, wgrad);
    const int CI = (int)wact->size(1);
    auto slabs = at::empty({(long long)dtg::bn_dx_wgrad_slabs(C, CI) * C * CI}, fopt);
    dtg::bn_bwd_coef_from_part(part.data_ptr<float>(), gamma.data_ptr<float>(), smean.data_ptr<float>(),
                               sinv.data_ptr<float>(), ws.data_ptr<float>(), dgamma.data_ptr<float>(),
                               dbeta.data_ptr<float>(), M, C, acc, cur_stream());
    dtg::bn_dx_wgrad(cbfp(dp), cbfp(x), ws.data_ptr<float>(), nullptr, nullptr, bfp(dx), nullptr, cbfp(*wact),
                     wact->stride(0), wgrad->data_ptr(), wgrad->scalar_type() == at::kBFloat16, slabs.data_ptr<float>(),
                     M, C, CI, cur_stream());
    return {dx, dres, dgamma, dbeta};
  }
  dtg::bn_bwd_from_part(cbfp(dp), cbfp(x), gamma.data_ptr<float>(), smean.data_ptr<float>(), sinv.data_ptr<float>(),
                        part.data_ptr<float>(), bfp(dx), want_dres ? bfp(*dres) : nullptr, dgamma.data_ptr<float>(),
                        dbeta.data_ptr<float>(), ws.data_ptr<float>(), M, C, acc, cur_stream());
  return {dx, dres, dgamma, dbeta};
}

// dw (+)= wgrad; dw is [K, R, S, C] contiguous, fp32 or bf16 (beta = 1 accumulates into a flat grad)
void conv_wgrad(Tensor dy, Tensor x, Tensor dw, double beta, int64_t stride, int64_t pad, int64_t stride_w,
                int64_t target_wgs, int64_t sched) {
  check_nhwc(dy, "dy");
  check_nhwc(x, "x");
  CHECK_CUDA(dw);
  TORCH_CHECK(dw.dim() == 4 && dw.is_contiguous(), "dw must be contiguous [K,R,S,C]");
  TORCH_CHECK(dw.scalar_type() == at::kFloat || dw.scalar_type() == at::kBFloat16, "dw fp32/bf16");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int K = dw.size(0), R = dw.size(1), S = dw.size(2);
  TORCH_CHECK(dw.size(3) == C && dy.size(3) == K && dy.size(0) == N, "wgrad shape mismatch");
  TORCH_CHECK(dtg::conv_supported(C, K, R, S, stride, pad, 2), "wgrad shape not supported by the HIP kernel");
  const int sw = stride_w > 0 ? (int)stride_w : (int)stride;
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / sw + 1;
  TORCH_CHECK(dy.size(1) == P && dy.size(2) == Q, "wgrad geometry mismatch");
  c10::DeviceGuard dg(x.device());
  const int split = dtg::conv_wgrad_split(N, H, W, C, K, R, S, stride, pad, sw, (int)target_wgs);
  auto ws = at::empty({(long long)split * K * R * S * C}, x.options().dtype(at::kFloat));
  dtg::conv_wgrad(cbfp(dy), cbfp(x), dw.data_ptr(), dw.scalar_type() == at::kBFloat16, (float)beta,
                  ws.data_ptr<float>(), split, N, H, W, C, K, R, S, stride, pad, cur_stream(), sw, (int)sched);
}

}  // namespace

void register_transformer_ops(pybind11::module_& m);  // transformer_ops.cc
void register_pool_ops(pybind11::module_& m);         // pool_ops.cc

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("conv_supported", &conv_supported);
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_dgrad", &conv_dgrad, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("H"), pybind11::arg("W"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("out") = pybind11::none(),
        pybind11::arg("beta") = 0.0, pybind11::arg("zero_rest") = true);
  m.def("conv_wgrad", &conv_wgrad, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("dw"),
        pybind11::arg("beta"), pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("stride_w") = 0,
        pybind11::arg("target_wgs") = 0, pybind11::arg("sched") = 0);
  m.def("gemm_bn", &gemm_bn, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("mode"),
        pybind11::arg("x") = pybind11::none(), pybind11::arg("mean") = pybind11::none(),
        pybind11::arg("invstd") = pybind11::none(), pybind11::arg("gamma") = pybind11::none(),
        pybind11::arg("beta") = pybind11::none(), pybind11::arg("mask") = pybind11::none(),
        pybind11::arg("out") = pybind11::none(), pybind11::arg("pooled") = false,
        pybind11::arg("x2") = pybind11::none(), pybind11::arg("mean2") = pybind11::none(),
        pybind11::arg("invstd2") = pybind11::none(), pybind11::arg("part2") = pybind11::none(),
        pybind11::arg("sub2_hw") = pybind11::none());
  m.def("bn_part_alloc", [](Tensor like, int64_t C, bool pooled) { return bn_part(like, C, pooled); },
        pybind11::arg("like"), pybind11::arg("C"), pybind11::arg("pooled") = false);
  m.def("bn_bwd2_part", &bn_bwd2_part, pybind11::arg("dp"), pybind11::arg("x"), pybind11::arg("part"),
        pybind11::arg("gamma"), pybind11::arg("smean"), pybind11::arg("sinv"), pybind11::arg("dgamma"),
        pybind11::arg("dbeta"), pybind11::arg("x2"), pybind11::arg("part2"), pybind11::arg("gamma2"),
        pybind11::arg("smean2"), pybind11::arg("sinv2"), pybind11::arg("dgamma2"), pybind11::arg("dbeta2"),
        pybind11::arg("wact") = pybind11::none(), pybind11::arg("wgrad") = pybind11::none(),
        pybind11::arg("wact2") = pybind11::none(), pybind11::arg("wgrad2") = pybind11::none());
  m.def("bn_dx_wgrad_ok", [](int64_t M, int64_t C, int64_t CI) { return dtg::bn_dx_wgrad_ok(M, (int)C, (int)CI); });
  m.def("conv_fwd_bn", &conv_fwd_bn, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("stride"),
        pybind11::arg("pad"), pybind11::arg("pooled") = false);
  m.def("conv_dgrad_bn", &conv_dgrad_bn, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("H"),
        pybind11::arg("W"), pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("x"), pybind11::arg("mean"),
        pybind11::arg("invstd"), pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("pooled") = false,
        pybind11::arg("bits") = pybind11::none());
  m.def("bn_fwd2_part", &bn_fwd2_part, pybind11::arg("x"), pybind11::arg("part"), pybind11::arg("gamma"),
        pybind11::arg("beta"), pybind11::arg("rmean"), pybind11::arg("rvar"), pybind11::arg("r"), pybind11::arg("part2"),
        pybind11::arg("gamma2"), pybind11::arg("beta2"), pybind11::arg("rmean2"), pybind11::arg("rvar2"),
        pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("bits") = pybind11::none());
  m.def("conv_fwd_c8", &conv_fwd_c8, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("R"), pybind11::arg("S"),
        pybind11::arg("stride"), pybind11::arg("pad"), pybind11::arg("with_stats") = false,
        pybind11::arg("stride_w") = 0);
  m.def("bn_fwd_part", &bn_fwd_part, pybind11::arg("x"), pybind11::arg("part"), pybind11::arg("res"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("rmean"), pybind11::arg("rvar"),
        pybind11::arg("momentum"), pybind11::arg("eps"), pybind11::arg("relu"), pybind11::arg("bits") = pybind11::none());
  m.def("bn_bwd_part", &bn_bwd_part, pybind11::arg("dp"), pybind11::arg("x"), pybind11::arg("part"),
        pybind11::arg("gamma"), pybind11::arg("smean"), pybind11::arg("sinv"), pybind11::arg("want_dres"),
        pybind11::arg("dgamma_acc") = pybind11::none(), pybind11::arg("dbeta_acc") = pybind11::none(),
        pybind11::arg("wact") = pybind11::none(), pybind11::arg("wgrad") = pybind11::none());
  m.doc() = "dtg gfx950 HIP kernels";
  m.def("sgd_apply", &sgd_apply);
  m.def("momentum_apply", &momentum_apply);
  m.def("adagrad_apply", &adagrad_apply);
  m.def("adam_apply", &adam_apply);
  m.def("axpby", &axpby);
  m.def("comm_spin", [](double seconds, int64_t wgs, int64_t lds_bytes) {
    dtg::comm_spin(seconds, (int)wgs, (int)lds_bytes, cur_stream());
  }, pybind11::arg("seconds"), pybind11::arg("wgs") = 32, pybind11::arg("lds_bytes") = 0);
  m.def("comm_emu", [](double seconds, int64_t wgs, int64_t mode, c10::optional<Tensor> scratch, int64_t base,
                       int64_t traffic_bytes, c10::optional<Tensor> bucket, double factor) {
    // scratch: a contiguous byte buffer (traffic mode); bucket: the contiguous fp32 / bf16 gradient slice (data mode)
    long long sbytes = 0, n = 0;
    int bf = 0;
    const Tensor* dev_t = nullptr;
    if (scratch.has_value() && scratch->defined()) {
      CHECK_IN(*scratch);
      TORCH_CHECK(((uintptr_t)scratch->data_ptr() % 16) == 0, "scratch: 16-B aligned");
      sbytes = scratch->numel() * scratch->element_size();
      dev_t = &*scratch;
    }
    if (bucket.has_value() && bucket->defined()) {
      CHECK_IN(*bucket);
      TORCH_CHECK(bucket->scalar_type() == at::kFloat || bucket->scalar_type() == at::kBFloat16, "bucket fp32/bf16");
      n = bucket->numel();
      bf = bucket->scalar_type() == at::kBFloat16;
      dev_t = &*bucket;
    }
    TORCH_CHECK(!(mode & 2) || sbytes > 0, "traffic mode needs scratch");
    TORCH_CHECK(!(mode & 4) || n > 0 || !(bucket.has_value() && bucket->defined()), "data mode needs the bucket");
    c10::optional<c10::DeviceGuard> dg;
    if (dev_t) dg.emplace(dev_t->device());
    return dtg::comm_emu(seconds, (int)wgs, (int)mode, sbytes ? scratch->data_ptr() : nullptr, sbytes, base,
                         traffic_bytes, n ? bucket->data_ptr() : nullptr, n, bf, (float)factor, cur_stream());
  }, pybind11::arg("seconds"), pybind11::arg("wgs") = 32, pybind11::arg("mode") = 0,
        pybind11::arg("scratch") = pybind11::none(), pybind11::arg("base") = 0, pybind11::arg("traffic_bytes") = 0,
        pybind11::arg("bucket") = pybind11::none(), pybind11::arg("factor") = 1.0);
  m.def("stem_stream_set", [](int64_t on) { dtg::stem_stream_set((int)on); });
  m.def("gemm_expand_k256_set", [](int64_t on) { dtg::gemm_expand_k256_set((int)on); });
  m.def("stem_pool_rows_set", [](int64_t on) { dtg::stem_pool_rows_set((int)on); });
  m.def("gemm_expand_s2_set", [](int64_t on) { dtg::gemm_expand_s2_set((int)on); });
  m.def("conv_halo_fwd_set", [](int64_t on) { dtg::conv3x3_halo_fwd_set((int)on); });
  m.def("conv_halo_dgrad_set", [](int64_t on) { dtg::conv3x3_halo_dgrad_set((int)on); });
  m.def("conv_halo_wgrad_set", [](int64_t on) { dtg::conv3x3_halo_wgrad_set((int)on); });
  m.def("conv_lin_wgrad_set", [](int64_t on) { dtg::conv3x3_lin_wgrad_set((int)on); });
  m.def("hyper_tick", [](Tensor hyper) {
    check_hyper(hyper);
    c10::DeviceGuard dg(hyper.device());
    dtg::hyper_tick(hyper.data_ptr<float>(), cur_stream());
  });
  m.def("stem_pack_weights", [](Tensor w) {
    CHECK_CUDA(w);
    CHECK_DT(w, at::kBFloat16);
    TORCH_CHECK(w.dim() == 4 && w.is_contiguous(at::MemoryFormat::ChannelsLast) && w.size(1) <= 4,
                "w: channels_last [K, C<=4, R, S]");
    const int K = w.size(0), C = w.size(1), R = w.size(2), S = w.size(3), S2 = (S + 1) / 2;
    const int KP = (R * S2 * 8 + 63) / 64 * 64;
    c10::DeviceGuard dg(w.device());
    auto wp = at::empty({K, KP}, w.options().memory_format(at::MemoryFormat::Contiguous));
    dtg::stem_pack_weights(cbfp(w), bfp(wp), K, C, R, S, S2, KP, cur_stream());
    return wp;
  });
  m.def("stem_dw_add", [](Tensor src, Tensor grad, bool pair) {
    // src [K, R, S2, 8] fp32 (pair) or [K, R, S, 8]; grad: the channels_last [K, C, R, S] parameter gradient
    CHECK_IN(src);
    CHECK_DT(src, at::kFloat);
    CHECK_CUDA(grad);
    TORCH_CHECK(grad.dim() == 4 && grad.is_contiguous(at::MemoryFormat::ChannelsLast), "grad: channels_last [K,C,R,S]");
    TORCH_CHECK(grad.scalar_type() == at::kFloat || grad.scalar_type() == at::kBFloat16, "grad fp32/bf16");
    const int K = grad.size(0), C = grad.size(1), R = grad.size(2), S = grad.size(3);
    TORCH_CHECK(src.dim() == 4 && src.size(0) == K && src.size(1) == R && src.size(3) == 8 && C <= 4 &&
                    src.size(2) == (pair ? (S + 1) / 2 : S), "stem dw source shape");
    c10::DeviceGuard dg(grad.device());
    dtg::stem_dw_add(src.data_ptr<float>(), grad.data_ptr(), grad.scalar_type() == at::kBFloat16, K, R, S, C,
                     (int)src.size(2), pair ? 1 : 0, cur_stream());
  });
  m.def("stream_probe", [](int64_t kind, Tensor a, c10::optional<Tensor> b, c10::optional<Tensor> o, Tensor sink,
                           int64_t wgs, int64_t unroll, bool nt) {
    // a / b / o: contiguous GPU buffers of equal byte size (a multiple of 16); sink: int32 [>= wgs]
    CHECK_IN(a);
    CHECK_IN(sink);
    TORCH_CHECK(sink.scalar_type() == at::kInt && sink.numel() >= wgs, "sink: int32 with >= wgs elements");
    const long long bytes = a.numel() * a.element_size();
    TORCH_CHECK(bytes % 16 == 0 && ((uintptr_t)a.data_ptr() % 16) == 0, "a: 16-B multiple, 16-B aligned");
    for (const auto* t : {&b, &o})
      if (t->has_value() && (*t)->defined()) {
        CHECK_IN(**t);
        TORCH_CHECK((*t)->numel() * (*t)->element_size() == bytes && ((uintptr_t)(*t)->data_ptr() % 16) == 0,
                    "b / o: the byte size of a, 16-B aligned");
      }
    TORCH_CHECK(kind >= 0 && kind <= 3, "kind 0..3");
    TORCH_CHECK(kind == 0 || (o.has_value() && o->defined()), "kinds 1-3 write o");
    TORCH_CHECK(kind != 3 || (b.has_value() && b->defined()), "kind 3 reads b");
    TORCH_CHECK(wgs >= 1 && wgs <= 65536, "wgs");
    c10::DeviceGuard dg(a.device());
    dtg::stream_probe((int)kind, a.data_ptr(), opt_ptr<void>(b), opt_ptr<void>(o), bytes / 16,
                      reinterpret_cast<unsigned*>(sink.data_ptr()), (int)wgs, (int)unroll, nt ? 1 : 0, cur_stream());
  }, pybind11::arg("kind"), pybind11::arg("a"), pybind11::arg("b") = pybind11::none(),
        pybind11::arg("o") = pybind11::none(), pybind11::arg("sink"), pybind11::arg("wgs") = 1024,
        pybind11::arg("unroll") = 4, pybind11::arg("nt") = false);
  m.def("launch_probe", [](int64_t grid, int64_t lds_bytes) {
    dtg::launch_probe((int)grid, (int)lds_bytes, cur_stream());
  });
  m.def("f32_to_bf16", &f32_to_bf16);
  m.def("bn_fwd_train", &bn_fwd_train);
  m.def("bn_fwd_infer", &bn_fwd_infer);
  m.def("bn_bwd", &bn_bwd, pybind11::arg("dy"), pybind11::arg("y"), pybind11::arg("x"), pybind11::arg("gamma"),
        pybind11::arg("smean"), pybind11::arg("sinv"), pybind11::arg("relu"), pybind11::arg("want_dres"),
        pybind11::arg("dgamma_acc") = pybind11::none(), pybind11::arg("dbeta_acc") = pybind11::none());
  m.def("softmax_xent", &softmax_xent);
  m.def("gemm_bn_force_cfg", [](int64_t c) { dtg::gemm_bn_force_cfg((int)c); });
  m.def("conv_force_tile", [](int64_t which, int64_t c) { dtg::conv_force_tile((int)which, (int)c); });
  m.def("conv_set_stages", [](int64_t which, int64_t s) { dtg::conv_set_stages((int)which, (int)s); });
  m.def("softmax_xent_bwd", &softmax_xent_bwd);
  m.def("gemm_pick_split", [](int64_t M, int64_t N, int64_t K, bool a_kc, int64_t target_wgs) {
    return dtg::gemm_pick_split((int)M, (int)N, (int)K, a_kc ? 1 : 0, (int)target_wgs);
  }, pybind11::arg("M"), pybind11::arg("N"), pybind11::arg("K"), pybind11::arg("a_kc") = false,
        pybind11::arg("target_wgs") = 0);
  m.def("gemm", &gemm, pybind11::arg("A"), pybind11::arg("a_kc"), pybind11::arg("B"), pybind11::arg("b_kc"),
        pybind11::arg("out"), pybind11::arg("alpha") = 1.0, pybind11::arg("beta") = 0.0,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("act") = 0, pybind11::arg("split_k") = 0,
        pybind11::arg("aux") = pybind11::none(), pybind11::arg("aux_mode") = 0,
        pybind11::arg("colsum") = pybind11::none());
  register_transformer_ops(m);
  register_pool_ops(m);
}
