// PyTorch bindings of the GEMM / conv lab kernels (module dtg._lab, built only by tools/build_ext.py --only lab and
// imported through dtg.ops._native.lab()): A/B candidates and negative results that are not part of the production
// extension _C -- the 256x256 8-phase GEMMs (gemm8.hip), the forced tile table (gemm_forced*.hip), the round-5
// main-loop lab (gemm5.hip) and the transposed fused BN dx + weight gradient (bn_dxT_wgrad.hip).  (The round-3 halo
// conv fork was retired in round 6: the production csrc/kernels/conv_halo.hip is the one tested and benchmarked.)
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "lab_api.h"

namespace dtg {
namespace lab {
int gemm5_bf16(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, int sched, hipStream_t st);
int gemm5p_bf16(const bf16_t* A, const bf16_t* B, void* C, int c_bf16, int M, int N, int K, const float* bias, int act,
                void* aux, int aux_mode, hipStream_t st, int grid);
int bn_dxT_wgrad_slabs(int C, int CI);
bool bn_dxT_wgrad(const bf16_t* dp, const bf16_t* x, const float* coef, bf16_t* dx, const bf16_t* act,
                  long long ldact, float* wgrad, float* slabs, long long M, int C, int CI, hipStream_t st);
}  // namespace lab
}  // namespace dtg

namespace {
using at::Tensor;
using dtg::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
const bf16_t* cbfp(const Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
bf16_t* bfp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }

// BN1 dx pass + conv1 weight gradient (bn_dxT_wgrad.hip): dx = a * dp + bx * x + c per channel (coef = [a, bx, c],
// fp32 [3 C]), wgrad (fp32 [C, CI]) += dx^T act; returns dx.  C x CI = 64 x 256, 128 x 256 or 128 x 512.
Tensor bn_dxT_wgrad(Tensor dp, Tensor x, Tensor coef, Tensor act, Tensor wgrad) {
  for (const Tensor* t : {&dp, &x, &act})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() && t->dim() == 2, "bf16 [M, *]");
  TORCH_CHECK(coef.is_cuda() && coef.scalar_type() == at::kFloat && coef.is_contiguous(), "coef fp32");
  TORCH_CHECK(wgrad.is_cuda() && wgrad.scalar_type() == at::kFloat && wgrad.is_contiguous(), "wgrad fp32");
  const long long M = x.size(0);
  const int C = (int)x.size(1), CI = (int)act.size(1);
  TORCH_CHECK(dp.sizes() == x.sizes() && act.size(0) == M && coef.numel() == 3LL * C && wgrad.numel() == (long long)C * CI,
              "shapes: dp, x [M, C], act [M, CI], coef [3 C], wgrad [C, CI]");
  const int ns = dtg::lab::bn_dxT_wgrad_slabs(C, CI);
  TORCH_CHECK(ns > 0, "C x CI = 64 x 256, 128 x 256 or 128 x 512");
  c10::DeviceGuard dg(x.device());
  auto dx = at::empty_like(x);
  auto slabs = at::empty({(long long)ns * C * CI}, x.options().dtype(at::kFloat));
  TORCH_CHECK(dtg::lab::bn_dxT_wgrad(cbfp(dp), cbfp(x), coef.data_ptr<float>(), bfp(dx), cbfp(act), act.stride(0),
                                     wgrad.data_ptr<float>(), slabs.data_ptr<float>(), M, C, CI, cur_stream()),
              "rows: a multiple of 32, at least 2048");
  return dx;
}

// out[M, N] = A[M, K] B[N, K]^T (bf16, contiguous); false if the shape is not one the kernel serves
bool gemm5(Tensor A, Tensor B, Tensor out, int64_t sched) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && out.is_cuda(), "GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16 &&
                  out.scalar_type() == at::kBFloat16, "bf16");
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && out.dim() == 2 && A.size(1) == B.size(1) && out.size(0) == A.size(0) &&
                  out.size(1) == B.size(0), "shapes A[M,K] B[N,K] out[M,N]");
  c10::DeviceGuard dg(A.device());
  return dtg::lab::gemm5_bf16(cbfp(A), cbfp(B), bfp(out), A.size(0), B.size(0), A.size(1), (int)sched,
                              cur_stream()) != 0;
}

// persistent v5 (C = A B^T, A [M,K], B [N,K]) with the production epilogue arguments; false if the shape is not
// served (M % 256, N % 192, K % 64)
bool gemm5p(Tensor A, Tensor B, Tensor out, c10::optional<Tensor> bias, int64_t act, c10::optional<Tensor> aux,
            int64_t aux_mode, int64_t grid) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && out.is_cuda(), "GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "bf16 operands");
  TORCH_CHECK(out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat, "out bf16 / fp32");
  TORCH_CHECK(A.is_contiguous() && B.is_contiguous() && out.is_contiguous(), "contiguous");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && out.dim() == 2 && A.size(1) == B.size(1) && out.size(0) == A.size(0) &&
                  out.size(1) == B.size(0), "shapes A[M,K] B[N,K] out[M,N]");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->scalar_type() == at::kFloat &&
                    bias->numel() == out.size(1), "bias fp32 [N]");
    bptr = bias->data_ptr<float>();
  }
  void* auxp = nullptr;
  if (aux_mode != 0) {
    TORCH_CHECK(aux.has_value() && aux->defined() && aux->sizes() == out.sizes() && aux->is_contiguous() &&
                    aux->scalar_type() == at::kBFloat16, "aux bf16 like out");
    auxp = aux->data_ptr();
  }
  c10::DeviceGuard dg(A.device());
  return dtg::lab::gemm5p_bf16(cbfp(A), cbfp(B), out.data_ptr(), out.scalar_type() == at::kBFloat16, A.size(0),
                               B.size(0), A.size(1), bptr, (int)act, auxp, (int)aux_mode, cur_stream(),
                               (int)grid) != 0;
}

// gemm (the production binding's operand conventions) through forced configuration `cfg`; false if the
// configuration does not apply to this problem
bool gemm_cfg(int64_t cfg, Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor out, double alpha, double beta,
              c10::optional<Tensor> bias, int64_t act, int64_t split_k, c10::optional<Tensor> aux, int64_t aux_mode) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && out.is_cuda(), "GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "bf16 operands");
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && out.dim() == 2, "2-D operands");
  TORCH_CHECK(A.stride(1) == 1 && B.stride(1) == 1 && out.stride(1) == 1, "inner dim must be contiguous");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out fp32/bf16");
  const int M = (int)(a_kc ? A.size(0) : A.size(1)), K = (int)(a_kc ? A.size(1) : A.size(0));
  const int N = (int)(b_kc ? B.size(0) : B.size(1)), Kb = (int)(b_kc ? B.size(1) : B.size(0));
  TORCH_CHECK(K == Kb && out.size(0) == M && out.size(1) == N, "shape mismatch");
  TORCH_CHECK(K % 8 == 0 || (!a_kc && !b_kc), "K-contiguous operands need K % 8 == 0");
  TORCH_CHECK((a_kc || M % 8 == 0) && (b_kc || N % 8 == 0), "K-major operands need 8-multiples");
  TORCH_CHECK(A.stride(0) % 8 == 0 && B.stride(0) % 8 == 0, "row strides must be 16-byte multiples");
  TORCH_CHECK(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0, "16-byte alignment");
  const float* bptr = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->is_contiguous() && bias->scalar_type() == at::kFloat && bias->numel() == N,
                "bias: fp32 [N]");
    bptr = bias->data_ptr<float>();
  }
  void* auxp = nullptr;
  if (aux_mode != 0) {
    TORCH_CHECK(aux_mode >= 1 && aux_mode <= 4 && aux.has_value() && aux->defined(), "aux_mode needs aux");
    TORCH_CHECK(aux->is_cuda() && aux->scalar_type() == at::kBFloat16 && aux->dim() == 2 && aux->size(0) == M &&
                    aux->size(1) == N && aux->stride(0) == out.stride(0) && aux->stride(1) == 1, "aux like out");
    auxp = aux->data_ptr();
  }
  c10::DeviceGuard dg(A.device());
  int sk = split_k > 0 ? (int)split_k : 1;
  Tensor ws;
  float* wsp = nullptr;
  if (sk > 1) {
    ws = at::empty({(long long)sk * M * N}, A.options().dtype(at::kFloat));
    wsp = ws.data_ptr<float>();
  }
  return dtg::gemm_lab_cfg((int)cfg, cbfp(A), A.stride(0), a_kc, cbfp(B), B.stride(0), b_kc, out.data_ptr(),
                           out.stride(0), out.scalar_type() == at::kBFloat16, M, N, K, (float)alpha, (float)beta, bptr,
                           (int)act, sk, wsp, cur_stream(), auxp, (int)aux_mode);
}

}  // namespace

PYBIND11_MODULE(_lab, m) {
  m.doc() = "dtg GEMM / conv lab kernels (A/B tools only, not part of the production extension)";
  m.def("gemm5", &gemm5, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("out"), pybind11::arg("sched") = 1);
  m.def("gemm5p", &gemm5p, pybind11::arg("A"), pybind11::arg("B"), pybind11::arg("out"),
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("act") = 0, pybind11::arg("aux") = pybind11::none(),
        pybind11::arg("aux_mode") = 0, pybind11::arg("grid") = 0);
  m.def("gemm_cfg", &gemm_cfg, pybind11::arg("cfg"), pybind11::arg("A"), pybind11::arg("a_kc"), pybind11::arg("B"),
        pybind11::arg("b_kc"), pybind11::arg("out"), pybind11::arg("alpha") = 1.0, pybind11::arg("beta") = 0.0,
        pybind11::arg("bias") = pybind11::none(), pybind11::arg("act") = 0, pybind11::arg("split_k") = 1,
        pybind11::arg("aux") = pybind11::none(), pybind11::arg("aux_mode") = 0);
  m.def("bn_dxT_wgrad", &bn_dxT_wgrad, pybind11::arg("dp"), pybind11::arg("x"), pybind11::arg("coef"),
        pybind11::arg("act"), pybind11::arg("wgrad"));
}
