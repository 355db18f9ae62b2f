// PyTorch bindings for NHWC pooling (pool.hip) and im2col/col2im (im2col.hip); registered into
// dtg._C by ops.cc.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "dtg/kernels.h"

namespace {

using at::Tensor;
using dtg::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
const bf16_t* cbfp(const Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
bf16_t* bfp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }

void check_nhwc8(const Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16, what, " must be a bf16 GPU tensor");
  TORCH_CHECK(t.dim() == 4 && t.is_contiguous(), what, " must be a contiguous [N,H,W,C] tensor");
  TORCH_CHECK(t.size(3) % 8 == 0, what, ": C % 8 == 0 required");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0, what, " must be 16-byte aligned");
}

// x: [N,H,W,C] -> (y [N,P,Q,C], argmax-in-window uint8 [N,P,Q,C])
std::vector<Tensor> maxpool_fwd(Tensor x, int64_t k, int64_t s, int64_t pad) {
  check_nhwc8(x, "x");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && pad >= 0 && pad < k, "unsupported pooling window");
  TORCH_CHECK(x.numel() / 8 < (1LL << 31), "max-pool kernels index 16-byte vectors with 32-bit math");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty output");
  c10::DeviceGuard dg(x.device());
  auto y = at::empty({N, P, Q, C}, x.options());
  auto idx = at::empty({N, P, Q, C}, x.options().dtype(at::kByte));
  dtg::maxpool_fwd(cbfp(x), bfp(y), idx.data_ptr<uint8_t>(), N, H, W, C, k, s, pad, P, Q, cur_stream());
  return {y, idx};
}

Tensor maxpool_bwd(Tensor dy, Tensor idx, int64_t H, int64_t W, int64_t k, int64_t s, int64_t pad) {
  check_nhwc8(dy, "dy");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.sizes() == dy.sizes() && idx.is_contiguous(),
              "idx must be uint8 shaped like dy");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  TORCH_CHECK((H + 2 * pad - k) / s + 1 == P && (W + 2 * pad - k) / s + 1 == Q, "pool geometry mismatch");
  TORCH_CHECK((long long)N * H * W * (C / 8) < (1LL << 31), "max-pool kernels index 16-byte vectors with 32-bit math");
  c10::DeviceGuard dg(dy.device());
  auto dx = at::empty({N, H, W, C}, dy.options());
  dtg::maxpool_bwd(cbfp(dy), idx.data_ptr<uint8_t>(), bfp(dx), N, (int)H, (int)W, C, k, s, pad, P, Q, cur_stream());
  return dx;
}

Tensor avgpool_fwd(Tensor x) {
  check_nhwc8(x, "x");
  const int N = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  c10::DeviceGuard dg(x.device());
  auto y = at::empty({N, C}, x.options());
  dtg::avgpool_fwd(cbfp(x), bfp(y), N, HW, C, cur_stream());
  return y;
}

Tensor avgpool_bwd(Tensor dy, int64_t H, int64_t W) {
  TORCH_CHECK(dy.is_cuda() && dy.scalar_type() == at::kBFloat16 && dy.dim() == 2 && dy.is_contiguous(), "dy [N,C]");
  TORCH_CHECK(dy.size(1) % 8 == 0, "C % 8 == 0 required");
  const int N = dy.size(0), C = dy.size(1);
  c10::DeviceGuard dg(dy.device());
  auto dx = at::empty({N, H, W, C}, dy.options());
  dtg::avgpool_bwd(cbfp(dy), bfp(dx), N, (int)(H * W), C, cur_stream());
  return dx;
}

// ---- fused stem tail (stem.hip) ------------------------------------------------------------------
void check_chan(const Tensor& t, int64_t C, const char* what) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == C, what,
              " must be a contiguous fp32 GPU tensor of C elements");
}

// y [N,H,W,C] (the stem conv output), part: its BN statistics partials (conv_fwd_c8 with_stats)
// -> (pooled [N,P,Q,C], argmax uint8 [N,P,Q,C], save_mean [C], save_invstd [C] [, y_am [N,P,Q,C]]); running
// stats updated.  save_yam: also return y at each window's argmax, which lets stem_bn_pool_bwd run its statistics
// pass over the pooled tensors
std::vector<Tensor> stem_bn_pool_fwd(Tensor y, Tensor part, Tensor gamma, Tensor beta, Tensor rmean, Tensor rvar,
                                     double momentum, double eps, int64_t k, int64_t s, int64_t pad, bool save_yam) {
  check_nhwc8(y, "y");
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.numel() == (long long)dtg::kBnStatSlots * 2 * C,
              "part must be the conv epilogue's [slots][2][C] fp32 partials");
  check_chan(gamma, C, "gamma");
  check_chan(beta, C, "beta");
  check_chan(rmean, C, "running_mean");
  check_chan(rvar, C, "running_var");
  TORCH_CHECK(k >= 1 && k <= 15 && s >= 1 && pad >= 0 && pad < k, "unsupported pooling window");
  TORCH_CHECK(y.numel() / 8 < (1LL << 31), "stem kernels index 16-byte vectors with 32-bit math");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty output");
  c10::DeviceGuard dg(y.device());
  auto fopt = y.options().dtype(at::kFloat);
  auto out = at::empty({N, P, Q, C}, y.options());
  auto idx = at::empty({N, P, Q, C}, y.options().dtype(at::kByte));
  auto smean = at::empty({C}, fopt), sinv = at::empty({C}, fopt), coef = at::empty({2LL * C}, fopt);
  Tensor yam;
  if (save_yam) yam = at::empty({N, P, Q, C}, y.options());
  dtg::stem_bn_pool_fwd(cbfp(y), part.data_ptr<float>(), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                        rmean.data_ptr<float>(), rvar.data_ptr<float>(), smean.data_ptr<float>(), sinv.data_ptr<float>(),
                        coef.data_ptr<float>(), bfp(out), idx.data_ptr<uint8_t>(), N, H, W, C, (int)k, (int)s, (int)pad,
                        P, Q, (float)momentum, (float)eps, cur_stream(), save_yam ? bfp(yam) : nullptr);
  if (save_yam) return {out, idx, smean, sinv, yam};
  return {out, idx, smean, sinv};
}

// x [N,H,W,C] (C <= 4, NHWC view of a channels_last image) -> [N, H+2*pad, Wp/2, 8]: the pixel-pair
// stem input (ops/conv.py stem_pairs), zero padding and packing in one pass
Tensor stem_pack_pairs(Tensor x, int64_t pad, int64_t Wp) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.is_contiguous(),
              "x must be a contiguous NHWC bf16 GPU tensor");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C >= 1 && C <= 4 && pad >= 0 && Wp % 2 == 0 && Wp >= W + pad, "bad pair-packing geometry");
  const int Hp = H + 2 * (int)pad;
  TORCH_CHECK((long long)N * Hp * Wp * 4 < (1LL << 40), "too large");
  c10::DeviceGuard dg(x.device());
  auto xp = at::empty({N, Hp, Wp / 2, 8}, x.options());
  dtg::stem_pack_pairs(cbfp(x), bfp(xp), N, H, W, C, (int)pad, Hp, (int)Wp, cur_stream());
  return xp;
}

// dout [N,P,Q,C], idx, y [N,H,W,C] -> dy [N,H,W,C] (gradient of the stem conv output); dgamma/dbeta
// accumulated into the given fp32 buffers when both are passed, else returned fresh
std::vector<Tensor> stem_bn_pool_bwd(Tensor dout, Tensor idx, Tensor y, Tensor gamma, Tensor beta, Tensor smean,
                                     Tensor sinv, int64_t k, int64_t s, int64_t pad,
                                     c10::optional<Tensor> dgamma_acc, c10::optional<Tensor> dbeta_acc,
                                     c10::optional<Tensor> yam) {
  check_nhwc8(dout, "dout");
  check_nhwc8(y, "y");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kByte && idx.sizes() == dout.sizes() && idx.is_contiguous(),
              "idx must be uint8 shaped like dout");
  const int N = y.size(0), H = y.size(1), W = y.size(2), C = y.size(3);
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(dout.size(0) == N && dout.size(1) == P && dout.size(2) == Q && dout.size(3) == C,
              "dout shape does not match the pooled geometry of y");
  TORCH_CHECK(y.numel() / 8 < (1LL << 31), "stem kernels index 16-byte vectors with 32-bit math");
  TORCH_CHECK(k <= 2 * s && pad < k, "stem backward gathers at most 2x2 windows per pixel (k <= 2*stride)");
  for (auto* t : {&gamma, &beta, &smean, &sinv}) check_chan(*t, C, "per-channel tensor");
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined() && dbeta_acc.has_value() && dbeta_acc->defined();
  const bool has_yam = yam.has_value() && yam->defined();
  if (has_yam)
    TORCH_CHECK(yam->is_cuda() && yam->scalar_type() == at::kBFloat16 && yam->sizes() == dout.sizes() &&
                    yam->is_contiguous(),
                "yam must be the forward's bf16 y-at-argmax tensor, shaped like dout");
  c10::DeviceGuard dg(y.device());
  auto fopt = y.options().dtype(at::kFloat);
  Tensor dgamma, dbeta;
  if (acc) {
    dgamma = *dgamma_acc;
    dbeta = *dbeta_acc;
    check_chan(dgamma, C, "dgamma accumulator");
    check_chan(dbeta, C, "dbeta accumulator");
  } else {
    dgamma = at::empty({C}, fopt);
    dbeta = at::empty({C}, fopt);
  }
  auto dy = at::empty_like(y);
  auto ws = at::empty({dtg::stem_bwd_workspace_floats((long long)N * H * W, C)}, fopt);
  dtg::stem_bn_pool_bwd(cbfp(dout), idx.data_ptr<uint8_t>(), cbfp(y), gamma.data_ptr<float>(), beta.data_ptr<float>(),
                        smean.data_ptr<float>(), sinv.data_ptr<float>(), bfp(dy), dgamma.data_ptr<float>(),
                        dbeta.data_ptr<float>(), acc ? 1 : 0, ws.data_ptr<float>(), N, H, W, C, (int)k, (int)s,
                        (int)pad, P, Q, cur_stream(), has_yam ? cbfp(*yam) : nullptr);
  return {dy, dgamma, dbeta};
}

// x [N,H,W,C] (any C) -> cols [N*P*Q, Kp] bf16, Kp >= R*S*C, multiple of 8
Tensor im2col(Tensor x, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t Kp) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.is_contiguous(), "x NHWC bf16");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(Kp % 8 == 0 && Kp >= R * S * C, "Kp must be >= R*S*C and a multiple of 8");
  TORCH_CHECK(stride >= 1 && pad >= 0, "bad stride/pad");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(P > 0 && Q > 0, "empty output");
  c10::DeviceGuard dg(x.device());
  auto cols = at::empty({(long long)N * P * Q, Kp}, x.options());
  dtg::im2col(cbfp(x), bfp(cols), N, H, W, C, R, S, stride, pad, Kp, cur_stream());
  return cols;
}

Tensor col2im(Tensor dcols, int64_t N, int64_t H, int64_t W, int64_t C, int64_t R, int64_t S, int64_t stride,
              int64_t pad) {
  TORCH_CHECK(dcols.is_cuda() && dcols.scalar_type() == at::kBFloat16 && dcols.dim() == 2 && dcols.is_contiguous(),
              "dcols bf16 2-D");
  const int P = (H + 2 * pad - R) / stride + 1, Q = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dcols.size(0) == N * P * Q && dcols.size(1) >= R * S * C && dcols.size(1) % 8 == 0, "dcols shape");
  c10::DeviceGuard dg(dcols.device());
  auto dx = at::empty({N, H, W, C}, dcols.options());
  dtg::col2im(cbfp(dcols), bfp(dx), N, H, W, C, R, S, stride, pad, dcols.size(1), cur_stream());
  return dx;
}

}  // namespace

void register_pool_ops(pybind11::module_& m) {
  m.def("maxpool_fwd", &maxpool_fwd);
  m.def("maxpool_bwd", &maxpool_bwd);
  m.def("avgpool_fwd", &avgpool_fwd);
  m.def("avgpool_bwd", &avgpool_bwd);
  m.def("stem_bn_pool_fwd", &stem_bn_pool_fwd, pybind11::arg("y"), pybind11::arg("part"), pybind11::arg("gamma"),
        pybind11::arg("beta"), pybind11::arg("rmean"), pybind11::arg("rvar"), pybind11::arg("momentum"),
        pybind11::arg("eps"), pybind11::arg("k"), pybind11::arg("s"), pybind11::arg("pad"),
        pybind11::arg("save_yam") = false);
  m.def("stem_pooled_stats_ok", &dtg::stem_pooled_stats_ok);
  m.def("stem_pack_pairs", &stem_pack_pairs, pybind11::arg("x"), pybind11::arg("pad"), pybind11::arg("Wp"));
  m.def("stem_bn_pool_bwd", &stem_bn_pool_bwd, pybind11::arg("dout"), pybind11::arg("idx"), pybind11::arg("y"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("smean"), pybind11::arg("sinv"),
        pybind11::arg("k"), pybind11::arg("s"), pybind11::arg("pad"), pybind11::arg("dgamma_acc") = pybind11::none(),
        pybind11::arg("dbeta_acc") = pybind11::none(), pybind11::arg("yam") = pybind11::none());
  m.def("im2col", &im2col);
  m.def("col2im", &col2im);
}
