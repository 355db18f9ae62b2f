// PyTorch bindings for the transformer kernels (transformer.hip) and the strided-batched GEMM.
// Registered into dtg._C by ops.cc (register_transformer_ops).  Every wrapper checks shapes,
// dtypes, alignment and -- for the raw-stride batched GEMM -- that the furthest element each
// operand touches lies inside its storage, before anything is launched.
#include <torch/extension.h>
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>

#include "dtg/kernels.h"

namespace {

using at::Tensor;
using dtg::bf16_t;

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }
bf16_t* bfp(const Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
const bf16_t* cbfp(const Tensor& t) { return reinterpret_cast<const bf16_t*>(t.data_ptr()); }
bool has(const c10::optional<Tensor>& t) { return t.has_value() && t->defined(); }

#define CHECK_GPU_BF16_CONTIG(x)                                               \
  TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor");                      \
  TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16");         \
  TORCH_CHECK((x).is_contiguous(), #x " must be contiguous");                  \
  TORCH_CHECK(((uintptr_t)(x).data_ptr() % 16) == 0, #x " must be 16-byte aligned")

#define CHECK_F32_CONTIG(x)                                                   \
  TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor");                     \
  TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be fp32");           \
  TORCH_CHECK((x).is_contiguous(), #x " must be contiguous");                 \
  TORCH_CHECK(((uintptr_t)(x).data_ptr() % 16) == 0, #x " must be 16-byte aligned")

// number of elements addressable from t.data_ptr() to the end of its storage
long long room(const Tensor& t) {
  return (long long)(t.storage().nbytes() / t.element_size()) - (long long)t.storage_offset();
}

// ---- strided batched GEMM ------------------------------------------------------------------------
// For z = zb*nh + zh (zb < nb, zh < nh): C_z = alpha * op(A_z) op(B_z) + beta * C_z with
// A_z = A + zb*sa_b + zh*sa_h (elements), etc.  Layout flags as in dtg._C.gemm.
void gemm_strided_batched(Tensor A, bool a_kc, Tensor B, bool b_kc, Tensor C, int64_t M, int64_t N, int64_t K,
                          int64_t lda, int64_t ldb, int64_t ldc, int64_t nb, int64_t nh, int64_t sa_b, int64_t sa_h,
                          int64_t sb_b, int64_t sb_h, int64_t sc_b, int64_t sc_h, double alpha, double beta) {
  TORCH_CHECK(A.is_cuda() && B.is_cuda() && C.is_cuda(), "operands must be GPU tensors");
  TORCH_CHECK(A.scalar_type() == at::kBFloat16 && B.scalar_type() == at::kBFloat16, "A, B must be bf16");
  TORCH_CHECK(C.scalar_type() == at::kFloat || C.scalar_type() == at::kBFloat16, "C must be fp32/bf16");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && nb > 0 && nh > 0, "empty problem");
  TORCH_CHECK(nb * nh < 65536, "too many batched problems");
  TORCH_CHECK(K % 8 == 0, "K % 8 == 0 required");
  TORCH_CHECK(a_kc || M % 8 == 0, "K-major A needs M % 8 == 0");
  TORCH_CHECK(b_kc || N % 8 == 0, "K-major B needs N % 8 == 0");
  for (long long s : {lda, ldb, sa_b, sa_h, sb_b, sb_h}) TORCH_CHECK(s % 8 == 0, "A/B strides must be multiples of 8");
  TORCH_CHECK(((uintptr_t)A.data_ptr() % 16) == 0 && ((uintptr_t)B.data_ptr() % 16) == 0, "16-byte alignment");
  TORCH_CHECK(lda >= (a_kc ? K : M) && ldb >= (b_kc ? K : N) && ldc >= N, "leading dimension too small");
  const long long a_ext = (nb - 1) * sa_b + (nh - 1) * sa_h + (a_kc ? (M - 1) * lda + K : (K - 1) * lda + M);
  const long long b_ext = (nb - 1) * sb_b + (nh - 1) * sb_h + (b_kc ? (N - 1) * ldb + K : (K - 1) * ldb + N);
  const long long c_ext = (nb - 1) * sc_b + (nh - 1) * sc_h + (M - 1) * ldc + N;
  TORCH_CHECK(a_ext <= room(A), "A: batched extent exceeds storage");
  TORCH_CHECK(b_ext <= room(B), "B: batched extent exceeds storage");
  TORCH_CHECK(c_ext <= room(C), "C: batched extent exceeds storage");
  c10::DeviceGuard dg(A.device());
  dtg::GemmBatch bt;
  bt.count = (int)(nb * nh);
  bt.nh = (int)nh;
  bt.sa_b = sa_b; bt.sa_h = sa_h; bt.sb_b = sb_b; bt.sb_h = sb_h; bt.sc_b = sc_b; bt.sc_h = sc_h;
  dtg::gemm_bf16(cbfp(A), lda, a_kc, cbfp(B), ldb, b_kc, C.data_ptr(), ldc, C.scalar_type() == at::kBFloat16,
                 (int)M, (int)N, (int)K, (float)alpha, (float)beta, nullptr, 0, 1, nullptr, cur_stream(), bt);
}

// ---- LayerNorm -----------------------------------------------------------------------------------------
void check_ln(const Tensor& x, int64_t H) {
  CHECK_GPU_BF16_CONTIG(x);
  TORCH_CHECK(x.dim() == 2 && x.size(1) == H, "expected [T, H]");
}

std::vector<c10::optional<Tensor>> ln_fwd(Tensor h, c10::optional<Tensor> res, Tensor gamma, Tensor beta, double eps,
                                          double p_in, int64_t seed_in, double p_out, int64_t seed_out,
                                          bool save_s) {
  const int64_t H = h.size(-1);
  check_ln(h, H);
  TORCH_CHECK(H % 8 == 0 && H <= dtg::ln_max_hidden(), "hidden size must be a multiple of 8 and <= ",
              dtg::ln_max_hidden());
  if (has(res)) {
    check_ln(*res, H);
    TORCH_CHECK(res->size(0) == h.size(0), "residual rows mismatch");
  }
  CHECK_F32_CONTIG(gamma);
  CHECK_F32_CONTIG(beta);
  TORCH_CHECK(gamma.numel() == H && beta.numel() == H, "gamma/beta size mismatch");
  TORCH_CHECK(p_in >= 0 && p_in < 1 && p_out >= 0 && p_out < 1, "dropout prob in [0, 1)");
  c10::DeviceGuard dg(h.device());
  const int T = (int)h.size(0);
  auto y = at::empty_like(h);
  c10::optional<Tensor> s;
  if (save_s) s = at::empty_like(h);
  auto fo = h.options().dtype(at::kFloat);
  auto mean = at::empty({T}, fo), rstd = at::empty({T}, fo);
  dtg::ln_fwd(cbfp(h), has(res) ? cbfp(*res) : nullptr, gamma.data_ptr<float>(), beta.data_ptr<float>(), bfp(y),
              save_s ? bfp(*s) : nullptr, mean.data_ptr<float>(), rstd.data_ptr<float>(), T, (int)H, (float)eps,
              (float)p_in, (uint32_t)seed_in, (float)p_out, (uint32_t)seed_out, cur_stream());
  return {y, s, mean, rstd};
}

// returns (ds, dh): ds = grad wrt s (residual path), dh = grad wrt the dropout input (if want_dh)
std::vector<c10::optional<Tensor>> ln_bwd(Tensor dy, Tensor s, Tensor gamma, Tensor mean, Tensor rstd,
                                          Tensor dgamma, Tensor dbeta, double p_in, int64_t seed_in, double p_out,
                                          int64_t seed_out, bool want_dh, c10::optional<Tensor> dbias) {
  const int64_t H = s.size(-1);
  check_ln(dy, H);
  check_ln(s, H);
  TORCH_CHECK(dy.size(0) == s.size(0), "dy/s rows mismatch");
  TORCH_CHECK(H % 8 == 0 && H <= dtg::ln_max_hidden(), "unsupported hidden size");
  CHECK_F32_CONTIG(gamma);
  CHECK_F32_CONTIG(mean);
  CHECK_F32_CONTIG(rstd);
  CHECK_F32_CONTIG(dgamma);
  CHECK_F32_CONTIG(dbeta);
  const int T = (int)s.size(0);
  TORCH_CHECK(mean.numel() == T && rstd.numel() == T, "stats size mismatch");
  TORCH_CHECK(gamma.numel() == H && dgamma.numel() == H && dbeta.numel() == H, "param size mismatch");
  if (has(dbias)) {
    CHECK_F32_CONTIG(*dbias);
    TORCH_CHECK(dbias->numel() == H, "dbias size mismatch");
  }
  c10::DeviceGuard dg(s.device());
  auto ds = at::empty_like(s);
  auto ws = at::empty({(long long)dtg::ln_bwd_blocks(T) * 3 * H}, s.options().dtype(at::kFloat));
  c10::optional<Tensor> dh;
  if (want_dh) dh = p_in > 0 ? at::empty_like(s) : ds;
  dtg::ln_bwd(cbfp(dy), cbfp(s), gamma.data_ptr<float>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), bfp(ds),
              (want_dh && p_in > 0) ? bfp(*dh) : nullptr, dgamma.data_ptr<float>(), dbeta.data_ptr<float>(),
              has(dbias) ? dbias->data_ptr<float>() : nullptr, ws.data_ptr<float>(), T, (int)H, (float)p_in, (uint32_t)seed_in, (float)p_out, (uint32_t)seed_out,
              cur_stream());
  return {ds, dh};
}

// ---- attention softmax ------------------------------------------------------------------------------------
// scores: fp32 [rows, Sk] (already scaled); mask: fp32 [B, Sk] additive, row r uses mask[r / rows_per_b]
std::vector<Tensor> attn_softmax_fwd(Tensor scores, c10::optional<Tensor> mask, int64_t rows_per_b, double p,
                                     int64_t seed) {
  CHECK_F32_CONTIG(scores);
  TORCH_CHECK(scores.dim() == 2, "scores must be [rows, Sk]");
  const int rows = (int)scores.size(0), Sk = (int)scores.size(1);
  TORCH_CHECK(Sk <= dtg::attn_max_keys(), "too many keys");
  TORCH_CHECK(p >= 0 && p < 1, "dropout prob in [0, 1)");
  if (has(mask)) {
    CHECK_F32_CONTIG(*mask);
    TORCH_CHECK(mask->dim() == 2 && mask->size(1) == Sk, "mask must be [B, Sk]");
    TORCH_CHECK(rows_per_b > 0 && (long long)mask->size(0) * rows_per_b == rows, "mask batch mismatch");
  }
  c10::DeviceGuard dg(scores.device());
  auto P = at::empty({rows, Sk}, scores.options().dtype(at::kBFloat16));
  Tensor Pd = p > 0 ? at::empty_like(P) : P;
  dtg::attn_softmax_fwd(scores.data_ptr<float>(), has(mask) ? mask->data_ptr<float>() : nullptr, bfp(P), bfp(Pd),
                        rows, (int)(rows_per_b > 0 ? rows_per_b : rows), Sk, (float)p, (uint32_t)seed, cur_stream());
  return {P, Pd};
}

Tensor attn_softmax_bwd(Tensor P, Tensor Pd, Tensor dPd, double scale) {
  TORCH_CHECK(P.is_cuda() && P.scalar_type() == at::kBFloat16 && P.is_contiguous() && P.dim() == 2, "P");
  TORCH_CHECK(Pd.sizes() == P.sizes() && Pd.scalar_type() == at::kBFloat16 && Pd.is_contiguous(), "Pd");
  CHECK_F32_CONTIG(dPd);
  TORCH_CHECK(dPd.sizes() == P.sizes(), "dPd shape");
  TORCH_CHECK(P.size(1) <= dtg::attn_max_keys(), "too many keys");
  c10::DeviceGuard dg(P.device());
  auto dS = at::empty_like(P);
  dtg::attn_softmax_bwd(cbfp(P), cbfp(Pd), dPd.data_ptr<float>(), bfp(dS), (int)P.size(0), (int)P.size(1),
                        (float)scale, cur_stream());
  return dS;
}

// ---- column sums -------------------------------------------------------------------------------------------
// out[v, n] (+)= sum_{t: sel[t]==v} x[t, n]; x bf16 [T, N] (row stride x.stride(0)), out fp32/bf16 [nsel*N]
void colsum(Tensor x, Tensor out, bool accumulate, c10::optional<Tensor> sel, int64_t nsel) {
  TORCH_CHECK(x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 2 && x.stride(1) == 1, "x");
  TORCH_CHECK(x.stride(0) % 8 == 0 && x.size(1) % 8 == 0 && ((uintptr_t)x.data_ptr() % 16) == 0,
              "x needs 16-byte rows (N % 8 == 0)");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous(), "out");
  TORCH_CHECK(out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16, "out fp32/bf16");
  const int T = (int)x.size(0), N = (int)x.size(1);
  TORCH_CHECK(nsel == 1 || nsel == 2, "nsel in {1, 2}");
  TORCH_CHECK(out.numel() == nsel * N, "out size mismatch");
  if (has(sel)) {
    TORCH_CHECK(sel->is_cuda() && sel->scalar_type() == at::kLong && sel->is_contiguous() && sel->numel() == T,
                "sel must be int64 [T]");
  } else {
    TORCH_CHECK(nsel == 1, "nsel > 1 needs a selector");
  }
  c10::DeviceGuard dg(x.device());
  const int splits = dtg::colsum_splits(T, N);
  auto ws = at::empty({(long long)splits * nsel * N}, x.options().dtype(at::kFloat));
  dtg::colsum(cbfp(x), x.stride(0), T, N, has(sel) ? reinterpret_cast<const long long*>(sel->data_ptr<int64_t>()) : nullptr,
              (int)nsel, out.data_ptr(), out.scalar_type() == at::kBFloat16, accumulate, ws.data_ptr<float>(), splits,
              cur_stream());
}

// ---- embeddings ----------------------------------------------------------------------------------------------
Tensor emb_fwd(Tensor ids, c10::optional<Tensor> tt, Tensor word, Tensor pos, Tensor type, int64_t S) {
  TORCH_CHECK(ids.is_cuda() && ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids int64");
  CHECK_GPU_BF16_CONTIG(word);
  CHECK_GPU_BF16_CONTIG(pos);
  CHECK_GPU_BF16_CONTIG(type);
  const int64_t H = word.size(1);
  TORCH_CHECK(H % 8 == 0 && pos.size(1) == H && type.size(1) == H, "embedding widths");
  const int T = (int)ids.numel();
  TORCH_CHECK(S > 0 && T % S == 0 && S <= pos.size(0), "sequence length vs position table");
  if (has(tt)) TORCH_CHECK(tt->is_cuda() && tt->scalar_type() == at::kLong && tt->is_contiguous() && tt->numel() == T,
                           "token types int64 [T]");
  c10::DeviceGuard dg(ids.device());
  auto s = at::empty({T, H}, word.options());
  dtg::emb_fwd(reinterpret_cast<const long long*>(ids.data_ptr<int64_t>()),
               has(tt) ? reinterpret_cast<const long long*>(tt->data_ptr<int64_t>()) : nullptr, cbfp(word), cbfp(pos),
               cbfp(type), bfp(s), T, (int)S, (int)H, cur_stream());
  return s;
}

// gW[sorted[i]] += ds[perm[i]]; sorted ascending (torch.sort of the ids), values < V unchecked on device:
// the caller guarantees ids are in range (checked once per batch by the model).
void emb_word_bwd(Tensor ds, Tensor sorted, Tensor perm, Tensor gW) {
  CHECK_GPU_BF16_CONTIG(ds);
  CHECK_GPU_BF16_CONTIG(gW);
  TORCH_CHECK(sorted.scalar_type() == at::kLong && perm.scalar_type() == at::kLong && sorted.is_contiguous() &&
                  perm.is_contiguous(), "sorted/perm int64");
  const int T = (int)ds.size(0), H = (int)ds.size(1);
  TORCH_CHECK(sorted.numel() == T && perm.numel() == T && gW.size(1) == H, "shape mismatch");
  c10::DeviceGuard dg(ds.device());
  dtg::emb_word_bwd(cbfp(ds), reinterpret_cast<const long long*>(sorted.data_ptr<int64_t>()),
                    reinterpret_cast<const long long*>(perm.data_ptr<int64_t>()), bfp(gW), T, H, cur_stream());
}

void emb_pos_bwd(Tensor ds, Tensor gP, int64_t S) {
  CHECK_GPU_BF16_CONTIG(ds);
  CHECK_GPU_BF16_CONTIG(gP);
  const int T = (int)ds.size(0), H = (int)ds.size(1);
  TORCH_CHECK(S > 0 && T % S == 0 && gP.size(0) >= S && gP.size(1) == H, "shape mismatch");
  c10::DeviceGuard dg(ds.device());
  dtg::emb_pos_bwd(cbfp(ds), bfp(gP), T, (int)S, H, cur_stream());
}

// ---- fused attention (attention.hip) ---------------------------------------------------------------
// qkv [B*S, 3H] bf16 ([Q | K | V], head h at columns h*64 of each); mask fp32 [B, S] additive or None
std::vector<Tensor> attn_fused_fwd(Tensor qkv, c10::optional<Tensor> mask, int64_t B, int64_t S, int64_t nh, double p,
                                   int64_t seed) {
  CHECK_GPU_BF16_CONTIG(qkv);
  TORCH_CHECK(dtg::attn_fused_supported((int)S, 64, 0), "fused attention: S % 64 == 0 and S <= 512 required");
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(0) == B * S && qkv.size(1) == 3 * nh * 64, "qkv must be [B*S, 3*nh*64]");
  TORCH_CHECK(p >= 0 && p < 1, "dropout prob in [0, 1)");
  if (has(mask)) {
    CHECK_F32_CONTIG(*mask);
    TORCH_CHECK(mask->numel() == B * S, "mask must be [B, S]");
  }
  c10::DeviceGuard dg(qkv.device());
  auto out = at::empty({B * S, nh * 64}, qkv.options());
  auto lse = at::empty({B * nh * S}, qkv.options().dtype(at::kFloat));
  dtg::attn_fwd(cbfp(qkv), has(mask) ? mask->data_ptr<float>() : nullptr, bfp(out), lse.data_ptr<float>(), (int)B,
                (int)S, (int)nh, (float)p, (uint32_t)seed, cur_stream());
  return {out, lse};
}

// dbias (optional, fp32 [3 * nh * 64]): the QKV bias gradient is ADDED into it by the kernel's epilogue
Tensor attn_fused_bwd(Tensor qkv, Tensor out, Tensor dout, Tensor lse, c10::optional<Tensor> mask, int64_t B,
                      int64_t S, int64_t nh, double p, int64_t seed, c10::optional<Tensor> dbias) {
  CHECK_GPU_BF16_CONTIG(qkv);
  CHECK_GPU_BF16_CONTIG(out);
  CHECK_GPU_BF16_CONTIG(dout);
  CHECK_F32_CONTIG(lse);
  TORCH_CHECK(dtg::attn_fused_supported((int)S, 64, 1), "fused attention backward: S % 64 == 0 and S <= 512");
  TORCH_CHECK(qkv.size(0) == B * S && qkv.size(1) == 3 * nh * 64, "qkv shape");
  TORCH_CHECK(out.sizes() == dout.sizes() && out.size(0) == B * S && out.size(1) == nh * 64, "out/dout shape");
  TORCH_CHECK(lse.numel() == B * nh * S, "lse size");
  if (has(mask)) {
    CHECK_F32_CONTIG(*mask);
    TORCH_CHECK(mask->numel() == B * S, "mask must be [B, S]");
  }
  if (has(dbias)) {
    CHECK_F32_CONTIG(*dbias);
    TORCH_CHECK(dbias->numel() == 3 * nh * 64 && dbias->device() == qkv.device(), "dbias must be fp32 [3 * nh * 64]");
  }
  c10::DeviceGuard dg(qkv.device());
  auto dqkv = at::empty_like(qkv);
  dtg::attn_bwd(cbfp(qkv), cbfp(out), cbfp(dout), lse.data_ptr<float>(), has(mask) ? mask->data_ptr<float>() : nullptr,
                bfp(dqkv), (int)B, (int)S, (int)nh, (float)p, (uint32_t)seed,
                has(dbias) ? dbias->data_ptr<float>() : nullptr, cur_stream());
  return dqkv;
}

}  // namespace

namespace py = pybind11;


// ---- BERT heads (heads.hip) -------------------------------------------------------------------------
static const long long* i64p(const Tensor& t) { return reinterpret_cast<const long long*>(t.data_ptr<int64_t>()); }

// rows of src [B*S, H] at (i / P) * S + pos[i] -> [B*P, H]
Tensor gather_rows(Tensor src, Tensor pos, int64_t S) {
  CHECK_GPU_BF16_CONTIG(src);
  TORCH_CHECK(pos.scalar_type() == at::kLong && pos.is_contiguous() && pos.dim() == 2, "pos: [B, P] int64");
  const int H = (int)src.size(1), P = (int)pos.size(1), R = (int)pos.numel();
  TORCH_CHECK(H % 8 == 0 && src.size(0) == pos.size(0) * S, "gather_rows shape mismatch");
  c10::DeviceGuard dg(src.device());
  Tensor out = at::empty({R, H}, src.options());
  dtg::gather_rows(cbfp(src), i64p(pos), bfp(out), R, P, (int)S, H, cur_stream());
  return out;
}

// dst rows (i / P) * S + pos[i] += src[i]; without pos: dst rows i * S (the [CLS] rows) += src[i]
void scatter_rows_add(Tensor dst, c10::optional<Tensor> pos, Tensor src, int64_t S) {
  CHECK_GPU_BF16_CONTIG(dst);
  CHECK_GPU_BF16_CONTIG(src);
  const int H = (int)dst.size(1), R = (int)src.size(0);
  TORCH_CHECK(src.size(1) == H && H % 8 == 0, "scatter_rows_add width mismatch");
  int P = 1;
  if (has(pos)) {
    TORCH_CHECK(pos->scalar_type() == at::kLong && pos->is_contiguous() && pos->dim() == 2 && pos->numel() == R,
                "pos: [B, P] int64");
    P = (int)pos->size(1);
    TORCH_CHECK(dst.size(0) == pos->size(0) * S, "scatter_rows_add rows");
  } else {
    TORCH_CHECK(dst.size(0) == (int64_t)R * S, "scatter_rows_add rows");
  }
  c10::DeviceGuard dg(dst.device());
  dtg::scatter_rows_add(bfp(dst), has(pos) ? i64p(*pos) : nullptr, cbfp(src), R, P, (int)S, H, cur_stream());
}

// -> (total loss [] fp32 = mean NSP cross-entropy + extra, softmax probabilities [B, 2] fp32)
std::vector<Tensor> nsp_loss_fwd(Tensor pooled, Tensor wn, Tensor bn, Tensor labels, c10::optional<Tensor> extra) {
  CHECK_GPU_BF16_CONTIG(pooled);
  CHECK_GPU_BF16_CONTIG(wn);
  CHECK_F32_CONTIG(bn);
  const int B = (int)pooled.size(0), H = (int)pooled.size(1);
  TORCH_CHECK(wn.size(0) == 2 && wn.size(1) == H && bn.numel() == 2 && H % 8 == 0, "NSP head is [2, H]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.numel() == B, "labels [B] int64");
  if (has(extra)) CHECK_F32_CONTIG(*extra);
  c10::DeviceGuard dg(pooled.device());
  Tensor probs = at::empty({B, 2}, pooled.options().dtype(at::kFloat));
  Tensor out = at::empty({}, pooled.options().dtype(at::kFloat));
  dtg::nsp_loss_fwd(cbfp(pooled), cbfp(wn), bn.data_ptr<float>(), i64p(labels),
                    has(extra) ? extra->data_ptr<float>() : nullptr, probs.data_ptr<float>(), out.data_ptr<float>(), B,
                    H, cur_stream());
  return {out, probs};
}

// -> dpre [B, H] bf16 (gradient before the pooler's tanh); accumulates gwn (bf16 [2, H]) and gbn (fp32 [2])
Tensor nsp_loss_bwd(Tensor pooled, Tensor wn, Tensor probs, Tensor labels, Tensor gout, Tensor gwn, Tensor gbn) {
  CHECK_GPU_BF16_CONTIG(pooled);
  CHECK_GPU_BF16_CONTIG(wn);
  CHECK_GPU_BF16_CONTIG(gwn);
  CHECK_F32_CONTIG(probs);
  CHECK_F32_CONTIG(gout);
  CHECK_F32_CONTIG(gbn);
  const int B = (int)pooled.size(0), H = (int)pooled.size(1);
  TORCH_CHECK(gwn.numel() == 2 * H && gbn.numel() == 2 && probs.numel() == 2 * B && labels.numel() == B, "shapes");
  c10::DeviceGuard dg(pooled.device());
  Tensor dpre = at::empty_like(pooled);
  dtg::nsp_loss_bwd(cbfp(pooled), cbfp(wn), probs.data_ptr<float>(), i64p(labels), gout.data_ptr<float>(), bfp(dpre),
                    bfp(gwn), gbn.data_ptr<float>(), B, H, cur_stream());
  return dpre;
}

Tensor row_sum(Tensor x, double scale) {
  CHECK_F32_CONTIG(x);
  c10::DeviceGuard dg(x.device());
  Tensor out = at::empty({}, x.options());
  dtg::row_sum(x.data_ptr<float>(), out.data_ptr<float>(), x.numel(), (float)scale, cur_stream());
  return out;
}

// sort-free word-embedding gradient: gW[ids[t]] += ds[t] (vocab rows owned per workgroup, token order)
bool emb_word_bwd_owned(Tensor ds, Tensor ids, Tensor gW) {
  CHECK_GPU_BF16_CONTIG(ds);
  CHECK_GPU_BF16_CONTIG(gW);
  TORCH_CHECK(ids.scalar_type() == at::kLong && ids.is_contiguous(), "ids int64");
  const int T = (int)ds.size(0), H = (int)ds.size(1), V = (int)gW.size(0);
  TORCH_CHECK(ids.numel() == T && gW.size(1) == H && H % 8 == 0, "shape mismatch");
  if ((long long)32 * H * 4 > 131072) return false;  // accumulator tile does not fit LDS: caller sorts instead
  c10::DeviceGuard dg(ds.device());
  dtg::emb_word_bwd_owned(cbfp(ds), i64p(ids), bfp(gW), T, H, V, cur_stream());
  return true;
}

// stream-ordered zero fill on a dtg kernel (no framework or runtime fill kernel)
void zero_(Tensor t) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "zero_: contiguous GPU tensor");
  TORCH_CHECK(((uintptr_t)t.data_ptr() % 16) == 0, "zero_: 16-byte aligned tensor");
  c10::DeviceGuard dg(t.device());
  dtg::fill_zero(t.data_ptr(), t.numel() * t.element_size(), cur_stream());
}

Tensor mul_bf16(Tensor a, Tensor b) {
  CHECK_GPU_BF16_CONTIG(a);
  CHECK_GPU_BF16_CONTIG(b);
  TORCH_CHECK(a.sizes() == b.sizes(), "mul_bf16 shape mismatch");
  TORCH_CHECK(((uintptr_t)a.data_ptr() % 16) == 0 && ((uintptr_t)b.data_ptr() % 16) == 0, "16-byte aligned");
  c10::DeviceGuard dg(a.device());
  auto out = at::empty_like(a);
  dtg::mul_bf16(cbfp(a), cbfp(b), bfp(out), a.numel(), cur_stream());
  return out;
}

Tensor mask_additive(Tensor mask) {
  TORCH_CHECK(mask.is_cuda() && mask.is_contiguous(), "mask: contiguous GPU tensor");
  TORCH_CHECK(mask.scalar_type() == at::kLong || mask.scalar_type() == at::kFloat, "mask int64 or fp32");
  c10::DeviceGuard dg(mask.device());
  auto out = at::empty(mask.sizes(), mask.options().dtype(at::kFloat));
  dtg::mask_additive(mask.data_ptr(), mask.scalar_type() == at::kFloat, out.data_ptr<float>(), mask.numel(),
                     cur_stream());
  return out;
}

void register_transformer_ops(py::module_& m) {
  m.def("mul_bf16", &mul_bf16);
  m.def("mask_additive", &mask_additive);
  m.def("gemm_strided_batched", &gemm_strided_batched);
  m.def("ln_fwd", &ln_fwd, py::arg("h"), py::arg("res"), py::arg("gamma"), py::arg("beta"), py::arg("eps") = 1e-12,
        py::arg("p_in") = 0.0, py::arg("seed_in") = 0, py::arg("p_out") = 0.0, py::arg("seed_out") = 0,
        py::arg("save_s") = true);
  m.def("ln_bwd", &ln_bwd, py::arg("dy"), py::arg("s"), py::arg("gamma"), py::arg("mean"), py::arg("rstd"),
        py::arg("dgamma"), py::arg("dbeta"), py::arg("p_in") = 0.0, py::arg("seed_in") = 0, py::arg("p_out") = 0.0,
        py::arg("seed_out") = 0, py::arg("want_dh") = true, py::arg("dbias") = py::none());
  m.def("attn_softmax_fwd", &attn_softmax_fwd);
  m.def("attn_softmax_bwd", &attn_softmax_bwd);
  m.def("colsum", &colsum, py::arg("x"), py::arg("out"), py::arg("accumulate") = true, py::arg("sel") = py::none(),
        py::arg("nsel") = 1);
  m.def("emb_fwd", &emb_fwd);
  m.def("attn_fused_fwd", &attn_fused_fwd);
  m.def("attn_fused_bwd", &attn_fused_bwd, py::arg("qkv"), py::arg("out"), py::arg("dout"), py::arg("lse"),
        py::arg("mask"), py::arg("B"), py::arg("S"), py::arg("nh"), py::arg("p"), py::arg("seed"),
        py::arg("dbias") = py::none());
  m.def("attn_fused_supported", [](int64_t S, int64_t dh, bool bwd) { return dtg::attn_fused_supported(S, dh, bwd) != 0; });
  m.def("emb_word_bwd", &emb_word_bwd);
  m.def("gather_rows", &gather_rows);
  m.def("scatter_rows_add", &scatter_rows_add);
  m.def("nsp_loss_fwd", &nsp_loss_fwd);
  m.def("nsp_loss_bwd", &nsp_loss_bwd);
  m.def("row_sum", &row_sum);
  m.def("emb_word_bwd_owned", &emb_word_bwd_owned);
  m.def("zero_", &zero_);
  m.def("emb_pos_bwd", &emb_pos_bwd);
}
