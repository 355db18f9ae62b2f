// Host-side launch API of dtg's HIP kernels.  Raw pointers + hipStream_t only: the torch
// bindings (csrc/bindings/) validate tensors and pass the current stream, so every launch is
// stream-ordered and hipGraph-capturable (no allocation, no sync inside).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtg {
typedef unsigned short bf16_t;

// ---- optimizer applies over flat buffers (optim.hip) -------------------------------------------
// hyper: device float[2] = {lr, step}
void sgd_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, long long n, const float* hyper, float wd,
               float gscale, int zero_grad, hipStream_t st);
void momentum_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* mom, long long n,
                    const float* hyper, float mu, float wd, int nesterov, float gscale, int zero_grad,
                    hipStream_t st);
void adagrad_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* acc, long long n,
                   const float* hyper, float eps, float gscale, int zero_grad, hipStream_t st);
void adam_apply(float* w, bf16_t* mirror, void* grad, int grad_bf16, float* m, float* v, long long n,
                const float* hyper, float b1, float b2, float eps, float wd, float gscale, int zero_grad,
                hipStream_t st);
void axpby(float* acc, const void* g, int g_bf16, long long n, float alpha, float beta, hipStream_t st);
void f32_to_bf16(const float* x, bf16_t* y, long long n, hipStream_t st);
void hyper_tick(float* hyper, hipStream_t st);
// heads.hip: out = a * b (bf16); BERT additive key mask (1 - m) * -10000 from int64 / fp32 m
void mul_bf16(const bf16_t* a, const bf16_t* b, bf16_t* out, long long n, hipStream_t st);
void mask_additive(const void* mask, int is_f32, float* out, long long n, hipStream_t st);
// zero `bytes` bytes at p (16-B aligned for the vector part) with a dtg kernel
void fill_zero(void* p, long long bytes, hipStream_t st);

// ---- emulated blocking collective (comm_emu.hip; parallel/ddp.py DTG_COMM_EMULATE) ------------------
void comm_spin(double seconds, int wgs, int lds_bytes, hipStream_t st);
// round-5 form: mode bits 1 busy-poll, 2 HBM traffic through scratch (base: window offset, advanced by the returned
// count), 4 data (bucket *= factor after the wait)
long long comm_emu(double seconds, int wgs, int mode, void* scratch, long long scratch_bytes, long long base,
                   long long traffic_bytes, void* buf, long long n, int buf_bf16, float factor, hipStream_t st);
void launch_probe(int grid, int lds_bytes, hipStream_t st);
// HBM streaming probe (stream_probe.hip): kind 0 read, 1 write, 2 copy, 3 read2/write1 over n16 16-B vectors
void stream_probe(int kind, const void* a, const void* b, void* o, long long n16, unsigned* sink, int wgs, int unroll,
                  int nt, hipStream_t st);

// ---- BatchNorm statistics fused into a GEMM / implicit-GEMM epilogue (dtg/bn_epi.cuh) ----------
// mode 1 (forward): per output column c, sum and sum of squares of the stored (bf16) output.
// mode 2 (backward through BN -> ReLU): the epilogue turns the GEMM result g (= dL/da, a = relu(bn(x)))
//   into dp = g * [gamma*xhat + beta > 0] (stored instead of g) and accumulates sum(dp) and
//   sum(dp * xhat), xhat = (x - mean) * invstd, x = the BN input (same layout as the output).
// mode 3 (backward through BN -> +residual -> ReLU, computed by the NEXT layer's dgrad): like mode 2, but
//   the relu mask is (mask > 0) for a given tensor (the block output) and the epilogue may accumulate
//   (beta) into C first: dp = [mask > 0] * (alpha*acc + beta*C).
// Partials land in part[kBnStatSlots][2][N] (zero-initialised fp32, atomically accumulated; tile t
// adds into slot t % kBnStatSlots) and are reduced by the BN finalize kernel.
constexpr int kBnStatSlots = 32;
struct BnEpi {
  float* part = nullptr;
  int mode = 0;
  const bf16_t* x = nullptr;
  const float* mean = nullptr;
  const float* invstd = nullptr;
  const float* gamma = nullptr;
  const float* beta = nullptr;
  const bf16_t* mask = nullptr;      // mode 3: relu mask as the bf16 block output (> 0) ...
  const uint8_t* maskbits = nullptr; // ... or as packed bits [M][N/8] (bit k of byte n/8 = column n+k)
  // mode 3, optional: a second BN fed by the same gradient (the projection shortcut's): its input x2
  // and statistics; (sum dp, sum dp*xhat2) go to part2 (same layout as part)
  const bf16_t* x2 = nullptr;
  const float* mean2 = nullptr;
  const float* invstd2 = nullptr;
  float* part2 = nullptr;
  // mode 3/4, optional: the residual gradient (beta * C) exists only on the rows (n, h, w) with h and w
  // even -- what a stride-2 1x1 projection's dgrad writes; every other row reads as zero and is not
  // loaded, so the projection's dgrad need not zero-fill them.  Row -> (h, w) by multiply-shift division
  // (magic m, shift l of H*W and of W, host-computed: bn_sub2_rows).
  int old_sub2 = 0;
  uint32_t old_hw = 1, old_w = 1, hw_m = 0, hw_l = 0, w_m = 0, w_l = 0;
};

// host: fill the old_sub2 fields of a BnEpi for an H x W image
inline void bn_sub2_rows(BnEpi& bn, int H, int W) {
  auto magic = [](uint32_t d, uint32_t& m, uint32_t& l) {
    l = 0;
    while ((1u << l) < d) ++l;
    m = (uint32_t)((((uint64_t)1 << 32) * (((uint64_t)1 << l) - d)) / d + 1);
  };
  bn.old_sub2 = 1;
  bn.old_hw = (uint32_t)(H * W);
  bn.old_w = (uint32_t)W;
  magic(bn.old_hw, bn.hw_m, bn.hw_l);
  magic(bn.old_w, bn.w_m, bn.w_l);
}

// ---- batchnorm NHWC (batchnorm.hip) ----------------------------------------------------------
long long bn_workspace_floats(long long M, int C);
// finish a forward BN from fused-epilogue statistics: finalize (coef = ws[0:2C]) + apply
// bits (optional, [M][C/8]): packed (y > 0) of the output, the relu mask a later backward re-reads
void bn_fwd_from_part(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                      float* rmean, float* rvar, float* smean, float* sinv, const float* part, float* ws, long long M,
                      int C, float momentum, float eps, int relu, hipStream_t st, uint8_t* bits = nullptr);
// y = relu(bn(x) + bn2(r)) with both BNs' statistics from epilogue partials (ws: 4C floats)
void bn_fwd2_from_part(const bf16_t* x, const bf16_t* r, bf16_t* y, const float* part, const float* part2,
                       const float* gamma, const float* beta, float* rmean, float* rvar, float* smean, float* sinv,
                       const float* gamma2, const float* beta2, float* rmean2, float* rvar2, float* smean2,
                       float* sinv2, float* ws, long long M, int C, float momentum, float eps, hipStream_t st,
                       uint8_t* bits = nullptr);
// two BNs fed by the same (relu-masked) gradient dp -- BN3 and the projection BN of a ResNet block:
// dx = a*dp + bx*x + c0 and dx2 = a2*dp + bx2*x2 + c02 in one pass over dp (ws: 6C floats)
void bn_bwd2_from_part(const bf16_t* dp, const bf16_t* x, const bf16_t* x2, const float* part, const float* part2,
                       const float* gamma, const float* smean, const float* sinv, const float* gamma2,
                       const float* smean2, const float* sinv2, bf16_t* dx, bf16_t* dx2, float* dgamma, float* dbeta,
                       float* dgamma2, float* dbeta2, float* ws, long long M, int C, int accum, hipStream_t st);
// finish a backward BN from mode-2 partials: dx = a*dp + bx*x + c0 (ws: 3C floats), dres = dp if given
void bn_bwd_coef_from_part(const float* part, const float* gamma, const float* smean, const float* sinv, float* coef,
                           float* dgamma, float* dbeta, long long M, int C, int accum, hipStream_t st);
void bn_dx_from_coef(const bf16_t* dp, const bf16_t* x, const float* coef, bf16_t* dx, bf16_t* dres, long long M, int C,
                     hipStream_t st);
// bn_dx_wgrad.hip: the dx pass (from bn_bwd_coef_from_part coefficients, optionally the projection shortcut's dx2
// from the same dp) fused with the weight gradient dW += dx^T act of the conv that produced x (C x CI = 256 x 64 or
// 512 x 128)
bool bn_dx_wgrad_ok(long long M, int C, int CI);
int bn_dx_wgrad_slabs(int C, int CI, int w2 = 0);
void bn_dx_wgrad(const bf16_t* dp, const bf16_t* x, const float* coef, const bf16_t* x2, const float* coef2,
                 bf16_t* dx, bf16_t* dx2, const bf16_t* act, long long ldact, void* wgrad, int wgrad_bf16,
                 float* slabs, long long M, int C, int CI, hipStream_t st, const bf16_t* act2 = nullptr,
                 long long ldact2 = 0, void* wgrad2 = nullptr, float* slabs2 = nullptr);
void bn_bwd_from_part(const bf16_t* dp, const bf16_t* x, const float* gamma, const float* smean, const float* sinv,
                      const float* part, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* ws, long long M,
                      int C, int accum, hipStream_t st);
void bn_fwd_train(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                  float* rmean, float* rvar, float* smean, float* sinv, float* ws, long long M, int C,
                  float momentum, float eps, int relu, hipStream_t st);
void bn_fwd_infer(const bf16_t* x, const bf16_t* res, bf16_t* y, const float* gamma, const float* beta,
                  const float* rmean, const float* rvar, float* ws, long long M, int C, float eps, int relu,
                  hipStream_t st);
void bn_bwd(const bf16_t* dy, const bf16_t* y, const bf16_t* x, const float* gamma, const float* smean,
            const float* sinv, bf16_t* dx, bf16_t* dres, float* dgamma, float* dbeta, float* ws, long long M, int C,
            int relu, int accum, hipStream_t st);

// ---- softmax cross-entropy (softmax_xent.hip) ------------------------------------------------
void softmax_xent(const void* x, int x_bf16, const long long* label, long long B, int V, float scale, float* loss,
                  void* dx, float* lse, hipStream_t st);
// dx = (softmax(x) - onehot(label)) * scale * (*g) from the forward's lse; g: device scalar (may be null = 1)
void softmax_xent_bwd(const void* x, int x_bf16, const long long* label, const float* lse, long long B, int V,
                      float scale, const float* g, void* dx, hipStream_t st);

// ---- GEMM (gemm.hip) -------------------------------------------------------------------------
// Two-level batch (e.g. [batch, heads] of attention): problem z = zb * nh + zh uses
// A + zb*sa_b + zh*sa_h etc. (element strides).  count = 1 for a plain GEMM.
struct GemmBatch {
  int count = 1, nh = 1;
  long long sa_b = 0, sa_h = 0, sb_b = 0, sb_h = 0, sc_b = 0, sc_h = 0;
};
// force the BN-epilogue GEMM tile (tools/bn_gemm_ab.py; 0 = heuristic).  (Forced tiles of the plain GEMM and the
// 256x256 8-phase kernels live in the lab extension, csrc/lab.)
void gemm_bn_force_cfg(int cfg);
void conv_force_tile(int which, int code);  // conv.hip: 0 fwd, 1 stride-1 dgrad
long long gemm_workspace_floats(int M, int N, int K, int split_k);
int gemm_pick_split(int M, int N, int K, int a_kc = 0, int target_wgs = 0);  // target 0: default (512)
void gemm_bf16(const bf16_t* A, long long lda, int a_kc, const bf16_t* B, long long ldb, int b_kc, void* C,
               long long ldc, int c_bf16, int M, int N, int K, float alpha, float beta, const float* bias, int act,
               int split_k, float* ws, hipStream_t st, const GemmBatch& batch = GemmBatch(), void* aux = nullptr,
               int aux_mode = 0);
// C[M,N] (bf16, row stride ldc) = A * op(B) (+ beta*C in mode 3) with BN statistics in the epilogue
// (bn.mode 1: B is [N,K] (forward); bn.mode 2/3: B is [K,N] (dgrad)).  A is [M,K] K-contiguous.
void gemm_bf16_bn(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, bf16_t* C, long long ldc, int M,
                  int N, int K, float beta, const BnEpi& bn, hipStream_t st);
// C = act(A * B + bias) (B [K,N], the dgrad layout; aux as in gemm_bf16) and colsum[n] += sum_m C[m, n]
// in the same epilogue (fp32 atomics; the bias gradient of the layer C is the output gradient of)
void gemm_bf16_colsum(const bf16_t* A, long long lda, const bf16_t* B, long long ldb, bf16_t* C, long long ldc, int M,
                      int N, int K, const float* bias, int act, void* aux, int aux_mode, float* colsum, hipStream_t st);

// ---- transformer blocks (transformer.hip) ------------------------------------------------------
int ln_max_hidden();
void ln_fwd(const bf16_t* h, const bf16_t* res, const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out,
            float* mean, float* rstd, int T, int H, float eps, float p_in, uint32_t seed_in, float p_out,
            uint32_t seed_out, hipStream_t st);
int ln_bwd_blocks(int T);  // ln_bwd workspace = ln_bwd_blocks(T) * 3H floats
void ln_bwd(const bf16_t* dy, const bf16_t* s, const float* gamma, const float* mean, const float* rstd,
            bf16_t* ds_out, bf16_t* dh_out, float* dgamma, float* dbeta, float* dbias, float* ws, int T, int H,
            float p_in, uint32_t seed_in, float p_out, uint32_t seed_out, hipStream_t st);
int attn_max_keys();
void attn_softmax_fwd(const float* sc, const float* mask, bf16_t* P, bf16_t* Pd, int rows, int rows_per_b, int Sk,
                      float p, uint32_t seed, hipStream_t st);
void attn_softmax_bwd(const bf16_t* P, const bf16_t* Pd, const float* dPd, bf16_t* dS, int rows, int Sk, float scale,
                      hipStream_t st);
int colsum_splits(int T, int N);  // workspace = splits * nsel * N floats
void colsum(const bf16_t* x, long long ld, int T, int N, const long long* sel, int nsel, void* out, int out_bf16,
            int accumulate, float* ws, int splits, hipStream_t st);
void emb_fwd(const long long* ids, const long long* tt, const bf16_t* word, const bf16_t* pos, const bf16_t* type,
             bf16_t* s, int T, int S, int H, hipStream_t st);
void emb_word_bwd(const bf16_t* ds, const long long* sorted, const long long* perm, bf16_t* gW, int T, int H,
                  hipStream_t st);
void emb_pos_bwd(const bf16_t* ds, bf16_t* gP, int T, int S, int H, hipStream_t st);

// ---- BERT pre-training heads and row plumbing (heads.hip) -----------------------------------------
void gather_rows(const bf16_t* src, const long long* pos, bf16_t* out, int R, int P, int S, int H, hipStream_t st);
void scatter_rows_add(bf16_t* dst, const long long* pos, const bf16_t* src, int R, int P, int S, int H,
                      hipStream_t st);
void nsp_loss_fwd(const bf16_t* pooled, const bf16_t* wn, const float* bn, const long long* labels, const float* extra,
                  float* probs, float* out, int B, int H, hipStream_t st);
void nsp_loss_bwd(const bf16_t* pooled, const bf16_t* wn, const float* probs, const long long* labels, const float* gout,
                  bf16_t* dpre, bf16_t* gwn, float* gbn, int B, int H, hipStream_t st);
void row_sum(const float* x, float* out, long long n, float scale, hipStream_t st);
void emb_word_bwd_owned(const bf16_t* ds, const long long* ids, bf16_t* gW, int T, int H, int V, hipStream_t st);

// ---- fused attention, head dim 64 (attention.hip) ---------------------------------------------
int attn_fused_supported(int S, int dh, int backward);
void attn_fwd(const bf16_t* qkv, const float* mask, bf16_t* out, float* lse, int B, int S, int nh, float p,
              uint32_t seed, hipStream_t st);
void attn_bwd(const bf16_t* qkv, const bf16_t* o, const bf16_t* dout, const float* lse, const float* mask,
              bf16_t* dqkv, int B, int S, int nh, float p, uint32_t seed, float* dbias, hipStream_t st);

// ---- pooling, NHWC (pool.hip) -----------------------------------------------------------------
void maxpool_fwd(const bf16_t* x, bf16_t* y, uint8_t* idx, int N, int H, int W, int C, int k, int s, int pad, int P,
                 int Q, hipStream_t st);
void maxpool_bwd(const bf16_t* dy, const uint8_t* idx, bf16_t* dx, int N, int H, int W, int C, int k, int s, int pad,
                 int P, int Q, hipStream_t st);
void avgpool_fwd(const bf16_t* x, bf16_t* y, int N, int HW, int C, hipStream_t st);
void avgpool_bwd(const bf16_t* dy, bf16_t* dx, int N, int HW, int C, hipStream_t st);

// ---- fused ResNet stem tail: BN (conv-epilogue statistics) + ReLU + max-pool (stem.hip) ----------
// fwd: finalize the BN statistics (coef = 2C floats: scale, shift; running stats updated) and write the
//      pooled output + window argmax in one pass over y [N,H,W,C].
// bwd: dy = BN-backward(relu-mask * maxpool-backward(dout)) without materialising either intermediate;
//      ws = stem_bwd_workspace_floats(N*H*W, C); dgamma/dbeta overwritten (accum = 0) or accumulated.
void stem_bn_pool_fwd(const bf16_t* y, const float* part, const float* gamma, const float* beta, float* rmean,
                      float* rvar, float* smean, float* sinv, float* coef, bf16_t* out, uint8_t* idx, int N, int H,
                      int W, int C, int k, int s, int pad, int P, int Q, float momentum, float eps, hipStream_t st,
                      bf16_t* yam = nullptr);
long long stem_bwd_workspace_floats(long long M, int C);
// the backward's statistics pass can run at pooled resolution (yam: y at each window's argmax, [N,P,Q,C],
// written by stem_bn_pool_fwd when given) for these channel counts
bool stem_pooled_stats_ok(int C);
// channels_last [K, C, R, S] stem weights -> pixel-pair form [K][KP] (KP >= R * S2 * 8, zero padded)
void stem_pack_weights(const bf16_t* w, bf16_t* wp, int K, int C, int R, int S, int S2, int KP, hipStream_t st);
// grad[K,R,S,C] (+)= the stem conv's padded-channel weight gradient (pair form: [K,R,S2,8], else [K,R,S,8])
void stem_dw_add(const float* src, void* grad, int grad_bf16, int K, int R, int S, int C, int S2, int pair,
                 hipStream_t st);
// x [N,H,W,C<=4] -> xp [N, H+2*pad, Wp, 4], zero padded (the pixel-pair stem conv's input)
void stem_pack_pairs(const bf16_t* x, bf16_t* xp, int N, int H, int W, int C, int pad, int Hp, int Wp,
                     hipStream_t st);
void stem_bn_pool_bwd(const bf16_t* dout, const uint8_t* idx, const bf16_t* y, const float* gamma, const float* beta,
                      const float* smean, const float* sinv, bf16_t* dy, float* dgamma, float* dbeta, int accum,
                      float* ws, int N, int H, int W, int C, int k, int s, int pad, int P, int Q, hipStream_t st,
                      const bf16_t* yam = nullptr);

// ---- im2col / col2im, NHWC (im2col.hip) --------------------------------------------------------
void im2col(const bf16_t* x, bf16_t* cols, int N, int H, int W, int C, int R, int S, int stride, int pad, int Kp,
            hipStream_t st);
void col2im(const bf16_t* dcols, bf16_t* dx, int N, int H, int W, int C, int R, int S, int stride, int pad, int Kp,
            hipStream_t st);

// ---- implicit-GEMM convolution, NHWC (conv.hip) ------------------------------------------------
// which: 0 fwd, 1 dgrad, 2 wgrad.  Strided dgrad runs one dense launch per residue class of dx.
int conv_supported(int C, int K, int R, int S, int stride, int pad, int which);
// direct 3x3 / s1 / p1 conv, 64 -> 64 channels, with the BN forward statistics into part (conv_halo.hip; conv_fwd
// takes it for BnEpi mode 1 when conv3x3_halo_bn_ok)
int conv3x3_halo_bn_ok(int C, int K, int H, int W);
bool conv3x3_halo_bn_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, float* part, hipStream_t st);
void conv3x3_halo_fwd_set(int on);  // (A/B tools, tests) the halo forward on / off
// its data gradient with the BN-backward mode-3 epilogue (packed mask bits, beta 0); false if bn is not that form
bool conv3x3_halo_bn_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dp, int N, int H, int W, const BnEpi& bn,
                           hipStream_t st);
void conv3x3_halo_dgrad_set(int on);  // (A/B tools) the halo data gradient on / off
// its weight gradient (W = 56): the split (= workgroups, one fp32 slab each) conv_wgrad uses, 0 if not this shape
int conv3x3_halo_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w);
void conv3x3_halo_wgrad(const bf16_t* dy, const bf16_t* x, float* ws, int grid, int N, int H, hipStream_t st);
void conv3x3_halo_wgrad_set(int on);
// linear-halo 3x3 weight gradient (conv_halo.hip) for 7x7 / 14x14 / 28x28 layers with C, K multiples of 64: split =
// band ranges (split-K slabs), 0 when the shape is not covered
int conv3x3_lin_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w);
void conv3x3_lin_wgrad(const bf16_t* dy, const bf16_t* x, float* ws, int split, int N, int H, int W, int C, int K,
                       hipStream_t st);
void conv3x3_lin_wgrad_set(int on);  // (A/B tools) on / off  // (A/B tools) the halo weight gradient on / off
void conv_fwd(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, int C, int K, int R, int S,
              int stride, int pad, hipStream_t st, const BnEpi& bn = BnEpi());
// returns 0 if bn.mode != 0 was asked for a geometry the fused statistics cannot cover (strided dgrad
// with residue classes no tap reaches)
// wT (optional): the weight transposed to [C][(r,s,k)] (K-contiguous), used by the stride-1 kernels
int conv_dgrad(const bf16_t* dy, const bf16_t* w, bf16_t* dx, int N, int H, int W, int C, int K, int R, int S,
               int stride, int pad, float beta, hipStream_t st, const BnEpi& bn = BnEpi(),
               const bf16_t* wT = nullptr, int zero_rest = 1);
void stem_stream_set(int on);  // the streaming stem conv (gemm_expand.hip) on / off (A/B tools)
void stem_pool_rows_set(int on);  // stem max-pool forward: the row-walking kernel (1, default) or row-parallel (0)
void gemm_expand_k256_set(int on);  // the streaming expand GEMM for K = 256 (gemm_expand.hip) on / off (A/B tools)
void gemm_expand_s2_set(int on);    // the stride-2 1x1 projection on the expand kernel (gemm_expand.hip) on / off
bool conv1x1_s2_expand_bn(const bf16_t* x, int Nb, int H, int W, int Cin, const bf16_t* w, bf16_t* y, int Kout,
                          float* part, hipStream_t st);
void conv_fwd_c8(const bf16_t* x, const bf16_t* w, bf16_t* y, int N, int H, int W, int K, int R, int S, int stride,
                 int pad, hipStream_t st, const BnEpi& bn = BnEpi(), int stride_w = 0);
void conv_set_stages(int which, int stages);  // which: 0 fwd, 1 dgrad, 2 wgrad
// stride_w (0 = stride): the W stride where it differs from the H stride (C8 forward and wgrad only)
int conv_wgrad_split(int N, int H, int W, int C, int K, int R, int S, int stride, int pad, int stride_w = 0,
                     int target_wgs = 0);  // target 0: 1024 workgroups
void conv_wgrad(const bf16_t* dy, const bf16_t* x, void* dw, int dw_bf16, float beta, float* ws, int split, int N,
                int H, int W, int C, int K, int R, int S, int stride, int pad, hipStream_t st, int stride_w = 0,
                int sched = 0);  // sched: LDS schedule code of this call (conv_set_stages codes), 0 = default

}  // namespace dtg
