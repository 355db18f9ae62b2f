// Transformer (BERT) building blocks on gfx950, bf16 activations, fp32 statistics:
//   * LayerNorm fwd with fused residual add + dropout of the branch input (and optional dropout
//     of the output, BERT's embedding LayerNorm), bwd with the dropout masks regenerated from a
//     counter hash (no mask tensors) and gamma/beta grads accumulated with per-block fp32 atomics;
//   * attention softmax fwd (additive key mask, attention-probability dropout) and bwd;
//   * column sums (bias gradients: per-block atomics into the fp32 grad; token-type embedding
//     gradient with a row selector: two-pass into bf16);
//   * embedding gather-sum fwd and the deterministic embedding bwd (sorted token segments: one
//     writer per vocabulary row, no atomics).
// One wave64 per row everywhere: a lane owns 8-element (16-byte) chunks lane, lane+64, ... so a
// row of H = 768 is 96 chunks -> every load is a dwordx4 and reductions are wave shuffles.
#include "dtg/common.h"
#include "dtg/kernels.h"
#include <stdlib.h>

namespace dtg {

// ---- counter-based dropout mask ----------------------------------------------------------------
// keep(seed, i) = fmix32(i * golden + seed) >= p * 2^32 (murmur3 finalizer).  Python mirror:
// dtg/ops/transformer.py::dropout_keep (used by the CPU reference and the tests).
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ bool keep_elem(uint32_t seed, uint32_t idx, uint32_t thresh) {
  return fmix32(idx * 0x9E3779B1u + seed) >= thresh;
}
// attention-probability dropout (the fused kernels' pair hash, attention.hip keep_attn): element idx is kept iff the
// low (even idx) / high (odd idx) 16 bits of fmix32((idx >> 1) * golden + seed) are >= floor(p * 2^16).  Python
// mirror: dtg/ops/transformer.py::attn_dropout_keep.
__device__ __forceinline__ bool keep_attn(uint32_t seed, uint32_t idx, uint32_t th16) {
  const uint32_t h = fmix32((idx >> 1) * 0x9E3779B1u + seed);
  return ((idx & 1u) ? (h >> 16) : (h & 0xffffu)) >= th16;
}
static inline uint32_t drop_thresh16(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 65536.0;
  return t >= 65535.0 ? 0xffffu : (t < 1.0 ? 1u : (uint32_t)t);
}
static inline uint32_t drop_thresh(float p) {
  if (p <= 0.f) return 0u;
  const double t = (double)p * 4294967296.0;
  return t >= 4294967295.0 ? 0xffffffffu : (uint32_t)t;
}

constexpr int kRowsPerBlock = 4;  // 4 waves, one row each

// ---- LayerNorm forward ---------------------------------------------------------------------------
// s = res + dropout_in(h)   (res may be null; s is rounded to bf16 and, if s_out, saved)
// y = dropout_out(gamma * (s - mean) * rstd + beta)
template <int NCH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16_t* __restrict__ h, const bf16_t* __restrict__ res,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     bf16_t* __restrict__ y, bf16_t* __restrict__ s_out,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int T, int H, float eps, uint32_t th_in, float sc_in,
                                                     uint32_t seed_in, uint32_t th_out, float sc_out,
                                                     uint32_t seed_out) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= T) return;
  const int nc = H >> 3;
  const long long base = (long long)row * H;
  float v[NCH][8];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = lane + 64 * j;
    if (c < nc) {
      load8_bf16(h + base + c * 8, v[j]);
      if (th_in) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
          v[j][k] = keep_elem(seed_in, (uint32_t)(base + c * 8 + k), th_in) ? v[j][k] * sc_in : 0.f;
      }
      if (res) {
        float r[8];
        load8_bf16(res + base + c * 8, r);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[j][k] += r[k];
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        v[j][k] = bf2f(f2bf(v[j][k]));  // statistics of the stored (bf16) sum
        sum += v[j][k];
      }
      // read again only in backward: non-temporal, so it does not evict what the next GEMM reads
      if (s_out) store8_bf16_nt(s_out + base + c * 8, v[j]);
    }
  }
  const float mean = wave_sum(sum) / H;
  float sq = 0.f;
#pragma unroll
  for (int j = 0; j < NCH; ++j)
    if (lane + 64 * j < nc)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = v[j][k] - mean;
        sq += d * d;
      }
  const float rstd = rsqrtf(wave_sum(sq) / H + eps);
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
#pragma unroll
  for (int j = 0; j < NCH; ++j) {
    const int c = lane + 64 * j;
    if (c < nc) {
      float g[8], b[8], o[8];
      load8_f32(gamma + c * 8, g);
      load8_f32(beta + c * 8, b);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        o[k] = (v[j][k] - mean) * rstd * g[k] + b[k];
        if (th_out) o[k] = keep_elem(seed_out, (uint32_t)(base + c * 8 + k), th_out) ? o[k] * sc_out : 0.f;
      }
      store8_bf16(y + base + c * 8, o);
    }
  }
}

// ---- LayerNorm backward ----------------------------------------------------------------------------
// g = dropout_out'(dy); ds = rstd * (g*gamma - mean(g*gamma) - xhat * mean(g*gamma*xhat))
// ds_out = ds (the residual-branch gradient); dh_out = dropout_in'(ds) (the branch gradient);
// per-block sums of g*xhat, g (and the branch gradient, for the fused bias grad) are written as
// partial rows and folded by ln_param_reduce_kernel.
//
// Lane layout: 4-element (8-byte) chunks lane, lane + 64, ... of the H/4 chunks of a row, so H = 768 is
// exactly 3 chunks per lane (16-byte chunks left half the lanes idle in the second pass).  The running
// dgamma / dbeta / dbias partials live in the wave's own LDS row [3][H] (each lane only ever touches its
// own columns, so no barrier inside the row loop), not in 36-48 accumulator registers: the kernel then
// fits 4 waves per SIMD (it needed 158 VGPRs = 3 per SIMD, and 1024 blocks of 4 waves ran as 1.33
// rounds of blocks).
__device__ __forceinline__ void unpack4_bf16(const uint2 v, float (&o)[4]) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
}
__device__ __forceinline__ void store4_bf16(bf16_t* p, const float (&o)[4]) {
  uint2 v;
  v.x = pack_bf2(o[0], o[1]);
  v.y = pack_bf2(o[2], o[3]);
  *reinterpret_cast<uint2*>(p) = v;
}

template <int NC4>
__global__ void __launch_bounds__(256) ln_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ s,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, bf16_t* __restrict__ ds_out,
                                                     bf16_t* __restrict__ dh_out, float* __restrict__ ws,
                                                     float* __restrict__ dbias, int T, int H,
                                                     uint32_t th_in, float sc_in, uint32_t seed_in, uint32_t th_out,
                                                     float sc_out, uint32_t seed_out) {
  extern __shared__ float red[];  // [4][3H]: per-wave running gamma, beta, branch-bias partials
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int nc = H >> 2;
  float4* accg = reinterpret_cast<float4*>(red + wv * 3 * H);  // chunk c of dgamma / dbeta / dbias at
  float4* accb = accg + nc;                                    // accg[c], accb[c], accz[c]
  float4* accz = accb + nc;
  const bool want_z = dh_out != nullptr || dbias != nullptr;
#pragma unroll
  for (int j = 0; j < NC4; ++j) {
    const int c = lane + 64 * j;
    if (c < nc) accg[c] = accb[c] = accz[c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // One row ahead in registers: the next row's dy / s (and its statistics) are loaded before this row's
  // reductions and stores, so each wave keeps two rows of HBM reads in flight.  (Two rows ahead took 150
  // VGPRs, 3 waves per SIMD; capped at 128 it spilled.)
  const int rstep = gridDim.x * kRowsPerBlock;
  int row = blockIdx.x * kRowsPerBlock + wv;
  uint2 pdy[NC4], ps[NC4];
  float pm = 0.f, pr = 0.f;
  auto prefetch = [&](int r) {
    if (r >= T) return;
    const long long b = (long long)r * H;
#pragma unroll
    for (int j = 0; j < NC4; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        pdy[j] = *reinterpret_cast<const uint2*>(dy + b + c * 4);
        ps[j] = *reinterpret_cast<const uint2*>(s + b + c * 4);
      }
    }
    pm = mean_in[r];
    pr = rstd_in[r];
  };
  prefetch(row);
  for (; row < T; row += rstep) {
    const long long base = (long long)row * H;
    const float mean = pm, rstd = pr;
    float g[NC4][4], xh[NC4][4];
#pragma unroll
    for (int j = 0; j < NC4; ++j) {
      unpack4_bf16(pdy[j], g[j]);
      unpack4_bf16(ps[j], xh[j]);
    }
    prefetch(row + rstep);
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int j = 0; j < NC4; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        const float4 gm = *reinterpret_cast<const float4*>(gamma + c * 4);
        const float gmv[4] = {gm.x, gm.y, gm.z, gm.w};
        const float4 tg = accg[c], tb = accb[c];
        float pg[4] = {tg.x, tg.y, tg.z, tg.w}, pb[4] = {tb.x, tb.y, tb.z, tb.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (th_out && !keep_elem(seed_out, (uint32_t)(base + c * 4 + k), th_out)) g[j][k] = 0.f;
          else if (th_out) g[j][k] *= sc_out;
          xh[j][k] = (xh[j][k] - mean) * rstd;
          pg[k] += g[j][k] * xh[j][k];
          pb[k] += g[j][k];
          g[j][k] *= gmv[k];
          a += g[j][k];
          b += g[j][k] * xh[j][k];
        }
        accg[c] = make_float4(pg[0], pg[1], pg[2], pg[3]);
        accb[c] = make_float4(pb[0], pb[1], pb[2], pb[3]);
      }
    }
    a = wave_sum(a) / H;
    b = wave_sum(b) / H;
#pragma unroll
    for (int j = 0; j < NC4; ++j) {
      const int c = lane + 64 * j;
      if (c < nc) {
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = rstd * (g[j][k] - a - xh[j][k] * b);
        store4_bf16(ds_out + base + c * 4, o);
        if (want_z) {
          const float4 tz = accz[c];
          float pz[4] = {tz.x, tz.y, tz.z, tz.w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            o[k] = (!th_in || keep_elem(seed_in, (uint32_t)(base + c * 4 + k), th_in)) ? o[k] * sc_in : 0.f;
            pz[k] += bf2f(f2bf(o[k]));  // the bias grad of the branch = column sum of the stored dh
          }
          accz[c] = make_float4(pz[0], pz[1], pz[2], pz[3]);
          if (dh_out) store4_bf16(dh_out + base + c * 4, o);
        }
      }
    }
  }
  __syncthreads();
  // per-block partials of [dgamma | dbeta | dbias] -> ws[block][3H]; ln_param_reduce_kernel sums them
  const int nred = dbias ? 3 * H : 2 * H;
  for (int i = threadIdx.x; i < nred; i += blockDim.x) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kRowsPerBlock; ++w) t += red[w * 3 * H + i];
    ws[(long long)blockIdx.x * 3 * H + i] = t;
  }
}

// out[i] += sum over the nb partial rows of ws[:, i]  (i < ncols; out = [dgamma | dbeta | dbias]).
// Grid (ncols/64, 8 row groups); block = 64 columns x 4 row lanes; a row group folds its rows with
// 8 loads in flight per thread, then one atomic per column per group (8-way, not nb-way).
__global__ void __launch_bounds__(256) ln_param_reduce_kernel(const float* __restrict__ ws, int nb, int H,
                                                              int ncols, float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta, float* __restrict__ dbias) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lr = threadIdx.x >> 6;
  const int per = (nb + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * per, r1 = min(nb, r0 + per);
  float t = 0.f;
  if (col < ncols) {
    int r = r0 + lr;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = ws[(long long)(r + 4 * k) * 3 * H + col];
#pragma unroll
      for (int k = 0; k < 8; ++k) t += v[k];
    }
    for (; r < r1; r += 4) t += ws[(long long)r * 3 * H + col];
  }
  red[lr][threadIdx.x & 63] = t;
  __syncthreads();
  if (lr == 0 && col < ncols) {
    t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(col < H ? dgamma + col : (col < 2 * H ? dbeta + (col - H) : dbias + (col - 2 * H)), t);
  }
}

// ---- attention softmax -------------------------------------------------------------------------------
// Row r of the [B*nh*Sq, Sk] fp32 score matrix (already scaled): P = softmax(s + mask[b]),
// Pd = dropout(P).  Lane owns columns lane + 64*j.
template <int NJ>
__global__ void __launch_bounds__(256) attn_softmax_fwd_kernel(const float* __restrict__ sc,
                                                               const float* __restrict__ mask, bf16_t* __restrict__ P,
                                                               bf16_t* __restrict__ Pd, int rows, int rows_per_b,
                                                               int Sk, uint32_t th, float scl, uint32_t seed) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long base = (long long)row * Sk;
  const float* mk = mask ? mask + (long long)(row / rows_per_b) * Sk : nullptr;
  float v[NJ];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    v[j] = -INFINITY;
    if (c < Sk) {
      v[j] = sc[base + c] + (mk ? mk[c] : 0.f);
      mx = fmaxf(mx, v[j]);
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    v[j] = (lane + 64 * j < Sk) ? __expf(v[j] - mx) : 0.f;
    sum += v[j];
  }
  const float inv = 1.f / wave_sum(sum);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < Sk) {
      const float p = v[j] * inv;
      P[base + c] = f2bf(p);
      if (Pd != P) Pd[base + c] = keep_attn(seed, (uint32_t)(base + c), th) ? f2bf(p * scl) : (bf16_t)0;
    }
  }
}

// dS = scale * (Pd*dPd - P * sum(Pd*dPd))  (P: softmax output, Pd: its dropout, dPd: grad wrt Pd)
template <int NJ>
__global__ void __launch_bounds__(256) attn_softmax_bwd_kernel(const bf16_t* __restrict__ P,
                                                               const bf16_t* __restrict__ Pd,
                                                               const float* __restrict__ dPd, bf16_t* __restrict__ dS,
                                                               int rows, int Sk, float scale) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const long long base = (long long)row * Sk;
  float pg[NJ], p[NJ];
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    pg[j] = p[j] = 0.f;
    if (c < Sk) {
      pg[j] = bf2f(Pd[base + c]) * dPd[base + c];
      p[j] = bf2f(P[base + c]);
      sum += pg[j];
    }
  }
  sum = wave_sum(sum);
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = lane + 64 * j;
    if (c < Sk) dS[base + c] = f2bf(scale * (pg[j] - p[j] * sum));
  }
}

// ---- column sums (bias grads; token-type grads with a row selector) ------------------------------------
// Block: 32 column chunks (8 columns each) x 8 row lanes; grid (ceil(N/256), splits).
// ws[split][v][N] = sum over the split's rows t with sel[t] == v (sel null: v = 0 for all rows).
// atomic_out: add straight into the fp32 output (accumulate) instead of writing ws partials.
template <int NS>
__global__ void __launch_bounds__(256) colsum_partial_kernel(const bf16_t* __restrict__ x, long long ld, int T,
                                                             int N, const long long* __restrict__ sel,
                                                             float* __restrict__ ws, float* __restrict__ atomic_out) {
  __shared__ float red[8][NS][256 + 4];
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int c = blockIdx.x * 32 + cl;
  const bool ok = c * 8 < N;
  float acc[NS][8];
#pragma unroll
  for (int v = 0; v < NS; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[v][k] = 0.f;
  if (ok) {
    const int step = gridDim.y * 8;
    int r = blockIdx.y * 8 + rl;
    if (!sel) {  // bias grads: 4 rows per iteration, four 16-B loads in flight
      for (; r + 3 * step < T; r += 4 * step) {
        float t0[8], t1[8], t2[8], t3[8];
        load8_bf16(x + (long long)r * ld + c * 8, t0);
        load8_bf16(x + (long long)(r + step) * ld + c * 8, t1);
        load8_bf16(x + (long long)(r + 2 * step) * ld + c * 8, t2);
        load8_bf16(x + (long long)(r + 3 * step) * ld + c * 8, t3);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[0][k] += (t0[k] + t1[k]) + (t2[k] + t3[k]);
      }
    }
    for (; r < T; r += step) {
      float t[8];
      load8_bf16(x + (long long)r * ld + c * 8, t);
      const int v = sel ? (int)sel[r] : 0;
#pragma unroll
      for (int u = 0; u < NS; ++u)
        if (u == v)
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[u][k] += t[k];
    }
  }
#pragma unroll
  for (int v = 0; v < NS; ++v)
#pragma unroll
    for (int k = 0; k < 8; ++k) red[rl][v][cl * 8 + k] = acc[v][k];
  __syncthreads();
  for (int i = threadIdx.x; i < NS * 256; i += 256) {
    const int v = i / 256, col = i % 256;
    const int n = blockIdx.x * 256 + col;
    if (n < N) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < 8; ++r) t += red[r][v][col];
      if (atomic_out) atomicAdd(atomic_out + (long long)v * N + n, t);
      else ws[((long long)blockIdx.y * NS + v) * N + n] = t;
    }
  }
}

// out[v][n] (+)= sum_split ws[split][v][n]; out fp32 or bf16
__global__ void __launch_bounds__(256) colsum_reduce_kernel(const float* __restrict__ ws, int splits, int NSN,
                                                            void* __restrict__ out, int out_bf16, int accumulate) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= NSN) return;
  float t = 0.f;
  for (int s = 0; s < splits; ++s) t += ws[(long long)s * NSN + i];
  if (out_bf16) {
    bf16_t* o = (bf16_t*)out;
    o[i] = f2bf(accumulate ? bf2f(o[i]) + t : t);
  } else {
    float* o = (float*)out;
    o[i] = accumulate ? o[i] + t : t;
  }
}

// ---- embeddings -------------------------------------------------------------------------------------
// s[t] = word[ids[t]] + pos[t % S] + type[tt[t]]   (position ids = arange(S) per sequence)
__global__ void __launch_bounds__(256) emb_fwd_kernel(const long long* __restrict__ ids,
                                                      const long long* __restrict__ tt, const bf16_t* __restrict__ word,
                                                      const bf16_t* __restrict__ pos, const bf16_t* __restrict__ type,
                                                      bf16_t* __restrict__ s, int T, int S, int H) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= T) return;
  const bf16_t* w = word + ids[row] * (long long)H;
  const bf16_t* p = pos + (long long)(row % S) * H;
  const bf16_t* ty = tt ? type + tt[row] * (long long)H : nullptr;
  for (int c = lane; c < (H >> 3); c += 64) {
    float a[8], b[8], d[8];
    load8_bf16(w + c * 8, a);
    load8_bf16(p + c * 8, b);
    if (ty) load8_bf16(ty + c * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += b[k] + (ty ? d[k] : 0.f);
    store8_bf16(s + (long long)row * H + c * 8, a);
  }
}

// Word-embedding grad: sorted ids; the wave at the start of each run of equal ids sums the run's
// rows (fp32) and adds once into gW[id] -> one writer per vocabulary row, deterministic.
__global__ void __launch_bounds__(256) emb_word_bwd_kernel(const bf16_t* __restrict__ ds,
                                                           const long long* __restrict__ sorted,
                                                           const long long* __restrict__ perm,
                                                           bf16_t* __restrict__ gW, int T, int H) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (i >= T) return;
  const long long id = sorted[i];
  if (i > 0 && sorted[i - 1] == id) return;
  int end = i + 1;
  while (end < T && sorted[end] == id) ++end;
  for (int c = lane; c < (H >> 3); c += 64) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = i; j < end; ++j) {
      float t[8];
      load8_bf16(ds + perm[j] * (long long)H + c * 8, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += t[k];
    }
    float o[8];
    bf16_t* g = gW + id * (long long)H + c * 8;
    load8_bf16(g, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] += acc[k];
    store8_bf16(g, o);
  }
}

// Position-embedding grad: gP[p] += sum_b ds[b*S + p]; one wave per position
__global__ void __launch_bounds__(256) emb_pos_bwd_kernel(const bf16_t* __restrict__ ds, bf16_t* __restrict__ gP,
                                                          int T, int S, int H) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (p >= S) return;
  for (int c = lane; c < (H >> 3); c += 64) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int r = p; r < T; r += S) {
      float t[8];
      load8_bf16(ds + (long long)r * H + c * 8, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += t[k];
    }
    float o[8];
    load8_bf16(gP + (long long)p * H + c * 8, o);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] += acc[k];
    store8_bf16(gP + (long long)p * H + c * 8, o);
  }
}

// ---- host launchers ---------------------------------------------------------------------------------------
static inline unsigned rows_grid(long long rows) { return (unsigned)((rows + kRowsPerBlock - 1) / kRowsPerBlock); }

int ln_max_hidden() { return 64 * 8 * 4; }

void ln_fwd(const bf16_t* h, const bf16_t* res, const float* gamma, const float* beta, bf16_t* y, bf16_t* s_out,
            float* mean, float* rstd, int T, int H, float eps, float p_in, uint32_t seed_in, float p_out,
            uint32_t seed_out, hipStream_t st) {
  if (T <= 0) return;
  const uint32_t ti = drop_thresh(p_in), to = drop_thresh(p_out);
  const float si = p_in > 0.f ? 1.f / (1.f - p_in) : 1.f, so = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
  const int nch = (H / 8 + 63) / 64;
#define DTG_LNF(NC)                                                                                                   \
  do { hipLaunchKernelGGL(ln_fwd_kernel<NC>, dim3(rows_grid(T)), dim3(256), 0, st, h, res, gamma, beta, y, s_out, mean, \
                     rstd, T, H, eps, ti, si, seed_in, to, so, seed_out); DTG_LAUNCH_CHECK(); } while (0)
  if (nch <= 1) DTG_LNF(1);
  else if (nch == 2) DTG_LNF(2);
  else DTG_LNF(4);
#undef DTG_LNF
}

// Blocks of the LayerNorm backward (each folds its rows' dgamma/dbeta/dbias into one partial row of
// the workspace): at most 1024 = 4 blocks (16 waves) per CU, BERT-base b256 8.84k -> 8.88k seq/s over 512
static int ln_bwd_cap() { return 1024; }

int ln_bwd_blocks(int T) {
  const int b = (T + kRowsPerBlock - 1) / kRowsPerBlock, cap = ln_bwd_cap();
  return b < cap ? (b < 1 ? 1 : b) : cap;
}

void ln_bwd(const bf16_t* dy, const bf16_t* s, const float* gamma, const float* mean, const float* rstd,
            bf16_t* ds_out, bf16_t* dh_out, float* dgamma, float* dbeta, float* dbias, float* ws, int T, int H,
            float p_in, uint32_t seed_in, float p_out, uint32_t seed_out, hipStream_t st) {
  if (T <= 0) return;
  const uint32_t ti = drop_thresh(p_in), to = drop_thresh(p_out);
  const float si = p_in > 0.f ? 1.f / (1.f - p_in) : 1.f, so = p_out > 0.f ? 1.f / (1.f - p_out) : 1.f;
  const int nb = ln_bwd_blocks(T);
  const int nc4 = (H / 4 + 63) / 64;  // 4-element chunks per lane (H = 768: 3)
  const size_t lds = (size_t)kRowsPerBlock * 3 * H * sizeof(float);
#define DTG_LNB(NC)                                                                                                  \
  do { hipLaunchKernelGGL(ln_bwd_kernel<NC>, dim3(nb), dim3(256), lds, st, dy, s, gamma, mean, rstd, ds_out, dh_out,     \
                     ws, dbias, T, H, ti, si, seed_in, to, so, seed_out); DTG_LAUNCH_CHECK(); } while (0)
  if (nc4 <= 1) DTG_LNB(1);
  else if (nc4 == 2) DTG_LNB(2);
  else if (nc4 == 3) DTG_LNB(3);
  else if (nc4 == 4) DTG_LNB(4);
  else DTG_LNB(8);
#undef DTG_LNB
  const int ncols = dbias ? 3 * H : 2 * H;
  hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((ncols + 63) / 64, 8), dim3(256), 0, st, ws, nb, H, ncols, dgamma,
                     dbeta, dbias); DTG_LAUNCH_CHECK();
}

int attn_max_keys() { return 64 * 16; }

void attn_softmax_fwd(const float* sc, const float* mask, bf16_t* P, bf16_t* Pd, int rows, int rows_per_b, int Sk,
                      float p, uint32_t seed, hipStream_t st) {
  if (rows <= 0) return;
  const uint32_t th = drop_thresh16(p);
  const float scl = p > 0.f ? 1.f / (1.f - p) : 1.f;
  if (!th) Pd = P;
  const int nj = (Sk + 63) / 64;
#define DTG_SMF(NJ)                                                                                            \
  do { hipLaunchKernelGGL(attn_softmax_fwd_kernel<NJ>, dim3(rows_grid(rows)), dim3(256), 0, st, sc, mask, P, Pd, rows, \
                     rows_per_b, Sk, th, scl, seed); DTG_LAUNCH_CHECK(); } while (0)
  if (nj <= 1) DTG_SMF(1);
  else if (nj == 2) DTG_SMF(2);
  else if (nj <= 4) DTG_SMF(4);
  else if (nj <= 8) DTG_SMF(8);
  else DTG_SMF(16);
#undef DTG_SMF
}

void attn_softmax_bwd(const bf16_t* P, const bf16_t* Pd, const float* dPd, bf16_t* dS, int rows, int Sk, float scale,
                      hipStream_t st) {
  if (rows <= 0) return;
  const int nj = (Sk + 63) / 64;
#define DTG_SMB(NJ) \
  do { hipLaunchKernelGGL(attn_softmax_bwd_kernel<NJ>, dim3(rows_grid(rows)), dim3(256), 0, st, P, Pd, dPd, dS, rows, Sk, scale); DTG_LAUNCH_CHECK(); } while (0)
  if (nj <= 1) DTG_SMB(1);
  else if (nj == 2) DTG_SMB(2);
  else if (nj <= 4) DTG_SMB(4);
  else if (nj <= 8) DTG_SMB(8);
  else DTG_SMB(16);
#undef DTG_SMB
}

int colsum_splits(int T, int N) {
  const int cb = (N + 255) / 256;
  int s = (256 + cb - 1) / cb;
  const int maxs = (T + 7) / 8;
  if (s > maxs) s = maxs;
  if (s > 256) s = 256;
  return s < 1 ? 1 : s;
}

void colsum(const bf16_t* x, long long ld, int T, int N, const long long* sel, int nsel, void* out, int out_bf16,
            int accumulate, float* ws, int splits, hipStream_t st) {
  if (T <= 0 || N <= 0) return;
  dim3 grid((N + 255) / 256, splits);
  float* aout = (!out_bf16 && accumulate) ? (float*)out : nullptr;
  if (nsel <= 1) { hipLaunchKernelGGL(colsum_partial_kernel<1>, grid, dim3(256), 0, st, x, ld, T, N, sel, ws, aout); DTG_LAUNCH_CHECK(); }
  else { hipLaunchKernelGGL(colsum_partial_kernel<2>, grid, dim3(256), 0, st, x, ld, T, N, sel, ws, aout); DTG_LAUNCH_CHECK(); }
  if (aout) return;
  const int nsn = (nsel <= 1 ? 1 : 2) * N;
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3((nsn + 255) / 256), dim3(256), 0, st, ws, splits, nsn, out, out_bf16,
                     accumulate); DTG_LAUNCH_CHECK();
}

void emb_fwd(const long long* ids, const long long* tt, const bf16_t* word, const bf16_t* pos, const bf16_t* type,
             bf16_t* s, int T, int S, int H, hipStream_t st) {
  if (T <= 0) return;
  hipLaunchKernelGGL(emb_fwd_kernel, dim3(rows_grid(T)), dim3(256), 0, st, ids, tt, word, pos, type, s, T, S, H); DTG_LAUNCH_CHECK();
}

void emb_word_bwd(const bf16_t* ds, const long long* sorted, const long long* perm, bf16_t* gW, int T, int H,
                  hipStream_t st) {
  if (T <= 0) return;
  hipLaunchKernelGGL(emb_word_bwd_kernel, dim3(rows_grid(T)), dim3(256), 0, st, ds, sorted, perm, gW, T, H); DTG_LAUNCH_CHECK();
}

// Position-embedding grad, batch split: one workgroup per position, G groups of threads each summing
// every G-th batch row of one 8-column chunk (unrolled by 4: independent loads in flight), then an LDS
// reduction over the groups.  The one-wave-per-position form ran 128 waves for BERT's 128 positions,
// each walking its 256 batch rows serially (161 us for 50 MB at batch 256).
template <int G>
__global__ void __launch_bounds__(1024) emb_pos_bwd_split_kernel(const bf16_t* __restrict__ ds,
                                                                 bf16_t* __restrict__ gP, int T, int S, int H) {
  extern __shared__ float red[];  // [G][nch * 8]
  const int nch = H >> 3, p = blockIdx.x;
  const int c = threadIdx.x % nch, g = threadIdx.x / nch;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g < G) {
    const long long step = (long long)G * S;
    long long r = p + (long long)g * S;
    for (; r + 3 * step < T; r += 4 * step) {
      float t0[8], t1[8], t2[8], t3[8];
      load8_bf16(ds + r * H + c * 8, t0);
      load8_bf16(ds + (r + step) * H + c * 8, t1);
      load8_bf16(ds + (r + 2 * step) * H + c * 8, t2);
      load8_bf16(ds + (r + 3 * step) * H + c * 8, t3);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += (t0[k] + t1[k]) + (t2[k] + t3[k]);
    }
    for (; r < T; r += step) {
      float t[8];
      load8_bf16(ds + r * H + c * 8, t);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += t[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) red[(g * nch + c) * 8 + k] = acc[k];
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nch * 8; i += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int j = 0; j < G; ++j) v += red[j * nch * 8 + i];
    const long long o = (long long)p * H + i;
    gP[o] = f2bf(bf2f(gP[o]) + v);
  }
}

void emb_pos_bwd(const bf16_t* ds, bf16_t* gP, int T, int S, int H, hipStream_t st) {
  if (T <= 0) return;
  const int nch = H / 8;
  if (H % 8 == 0 && nch <= 128) {
    const int threads = nch * 8;  // G = 8 groups
    hipLaunchKernelGGL(emb_pos_bwd_split_kernel<8>, dim3(S), dim3(threads), (size_t)8 * nch * 8 * sizeof(float), st,
                       ds, gP, T, S, H); DTG_LAUNCH_CHECK();
    return;
  }
  hipLaunchKernelGGL(emb_pos_bwd_kernel, dim3(rows_grid(S)), dim3(256), 0, st, ds, gP, T, S, H); DTG_LAUNCH_CHECK();
}

}  // namespace dtg
