// BERT pre-training heads and their row plumbing, so the whole loss runs on dtg kernels (no vendor GEMM,
// no sort, no framework loss or index kernels on the step):
//
//   gather_rows        hm[i] = seq[(i / P) * S + pos[i]]          masked-LM rows (pos: [B, P] positions)
//   scatter_rows_add   dseq[(i / P) * S + pos[i]] += dhm[i]         (pos == null: rows i * S, the [CLS] rows);
//                      repeated positions within a sequence accumulate (added in order, one wave per sequence)
//   nsp_loss_fwd       logits = pooled Wn^T + bn ([B, 2]), softmax cross-entropy, mean over B, + the MLM
//                      loss -> the total pre-training loss (one workgroup: a deterministic reduction order)
//   nsp_loss_bwd       dlogits = (p - onehot) * g / B;  dpre = (dlogits Wn) * (1 - pooled^2)  (tanh');
//                      dWn += dlogits^T pooled;  dbn += colsum(dlogits)
//   row_sum            out = scale * sum(x)  (the MLM loss from the per-row cross-entropies)
//   emb_word_bwd_owned dWemb[v] += sum_{t: ids[t] = v} ds[t]: each workgroup OWNS a tile of vocabulary rows,
//                      scans the ids for its tile and adds the matching rows in token order -- sort-free,
//                      no atomics, deterministic (replaces a radix sort + per-run reduction)
//
// Reference: the reference trains a 2-parameter toy; this is BASELINE.json config 5 (BERT-base).
#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

namespace {

// one wave per row, 8 columns per lane per step
__global__ void __launch_bounds__(256) gather_rows_kernel(const bf16_t* __restrict__ src, const long long* __restrict__ pos,
                                                          bf16_t* __restrict__ out, int R, int P, int S, int H) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= R) return;
  const long long row = (long long)(i / P) * S + pos[i];
  const uint4* s = reinterpret_cast<const uint4*>(src + row * H);
  uint4* d = reinterpret_cast<uint4*>(out + (long long)i * H);
  for (int c = lane; c < (H >> 3); c += 64) d[c] = s[c];
}

// One wave per (sequence, 512-column block): the wave adds that sequence's P rows IN ORDER, so positions that
// repeat within a sequence (padded masked_lm_positions are commonly all 0) accumulate every update -- no lost
// read-modify-write race, and a deterministic summation order.  pos == null: P = 1, row i -> dst row i * S.
__global__ void __launch_bounds__(256) scatter_rows_add_kernel(bf16_t* __restrict__ dst, const long long* __restrict__ pos,
                                                               const bf16_t* __restrict__ src, int nseq, int P, int S,
                                                               int H) {
  const int lane = threadIdx.x & 63;
  const int nvec = H >> 3, wps = (nvec + 63) / 64;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int b = wv / wps, c = (wv % wps) * 64 + lane;
  if (b >= nseq || c >= nvec) return;
  for (int j = 0; j < P; ++j) {
    const long long i = (long long)b * P + j;
    const long long row = pos ? (long long)b * S + pos[i] : i * S;
    float a[8], v[8];
    load8_bf16(dst + row * H + c * 8, a);
    load8_bf16(src + i * H + c * 8, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += v[k];
    store8_bf16(dst + row * H + c * 8, a);
  }
}

constexpr int kNspThreads = 1024;

// single workgroup: wave w takes rows w, w + 16, ...; lane 0 keeps the wave's loss sum; the 16 wave sums
// are added in wave order
__global__ void __launch_bounds__(kNspThreads) nsp_loss_fwd_kernel(const bf16_t* __restrict__ pooled,
                                                                  const bf16_t* __restrict__ wn,
                                                                  const float* __restrict__ bn,
                                                                  const long long* __restrict__ labels,
                                                                  const float* __restrict__ extra,
                                                                  float* __restrict__ probs, float* __restrict__ out,
                                                                  int B, int H) {
  __shared__ float wsum[kNspThreads / 64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  for (int b = wave; b < B; b += kNspThreads / 64) {
    float d0 = 0.f, d1 = 0.f;
    for (int c = lane; c < (H >> 3); c += 64) {
      float x[8], w0[8], w1[8];
      load8_bf16(pooled + (long long)b * H + c * 8, x);
      load8_bf16(wn + c * 8, w0);
      load8_bf16(wn + H + c * 8, w1);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        d0 = fmaf(x[k], w0[k], d0);
        d1 = fmaf(x[k], w1[k], d1);
      }
    }
    d0 = wave_sum(d0) + bn[0];
    d1 = wave_sum(d1) + bn[1];
    const float m = fmaxf(d0, d1);
    const float e0 = __expf(d0 - m), e1 = __expf(d1 - m);
    const float lse = m + __logf(e0 + e1);
    const long long y = labels[b];
    if (lane == 0) {
      probs[2 * b] = e0 / (e0 + e1);
      probs[2 * b + 1] = e1 / (e0 + e1);
      if (y >= 0) acc += lse - (y == 0 ? d0 : d1);
    }
  }
  if (lane == 0) wsum[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < kNspThreads / 64; ++w) t += wsum[w];
    out[0] = t / (float)B + (extra ? extra[0] : 0.f);
  }
}

// grid: H / 64 workgroups of 64 columns x 16 batch groups; column reductions over the batch through LDS in a
// fixed order (deterministic)
__global__ void __launch_bounds__(1024) nsp_loss_bwd_kernel(const bf16_t* __restrict__ pooled,
                                                           const bf16_t* __restrict__ wn,
                                                           const float* __restrict__ probs,
                                                           const long long* __restrict__ labels,
                                                           const float* __restrict__ gout, bf16_t* __restrict__ dpre,
                                                           bf16_t* __restrict__ gwn, float* __restrict__ gbn, int B, int H) {
  __shared__ float red[2][16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int h = blockIdx.x * 64 + tx;
  const float g = gout[0] / (float)B;
  const float w0 = h < H ? bf2f(wn[h]) : 0.f, w1 = h < H ? bf2f(wn[H + h]) : 0.f;
  float a0 = 0.f, a1 = 0.f;
  for (int b = ty; b < B; b += 16) {
    const long long y = labels[b];
    const float s = y >= 0 ? g : 0.f;
    const float l0 = (probs[2 * b] - (y == 0 ? 1.f : 0.f)) * s;
    const float l1 = (probs[2 * b + 1] - (y == 1 ? 1.f : 0.f)) * s;
    if (h < H) {
      const float p = bf2f(pooled[(long long)b * H + h]);
      dpre[(long long)b * H + h] = f2bf((l0 * w0 + l1 * w1) * fmaf(-p, p, 1.f));
      a0 = fmaf(l0, p, a0);
      a1 = fmaf(l1, p, a1);
    }
  }
  red[0][ty][tx] = a0;
  red[1][ty][tx] = a1;
  __syncthreads();
  if (ty == 0 && h < H) {
    float t0 = 0.f, t1 = 0.f;
    for (int k = 0; k < 16; ++k) {
      t0 += red[0][k][tx];
      t1 += red[1][k][tx];
    }
    gwn[h] = f2bf(bf2f(gwn[h]) + t0);
    gwn[H + h] = f2bf(bf2f(gwn[H + h]) + t1);
  }
  if (blockIdx.x == 0 && threadIdx.x < 2) {
    const int c = threadIdx.x;
    float t = 0.f;
    for (int b = 0; b < B; ++b) {
      const long long y = labels[b];
      if (y >= 0) t += (probs[2 * b + c] - (y == c ? 1.f : 0.f)) * g;
    }
    gbn[c] += t;
  }
}

__global__ void __launch_bounds__(1024) row_sum_kernel(const float* __restrict__ x, float* __restrict__ out, long long n,
                                                      float scale) {
  __shared__ float wsum[16];
  float acc = 0.f;
  for (long long i = threadIdx.x; i < n; i += 1024) acc += x[i];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += wsum[w];
    out[0] = t * scale;
  }
}

// Word-embedding gradient, sort-free.  Workgroup w owns vocabulary rows [w*VT, (w+1)*VT).  It walks the ids in
// chunks of 2048 (8 consecutive tokens per thread, the next chunk's ids loaded under the current one), compacts
// the matching token indices IN TOKEN ORDER into an LDS list (per-thread hit counts, a block-wide exclusive
// scan), and whenever the list fills (or at the end) adds the listed rows of ds into an fp32 LDS accumulator
// [VT][H]: thread t owns 8-column chunk t and walks the list in order, 8 rows of loads in flight at a time, so
// every vocabulary row is summed in token order by exactly one thread per chunk -- deterministic without
// atomics.  Rows that received anything are added once into the bf16 gradient.  (The first form walked 256
// ids per step with one dependent load per step and one per listed row: 420 us per BERT-base step.)
constexpr int kEmbVT = 32, kEmbList = 2048, kEmbTPT = 8, kEmbChunk = 256 * kEmbTPT;

__device__ __forceinline__ void unpack8_bf16_u4(const uint4& v, float (&o)[8]) {
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  o[4] = __uint_as_float(v.z << 16); o[5] = __uint_as_float(v.z & 0xffff0000u);
  o[6] = __uint_as_float(v.w << 16); o[7] = __uint_as_float(v.w & 0xffff0000u);
}

__global__ void __launch_bounds__(256) emb_word_bwd_owned_kernel(const bf16_t* __restrict__ ds,
                                                                const long long* __restrict__ ids,
                                                                bf16_t* __restrict__ gW, int T, int H, int V) {
  extern __shared__ float acc[];  // [kEmbVT][H]
  __shared__ int list[kEmbList];
  __shared__ int wsum[4];
  __shared__ int touched[kEmbVT];
  typedef __attribute__((address_space(3))) float lds_f;
  lds_f* accl = (lds_f*)acc;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int v0 = blockIdx.x * kEmbVT;
  const int nch = H >> 3;
  for (int i = tid; i < kEmbVT * H; i += 256) accl[i] = 0.f;
  if (tid < kEmbVT) touched[tid] = 0;
  __syncthreads();
  auto flush = [&](int n) {  // list[0, n) into acc, in list (= token) order per column chunk
    for (int c = tid; c < nch; c += 256) {
      int j = 0;
      for (; j + 8 <= n; j += 8) {
        uint4 x[8];
        int r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int t = list[j + u];
          r[u] = (int)(ids[t] - v0);
          x[u] = *reinterpret_cast<const uint4*>(ds + (long long)t * H + c * 8);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float f[8];
          unpack8_bf16_u4(x[u], f);
          lds_f* a = accl + r[u] * H + c * 8;
#pragma unroll
          for (int k = 0; k < 8; ++k) a[k] += f[k];
        }
      }
      for (; j < n; ++j) {
        const int t = list[j];
        const int r = (int)(ids[t] - v0);
        float f[8];
        load8_bf16(ds + (long long)t * H + c * 8, f);
        lds_f* a = accl + r * H + c * 8;
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] += f[k];
      }
    }
  };
  long long nid[kEmbTPT];
  auto load_ids = [&](int base) {
#pragma unroll
    for (int j = 0; j < kEmbTPT; ++j) {
      const int t = base + tid * kEmbTPT + j;
      nid[j] = t < T ? ids[t] : -1;
    }
  };
  int nlist = 0;  // block-uniform
  load_ids(0);
  for (int base = 0; base < T; base += kEmbChunk) {
    long long id[kEmbTPT];
#pragma unroll
    for (int j = 0; j < kEmbTPT; ++j) id[j] = nid[j];
    if (base + kEmbChunk < T) load_ids(base + kEmbChunk);  // next chunk's ids in flight under this one
    unsigned hm = 0;
#pragma unroll
    for (int j = 0; j < kEmbTPT; ++j)
      if (id[j] >= v0 && id[j] < v0 + kEmbVT && id[j] < V) hm |= 1u << j;
    // block exclusive scan of the per-thread hit counts (thread order = token order)
    const int cnt = __popc(hm);
    int inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[wave] = inc;
    __syncthreads();
    int off = inc - cnt;
    for (int w = 0; w < wave; ++w) off += wsum[w];
    const int total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (total > 0) {
      if (nlist + total > kEmbList) {  // block-uniform: flush the list first
        flush(nlist);
        __syncthreads();
        nlist = 0;
      }
      int k = nlist + off;
#pragma unroll
      for (int j = 0; j < kEmbTPT; ++j)
        if (hm & (1u << j)) {
          list[k++] = base + tid * kEmbTPT + j;
          touched[(int)(id[j] - v0)] = 1;
        }
      nlist += total;
    }
    __syncthreads();  // list written; wsum free for the next chunk
  }
  flush(nlist);
  __syncthreads();
  for (int r = 0; r < kEmbVT && v0 + r < V; ++r) {
    if (!touched[r]) continue;
    for (int c = tid; c < nch; c += 256) {
      float o[8];
      bf16_t* g = gW + (long long)(v0 + r) * H + c * 8;
      load8_bf16(g, o);
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] += accl[r * H + c * 8 + k];
      store8_bf16(g, o);
    }
  }
}

}  // namespace

void gather_rows(const bf16_t* src, const long long* pos, bf16_t* out, int R, int P, int S, int H, hipStream_t st) {
  if (R <= 0) return;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((R + 3) / 4), dim3(256), 0, st, src, pos, out, R, P, S, H); DTG_LAUNCH_CHECK();
}

void scatter_rows_add(bf16_t* dst, const long long* pos, const bf16_t* src, int R, int P, int S, int H,
                      hipStream_t st) {
  if (R <= 0) return;
  if (!pos) P = 1;
  const int nseq = R / P, waves = nseq * (((H >> 3) + 63) / 64);
  hipLaunchKernelGGL(scatter_rows_add_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, dst, pos, src, nseq, P, S, H);
  DTG_LAUNCH_CHECK();
}

void nsp_loss_fwd(const bf16_t* pooled, const bf16_t* wn, const float* bn, const long long* labels, const float* extra,
                  float* probs, float* out, int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(nsp_loss_fwd_kernel, dim3(1), dim3(kNspThreads), 0, st, pooled, wn, bn, labels, extra, probs, out,
                     B, H); DTG_LAUNCH_CHECK();
}

void nsp_loss_bwd(const bf16_t* pooled, const bf16_t* wn, const float* probs, const long long* labels, const float* gout,
                  bf16_t* dpre, bf16_t* gwn, float* gbn, int B, int H, hipStream_t st) {
  hipLaunchKernelGGL(nsp_loss_bwd_kernel, dim3((H + 63) / 64), dim3(1024), 0, st, pooled, wn, probs, labels, gout, dpre,
                     gwn, gbn, B, H); DTG_LAUNCH_CHECK();
}

void row_sum(const float* x, float* out, long long n, float scale, hipStream_t st) {
  hipLaunchKernelGGL(row_sum_kernel, dim3(1), dim3(1024), 0, st, x, out, n, scale); DTG_LAUNCH_CHECK();
}

void emb_word_bwd_owned(const bf16_t* ds, const long long* ids, bf16_t* gW, int T, int H, int V, hipStream_t st) {
  const size_t lds = (size_t)kEmbVT * H * sizeof(float);
  static bool attr = false;
  if (!attr) {
    DTG_HIP_CHECK(hipFuncSetAttribute((const void*)emb_word_bwd_owned_kernel,
                                      hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    attr = true;
  }
  hipLaunchKernelGGL(emb_word_bwd_owned_kernel, dim3((V + kEmbVT - 1) / kEmbVT), dim3(256), lds, st, ds, ids, gW, T, H,
                     V); DTG_LAUNCH_CHECK();
}

// ---- small BERT step helpers on dtg kernels (no framework elementwise launches on the step) ------------------
// out = a * b, bf16, 8 elements per lane (the MLM head's gelu'(pre) multiply)
__global__ void __launch_bounds__(256) mul_bf16_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ out, long long n) {
  const long long nvec = n >> 3;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long v = (long long)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
    float x[8], y[8];
    load8_bf16(a + (v << 3), x);
    load8_bf16(b + (v << 3), y);
#pragma unroll
    for (int k = 0; k < 8; ++k) x[k] *= y[k];
    store8_bf16(out + (v << 3), x);
  }
  if (blockIdx.x == 0)
    for (long long i = (nvec << 3) + threadIdx.x; i < n; i += blockDim.x) out[i] = f2bf(bf2f(a[i]) * bf2f(b[i]));
}

void mul_bf16(const bf16_t* a, const bf16_t* b, bf16_t* out, long long n, hipStream_t st) {
  if (n <= 0) return;
  mul_bf16_kernel<<<grid_for((n >> 3) + 1, 256, 4096), 256, 0, st>>>(a, b, out, n); DTG_LAUNCH_CHECK();
}

// additive key mask: (1 - mask) * -10000 as fp32, from an int64 or fp32 [B, S] 1/0 mask (BERT)
template <class T>
__global__ void __launch_bounds__(256) mask_additive_kernel(const T* __restrict__ m, float* __restrict__ out, long long n) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    out[i] = (1.f - (float)m[i]) * -10000.f;
}

void mask_additive(const void* mask, int is_f32, float* out, long long n, hipStream_t st) {
  if (n <= 0) return;
  const int grid = grid_for(n, 256, 4096);
  if (is_f32) mask_additive_kernel<float><<<grid, 256, 0, st>>>((const float*)mask, out, n);
  else mask_additive_kernel<long long><<<grid, 256, 0, st>>>((const long long*)mask, out, n);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
