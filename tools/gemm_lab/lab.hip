// Standalone GEMM lab (not part of the package): C[M,N] = A[M,K] * B[N,K]^T, bf16 in, bf16 out,
// for iterating on main-loop schedules without rebuilding the extension.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I csrc/include tools/gemm_lab/lab.hip -o tools/gemm_lab/lab
//   tools/gemm_lab/lab M N K [iters]
// Variants are timed interleaved in one process (cdna_hip_programming.md §5.4 rule 24) on uniform
// random [-1, 1) operands, and checked against an fp32 reference GEMM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>
#include "dtg/common.h"
#include "dtg/mfma_gemm.cuh"

using namespace dtg;
using namespace dtg::gemm;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// ---------------------------------------------------------------------------------------------
// v1: 256x256 tile, 4 waves (2x2), each wave 128x128 = acc[8][8] of 16x16 (256 registers), one wave
// per SIMD.  BK = 64, 2 LDS stages (128 KB), one barrier per K-tile placed between the two 32-deep
// k-steps: the ks1 fragments are read under the ks0 MFMAs, the next tile's ks0 fragments under the
// ks1 MFMAs, and the DMA of tile t+2 is issued right after the barrier (1.5 tiles of flight).
namespace v1 {
constexpr int BM = 256, NW = 4, NTH = 256;
constexpr int A_BYTES = BM * 64 * 2;             // A operand, one stage: 32 KB

template <int JN, class SA, class SB>
__device__ __forceinline__ void stage_tile(const SA& sa, const SB& sb, lds_char* buf, int bm0, int bn0, int k0, int wave,
                                           int lane) {
  stage_kc<BM, SA, NW>(sa, buf, bm0, k0, wave, lane);
  stage_kc<32 * JN, SB, NW>(sb, buf + A_BYTES, bn0, k0, wave, lane);
}

template <int JN>
__device__ __forceinline__ void read_frags(const lds_char* buf, int wm, int wn, int ks, int lane, v8bf (&a)[8],
                                           v8bf (&b)[JN]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = frag_kc(buf, wm * 128 + i * 16, ks, lane);
#pragma unroll
  for (int j = 0; j < JN; ++j) b[j] = frag_kc(buf + A_BYTES, wn * 16 * JN + j * 16, ks, lane);
}

template <int JN>
__device__ __forceinline__ void mfma_block(const v8bf (&a)[8], const v8bf (&b)[JN], f32x4 (&acc)[8][JN]) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
}

template <int SCHED, int JN = 8>
__global__ void __launch_bounds__(NTH, 1) kern(const bf16_t* __restrict__ A, const bf16_t* __restrict__ B,
                                               bf16_t* __restrict__ C, int M, int N, int K) {
  constexpr int BN = 32 * JN, STAGE = A_BYTES + BN * 64 * 2, LDS = 2 * STAGE;
  __shared__ __attribute__((aligned(16))) char smem_raw[LDS];
  lds_char* smem = (lds_char*)smem_raw;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = N / BN;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int bm0 = (t / tiles_n) * BM, bn0 = (t % tiles_n) * BN;
  DenseKC<false> sa{A, K, M, K};
  DenseKC<false> sb{B, K, N, K};
  const int nk = K / 64;
  f32x4 acc[8][JN];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  v8bf a0[8], b0[JN], a1[8], b1[JN];
  constexpr int LPT = 8 + JN;  // LDS-DMA instructions per wave per K-tile (A: 256/32, B: 32*JN/32)
  // prologue: tiles 0 and 1 in flight, tile 0 visible, ks0 fragments of tile 0 in registers
  stage_tile<JN>(sa, sb, smem, bm0, bn0, 0, wave, lane);
  if (nk > 1) stage_tile<JN>(sa, sb, smem + STAGE, bm0, bn0, 64, wave, lane);
  if (nk > 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPT) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  read_frags(smem, wm, wn, 0, lane, a0, b0);
  for (int kt = 0; kt < nk; ++kt) {
    lds_char* cur = smem + (kt & 1) * STAGE;
    lds_char* nxt = smem + ((kt + 1) & 1) * STAGE;
    // first half: ks0 MFMAs under the ks1 reads of this tile
    read_frags(cur, wm, wn, 1, lane, a1, b1);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);  // reads issued ahead of the MFMAs
    mfma_block(a0, b0, acc);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      }
    }
    // every ds_read of this tile retired; tile kt+1's DMA (this wave's part) landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // tile kt+1 visible to all; nobody reads buffer (kt & 1) any more
    if (kt + 2 < nk) stage_tile<JN>(sa, sb, cur, bm0, bn0, (kt + 2) * 64, wave, lane);
    read_frags(nxt, wm, wn, 0, lane, a0, b0);  // (past the last tile: harmless reads of stale LDS)
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    mfma_block(a1, b1, acc);
    if constexpr (SCHED == 2) __builtin_amdgcn_sched_barrier(0);
    if constexpr (SCHED == 1) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);  // VMEM read (LDS-DMA)
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // MFMA
      }
    }
  }
  // epilogue: bf16 through LDS, one 32 KB [128][128] region per wave, 16-B row stores
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  lds_char* reg = smem + wave * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < JN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = i * 16 + (lane >> 4) * 4 + r, col = j * 16 + (lane & 15);
        // 16-B chunk XOR (row & 15) keeps the column writes spread over the banks
        const int off = row * 256 + ((((col >> 3) ^ (row & 15))) << 4) + (col & 7) * 2;
        *reinterpret_cast<__attribute__((address_space(3))) bf16_t*>(reg + off) = f2bf(acc[i][j][r]);
      }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll 4
  for (int c = lane; c < 128 * 2 * JN; c += 64) {
    const int row = c / (2 * JN), ch = c % (2 * JN);
    const v8bf v = *reinterpret_cast<const lds_v8bf*>(reg + row * 256 + ((ch ^ (row & 15)) << 4));
    *reinterpret_cast<v8bf*>(C + (long long)(bm0 + wm * 128 + row) * N + bn0 + wn * 16 * JN + ch * 8) = v;
  }
}
}  // namespace v1

// ---------------------------------------------------------------------------------------------
// reference: fp32 accumulate, one thread per output
__global__ void ref_kernel(const bf16_t* A, const bf16_t* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(long long)m * K + k]) * bf2f(B[(long long)n * K + k]);
  C[(long long)m * N + n] = s;
}

static uint16_t f2bf_host(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7FFF + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f_host(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

typedef void (*launch_fn)(const bf16_t*, const bf16_t*, bf16_t*, int, int, int, hipStream_t);

template <int S, int JN = 8>
static void launch_v1(const bf16_t* A, const bf16_t* B, bf16_t* C, int M, int N, int K, hipStream_t st) {
  if (N % (32 * JN)) return;
  hipLaunchKernelGGL((v1::kern<S, JN>), dim3((M / 256) * (N / (32 * JN))), dim3(256), 0, st, A, B, C, M, N, K);
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096, N = argc > 2 ? atoi(argv[2]) : 4096, K = argc > 3 ? atoi(argv[3]) : 4096;
  const int iters = argc > 4 ? atoi(argv[4]) : 20;
  if (M % 256 || N % 256 || K % 64) {
    printf("shape must be multiples of 256 x 256 x 64\n");
    return 1;
  }
  std::vector<uint16_t> ha((size_t)M * K), hb((size_t)N * K);
  uint32_t s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xFFFF) / 32768.0f - 1.0f; };
  for (auto& v : ha) v = f2bf_host(rnd());
  for (auto& v : hb) v = f2bf_host(rnd());
  bf16_t *A, *B, *C;
  float* R;
  CK(hipMalloc(&A, ha.size() * 2));
  CK(hipMalloc(&B, hb.size() * 2));
  CK(hipMalloc(&C, (size_t)M * N * 2));
  CK(hipMalloc(&R, (size_t)M * N * 4));
  CK(hipMemcpy(A, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, A, B, R, M, N, K);
  CK(hipDeviceSynchronize());
  std::vector<float> hr((size_t)M * N);
  CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
  struct V { const char* name; launch_fn f; std::vector<float> ms; };
  std::vector<V> vs = {{"v1 4w 128x128/wave", launch_v1<0>, {}}, {"v1 + sched groups", launch_v1<1>, {}},
                         {"v1 + sched_barrier fences", launch_v1<2>, {}},
                         {"v1 256x192 (128x96/wave)", launch_v1<0, 6>, {}},
                         {"v1 256x192 fences", launch_v1<2, 6>, {}}};
  std::vector<uint16_t> hc((size_t)M * N);
  for (auto& v : vs) {  // correctness
    CK(hipMemset(C, 0, (size_t)M * N * 2));
    v.f(A, B, C, M, N, K, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
    double maxerr = 0, maxref = 0;
    for (size_t i = 0; i < hc.size(); ++i) {
      maxerr = std::max(maxerr, (double)fabsf(bf2f_host(hc[i]) - hr[i]));
      maxref = std::max(maxref, (double)fabsf(hr[i]));
    }
    printf("%-28s max|err| %.4g (max|ref| %.4g)%s\n", v.name, maxerr, maxref, maxerr > 1e-2 * maxref ? "  WRONG" : "");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int round = 0; round < 5; ++round)
    for (auto& v : vs) {
      for (int i = 0; i < 3; ++i) v.f(A, B, C, M, N, K, 0);
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < iters; ++i) v.f(A, B, C, M, N, K, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / iters);
    }
  const double flop = 2.0 * M * N * K;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    printf("%-28s %dx%dx%d  median %.1f us  min %.1f us  %.0f TF/s\n", v.name, M, N, K, v.ms[2] * 1e3, v.ms[0] * 1e3,
           flop / (v.ms[2] * 1e-3) / 1e12);
  }
  return 0;
}
