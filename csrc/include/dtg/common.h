// Shared device helpers for dtg's gfx950 (CDNA4) kernels.
// Wave64 everywhere; bf16 is carried as raw 16-bit words and converted with the native
// v_cvt_pk_bf16_f32 path (plain __bf16 casts lower to it at -O3 on gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <stdexcept>

namespace dtg {

constexpr int kWave = 64;

typedef unsigned short bf16_t;  // raw bf16 bits
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(bf16_t, b);
}

// pack two floats into one dword of 2x bf16 (lo in low half): ONE v_cvt_pk_bf16_f32 with both sources (two
// scalar conversions cost a convert each plus a shift and an or)
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;
typedef __attribute__((ext_vector_type(2))) float f32x2v;
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  const bf16x2v b = __builtin_convertvector((f32x2v){lo, hi}, bf16x2v);
  return __builtin_bit_cast(uint32_t, b);
}

struct alignas(16) u32x4 { uint32_t x, y, z, w; };

// Load 8 bf16 (16 bytes) -> 8 floats.
__device__ __forceinline__ void load8_bf16(const bf16_t* p, float (&o)[8]) {
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  o[4] = __uint_as_float(v.z << 16); o[5] = __uint_as_float(v.z & 0xffff0000u);
  o[6] = __uint_as_float(v.w << 16); o[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ void store8_bf16(bf16_t* p, const float (&o)[8]) {
  uint4 v;
  v.x = pack_bf2(o[0], o[1]); v.y = pack_bf2(o[2], o[3]);
  v.z = pack_bf2(o[4], o[5]); v.w = pack_bf2(o[6], o[7]);
  *reinterpret_cast<uint4*>(p) = v;
}

// store8_bf16 with a non-temporal hint: for tensors read again only much later (saved for backward)
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4v;
__device__ __forceinline__ void store8_bf16_nt(bf16_t* p, const float (&o)[8]) {
  u32x4v v;
  v.x = pack_bf2(o[0], o[1]); v.y = pack_bf2(o[2], o[3]);
  v.z = pack_bf2(o[4], o[5]); v.w = pack_bf2(o[6], o[7]);
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4v*>(p));
}

// load8_bf16 with a non-temporal hint: the last read of a tensor in this step (its lines are evicted first,
// so freshly written data that the next kernel reads stays in the caches)
__device__ __forceinline__ void load8_bf16_nt(const bf16_t* p, float (&o)[8]) {
  const u32x4v v = __builtin_nontemporal_load(reinterpret_cast<const u32x4v*>(p));
  o[0] = __uint_as_float(v.x << 16); o[1] = __uint_as_float(v.x & 0xffff0000u);
  o[2] = __uint_as_float(v.y << 16); o[3] = __uint_as_float(v.y & 0xffff0000u);
  o[4] = __uint_as_float(v.z << 16); o[5] = __uint_as_float(v.z & 0xffff0000u);
  o[6] = __uint_as_float(v.w << 16); o[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ void load8_f32(const float* p, float (&o)[8]) {
  const float4 a = *reinterpret_cast<const float4*>(p);
  const float4 b = *reinterpret_cast<const float4*>(p + 4);
  o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
}

__device__ __forceinline__ void store8_f32(float* p, const float (&o)[8]) {
  *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a linear workgroup id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): consecutive logical tiles land on the same XCD (same L2).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int NX = 8;
  if (nwg <= NX) return orig;
  const int q = nwg / NX, r = nwg % NX, xcd = orig % NX;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / NX;
}

inline int grid_for(long long n_vec, int block, int cap = 2048) {
  long long g = (n_vec + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace dtg

namespace dtg {
// A failed HIP call or kernel launch (too much LDS for a new shape, an invalid grid, a dead device) raises:
// pybind11 turns std::runtime_error into a Python RuntimeError, so no op returns an unwritten output.
[[noreturn]] inline void hip_fail(hipError_t e, const char* what, const char* file, int line) {
  char buf[512];
  snprintf(buf, sizeof(buf), "dtg: %s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
  throw std::runtime_error(buf);
}

// After every <<<>>> launch.  hipErrorNotReady is the "still running" answer of an earlier stream / event
// query (the caching allocator polls events), never a launch failure.
inline void launch_check(const char* file, int line) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess && e != hipErrorNotReady) hip_fail(e, "kernel launch", file, line);
}
}  // namespace dtg

#define DTG_HIP_CHECK(expr)                                         \
  do {                                                              \
    hipError_t _e = (expr);                                         \
    if (_e != hipSuccess) ::dtg::hip_fail(_e, #expr, __FILE__, __LINE__); \
  } while (0)

#define DTG_LAUNCH_CHECK() ::dtg::launch_check(__FILE__, __LINE__)
