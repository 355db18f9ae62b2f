// HBM streaming probe: the bandwidth ceiling the ResNet step's streaming kernels are judged against.
//
// torch's copy_ / sum (tools/hbm_roof.py, round 4) under-read the card: dtg's own BN passes ran faster than
// that "ceiling".  These kernels stream with the access shape the BN / dx passes use -- 16-B vector loads and
// stores per lane, U independent vectors in flight per lane, optional non-temporal hints, a grid that is a
// whole number of workgroups per CU -- so the ceiling is measured with the same instruments as the kernels.
//
//   kind 0  read-only    r[i]                 (a u32 xor per block is the only write: nothing is elided)
//   kind 1  write-only   o[i] = const
//   kind 2  copy         o[i] = a[i]
//   kind 3  read2/write1 o[i] = a[i] + b[i]   (integer add on the raw words: no VALU cost to speak of)
//
// Each workgroup streams a contiguous slab of n / G vectors (tail to the last), U vectors per lane per
// iteration, so every wave keeps U x 1 KiB of loads in flight.
#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

namespace {

template <int KIND, int U, bool NT>
__global__ void __launch_bounds__(256) stream_probe_kernel(const u32x4v* __restrict__ a, const u32x4v* __restrict__ b,
                                                          u32x4v* __restrict__ o, long long n, unsigned* __restrict__ sink) {
  const long long G = gridDim.x;
  const long long per = (n / G) / (256 * U) * (256 * U);  // whole iterations per workgroup
  const long long beg = (long long)blockIdx.x * per;
  const long long end = blockIdx.x == G - 1 ? n : beg + per;
  u32x4v acc = {0u, 0u, 0u, 0u};
  long long i = beg + threadIdx.x;
  for (; i + 256LL * (U - 1) < end; i += 256LL * U) {
    u32x4v va[U], vb[U];
    if constexpr (KIND != 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) va[u] = NT ? __builtin_nontemporal_load(a + i + 256LL * u) : a[i + 256LL * u];
    }
    if constexpr (KIND == 3) {
#pragma unroll
      for (int u = 0; u < U; ++u) vb[u] = NT ? __builtin_nontemporal_load(b + i + 256LL * u) : b[i + 256LL * u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (KIND == 0) {
        acc ^= va[u];
      } else {
        u32x4v v;
        if constexpr (KIND == 1) v = u32x4v{(unsigned)u, 1u, 2u, 3u};
        else if constexpr (KIND == 2) v = va[u];
        else v = va[u] + vb[u];
        if (NT) __builtin_nontemporal_store(v, o + i + 256LL * u);
        else o[i + 256LL * u] = v;
      }
    }
  }
  for (; i < end; i += 256) {  // tail (last workgroup only)
    if constexpr (KIND == 0) acc ^= a[i];
    else if constexpr (KIND == 1) o[i] = u32x4v{0u, 1u, 2u, 3u};
    else if constexpr (KIND == 2) o[i] = a[i];
    else o[i] = a[i] + b[i];
  }
  if constexpr (KIND == 0) {
    const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (x == 0x9e3779b9u) sink[blockIdx.x] = x;  // data-dependent, practically never taken: keeps the loads
  }
}

template <int KIND, bool NT>
void launch_u(int unroll, const u32x4v* a, const u32x4v* b, u32x4v* o, long long n, unsigned* sink, int G,
              hipStream_t st) {
  switch (unroll) {
    case 1: stream_probe_kernel<KIND, 1, NT><<<G, 256, 0, st>>>(a, b, o, n, sink); break;
    case 2: stream_probe_kernel<KIND, 2, NT><<<G, 256, 0, st>>>(a, b, o, n, sink); break;
    case 8: stream_probe_kernel<KIND, 8, NT><<<G, 256, 0, st>>>(a, b, o, n, sink); break;
    default: stream_probe_kernel<KIND, 4, NT><<<G, 256, 0, st>>>(a, b, o, n, sink); break;
  }
  DTG_LAUNCH_CHECK();
}

template <int KIND>
void launch_k(int unroll, bool nt, const u32x4v* a, const u32x4v* b, u32x4v* o, long long n, unsigned* sink, int G,
              hipStream_t st) {
  if (nt) launch_u<KIND, true>(unroll, a, b, o, n, sink, G, st);
  else launch_u<KIND, false>(unroll, a, b, o, n, sink, G, st);
}

}  // namespace

void stream_probe(int kind, const void* a, const void* b, void* o, long long n16, unsigned* sink, int wgs, int unroll,
                  int nt, hipStream_t st) {
  if (n16 <= 0) return;
  if (wgs < 1) wgs = 1;
  const u32x4v* pa = (const u32x4v*)a;
  const u32x4v* pb = (const u32x4v*)b;
  u32x4v* po = (u32x4v*)o;
  switch (kind) {
    case 0: launch_k<0>(unroll, nt, pa, pb, po, n16, sink, wgs, st); break;
    case 1: launch_k<1>(unroll, nt, pa, pb, po, n16, sink, wgs, st); break;
    case 2: launch_k<2>(unroll, nt, pa, pb, po, n16, sink, wgs, st); break;
    default: launch_k<3>(unroll, nt, pa, pb, po, n16, sink, wgs, st); break;
  }
}

}  // namespace dtg
