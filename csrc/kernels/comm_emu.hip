// Emulated blocking collective (parallel/ddp.py, DTG_COMM_EMULATE).
//
// On one GPU a one-rank RCCL all-reduce is a local copy that finishes at once, so a one-card run never
// shows what decides multi-GPU scaling: RCCL's channel workgroups sitting on CUs for the whole
// bus-transfer time of each bucket, waiting on peers, next to the backward's kernels.  This kernel stands
// in for one such collective: `wgs` workgroups of 256 threads (RCCL launches one 256-thread block per
// channel) each hold their CU slot until `ticks` of the 100 MHz real-time counter have passed since the
// workgroup started, then exit.  Every workgroup reaches its exit (bounded by `ticks`, capped on the host).
//
// Mode bits (round 5: the round-4 form -- one sleeping lane, no memory traffic -- was optimistic only):
//   kBusy     every wave's lane 0 busy-polls the clock (no s_sleep), as RCCL's primitives spin on their
//             flags: the collective takes issue slots on every SIMD it occupies;
//   kTraffic  the workgroups also stream `traffic_bytes` (read + write, half each) through a scratch buffer,
//             spread evenly over the emulated time: the HBM traffic a ring all-reduce moves
//             (~2 (N-1)/N x bucket read and written), which the backward's HBM-bound kernels compete with;
//   kData     after the wait the bucket is read and written back multiplied by `factor` (= N): the sum of N
//             identical replicas, i.e. what an N-rank all-reduce of N equal gradients returns, so a test can
//             check that every gradient of the bucket was final when the collective read it.
#include <stdexcept>

#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

constexpr int kEmuBusy = 1, kEmuTraffic = 2, kEmuData = 4;

__global__ void __launch_bounds__(256) comm_spin_kernel(unsigned long long ticks) {
  extern __shared__ float lds_hold[];  // dynamic LDS, sized by the launch: held, never touched
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  }
  __syncthreads();
}

// scratch: `slots` windows of 32 KiB (16 KiB read + 16 KiB written per piece), far larger than the 256 MiB
// Infinity Cache so the traffic reaches HBM; piece k of workgroup b uses window (base + k * G + b) % slots, and the
// host advances `base` from launch to launch
__global__ void __launch_bounds__(256) comm_emu_kernel(unsigned long long ticks, int mode, u32x4v* __restrict__ scratch,
                                                       long long slots, long long base, long long pieces_per_wg,
                                                       void* __restrict__ buf, long long n, int buf_bf16, float factor) {
  const int tid = threadIdx.x;
  const unsigned long long t0 = wall_clock64();
  constexpr int kPieceVec = 256 * 4;  // one piece: 4 x 16 B per thread (16 KiB read + 16 KiB written)
  if (mode & kEmuTraffic) {
    for (long long k = 0; k < pieces_per_wg; ++k) {
      // piece k may start at t0 + k * ticks / pieces: the traffic is spread over the emulated bus time
      const unsigned long long due = t0 + (unsigned long long)((double)ticks * k / pieces_per_wg);
      if ((tid & 63) == 0)
        while (wall_clock64() < due) {
          if (!(mode & kEmuBusy)) __builtin_amdgcn_s_sleep(2);
        }
      u32x4v* rd = scratch + ((base + k * gridDim.x + blockIdx.x) % slots) * 2 * kPieceVec;
      u32x4v* wr = rd + kPieceVec;
      u32x4v v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(rd + tid + 256 * u);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u].x += (unsigned)k;
        __builtin_nontemporal_store(v[u], wr + tid + 256 * u);
      }
    }
  }
  if ((tid & 63) == 0 && ((mode & kEmuBusy) || tid == 0)) {
    while (wall_clock64() - t0 < ticks) {
      if (!(mode & kEmuBusy)) __builtin_amdgcn_s_sleep(8);
    }
  }
  __syncthreads();
  if (mode & kEmuData) {  // bucket *= factor (N identical replicas summed)
    const long long stride = (long long)gridDim.x * 256;
    if (buf_bf16) {
      bf16_t* b = (bf16_t*)buf;
      for (long long i = (long long)blockIdx.x * 256 + tid; i < n; i += stride) b[i] = f2bf(bf2f(b[i]) * factor);
    } else {
      float* b = (float*)buf;
      for (long long i = (long long)blockIdx.x * 256 + tid; i < n; i += stride) b[i] *= factor;
    }
  }
}

static int wall_clock_khz() {
  static int khz = 0;
  if (khz == 0) {
    int dev = 0;
    DTG_HIP_CHECK(hipGetDevice(&dev));
    DTG_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    if (khz <= 0) khz = 100000;  // gfx9 real-time counter: 100 MHz
  }
  return khz;
}

void comm_spin(double seconds, int wgs, int lds_bytes, hipStream_t st) {
  if (!(seconds > 0.0)) return;
  if (seconds > 0.1) seconds = 0.1;  // one emulated bucket never holds the chip longer than 100 ms
  if (wgs < 1) wgs = 1;
  if (wgs > 256) wgs = 256;
  if (lds_bytes < 0) lds_bytes = 0;
  if (lds_bytes > 64 * 1024) lds_bytes = 64 * 1024;
  const unsigned long long ticks = (unsigned long long)(seconds * wall_clock_khz() * 1e3);
  comm_spin_kernel<<<wgs, 256, lds_bytes, st>>>(ticks);
  DTG_LAUNCH_CHECK();
}

// returns the number of 32 KiB scratch windows this launch used (the caller's next `base` offset advance)
long long comm_emu(double seconds, int wgs, int mode, void* scratch, long long scratch_bytes, long long base,
                   long long traffic_bytes, void* buf, long long n, int buf_bf16, float factor, hipStream_t st) {
  if (seconds < 0.0) seconds = 0.0;
  if (seconds > 0.1) seconds = 0.1;
  if (wgs < 1) wgs = 1;
  if (wgs > 256) wgs = 256;
  constexpr long long kWin = 2LL * 256 * 4 * 16;  // 32 KiB: one piece's read + write halves
  long long pieces = 0, slots = 1;
  if ((mode & kEmuTraffic) && traffic_bytes > 0) {
    slots = scratch == nullptr ? 0 : scratch_bytes / kWin;
    if (slots < wgs) throw std::runtime_error("comm_emu: scratch smaller than 32 KiB per workgroup");
    pieces = (traffic_bytes + (long long)wgs * kWin - 1) / ((long long)wgs * kWin);
  } else {
    mode &= ~kEmuTraffic;
  }
  if (!(mode & kEmuData)) n = 0;
  const unsigned long long ticks = (unsigned long long)(seconds * wall_clock_khz() * 1e3);
  comm_emu_kernel<<<wgs, 256, 0, st>>>(ticks, mode, (u32x4v*)scratch, slots, base % slots, pieces, buf, n, buf_bf16,
                                       factor);
  DTG_LAUNCH_CHECK();
  return pieces * wgs;
}

// Test hook for the launch checks: the same kernel with an unvalidated grid / dynamic LDS size, so a test can
// request an impossible launch (grid 0, LDS above the 160 KB per-CU limit) and expect a Python RuntimeError.
void launch_probe(int grid, int lds_bytes, hipStream_t st) {
  comm_spin_kernel<<<grid, 256, lds_bytes, st>>>(0ull);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
