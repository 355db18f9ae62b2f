// Emulated blocking collective (parallel/ddp.py, DTG_COMM_EMULATE).
//
// On one GPU a one-rank RCCL all-reduce is a local copy that finishes at once, so a one-card run never
// shows what decides multi-GPU scaling: RCCL's channel workgroups sitting on CUs for the whole
// bus-transfer time of each bucket, waiting on peers, next to the backward's kernels.  This kernel stands
// in for one such collective: `wgs` workgroups of 256 threads (RCCL launches one 256-thread block per
// channel) each hold their CU slot (waves + optional LDS) until `ticks` of the 100 MHz real-time counter
// have passed since the workgroup started, then exit.  The spinning lane sleeps between polls, so the
// emulation takes CU residency but almost no issue slots -- an optimistic stand-in for RCCL's busy-polling
// blocks, pessimistic nowhere.  Every workgroup reaches its exit (bounded by `ticks`, capped on the host).
#include <stdexcept>

#include "dtg/common.h"
#include "dtg/kernels.h"

namespace dtg {

__global__ void __launch_bounds__(256) comm_spin_kernel(unsigned long long ticks) {
  extern __shared__ float lds_hold[];  // dynamic LDS, sized by the launch: held, never touched
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  }
  __syncthreads();
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

// Test hook for the launch checks: the same kernel with an unvalidated grid / dynamic LDS size, so a test can
// request an impossible launch (grid 0, LDS above the 160 KB per-CU limit) and expect a Python RuntimeError.
void launch_probe(int grid, int lds_bytes, hipStream_t st) {
  comm_spin_kernel<<<grid, 256, lds_bytes, st>>>(0ull);
  DTG_LAUNCH_CHECK();
}

}  // namespace dtg
