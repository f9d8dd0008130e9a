// Debug / fault-injection kernels (tests of the comm watchdog).
#include "kernels.h"

namespace tdl {
namespace {

// one lane spins on the 100 MHz constant clock for `ticks` (bounded by the host: ≤ 60 s)
__global__ void spin_kernel(uint64_t ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

}  // namespace

void debug_spin_launch(double ms, hipStream_t st) {
  if (ms <= 0) return;
  if (ms > 60000) ms = 60000;
  hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, st, (uint64_t)(ms * 1e5));
}

}  // namespace tdl
