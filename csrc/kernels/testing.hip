// Test support kernels (not on any metric path).
//
// spin_on_flag: one lane polls a pinned, device-visible host flag until it becomes nonzero or
// max_ms of wall clock have passed, whichever comes first, so every wave always exits.  Tests
// use it to hold a stream ahead of a collective and exercise the sync deadline
// (tests/gpu/test_rccl_direct.py).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

__global__ __launch_bounds__(kWave) void spin_on_flag_kernel(const int* flag, uint64_t max_ticks) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = wall_clock64();  // constant 100 MHz counter
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    if (wall_clock64() - t0 > max_ticks) break;
    __builtin_amdgcn_s_sleep(64);
  }
}

}  // namespace

int launch_spin_on_flag(const int* flag, int64_t max_ms, hipStream_t stream) {
  if (!flag || max_ms <= 0) return -1;
  const uint64_t ticks = static_cast<uint64_t>(max_ms) * 100000ull;  // 100 MHz
  hipLaunchKernelGGL(spin_on_flag_kernel, dim3(1), dim3(kWave), 0, stream, flag, ticks);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
