// K3t: trapezoid area of x-sorted (x, y) rows - the tail of AUC(reorder=True) on K3a.
//
// Reference (torcheval/metrics/functional/aggregation/auc.py:10-33, class aggregation/auc.py:
// 94-119): torch.sort(x, stable=True) + gather(y) + torch.trapz(y, x), float32.  Here the x rows
// come out of K3a's ascending stable sort with y carried through as the payload (its f32 bits in
// the int32 order buffer, so no gather), and this kernel sums (x[i+1] - x[i]) (y[i+1] + y[i]) / 2:
// the differences and pair sums in float32 as the reference forms them, the products and the sum
// in FP64.  Grid blocks write FP64 partials of fixed spans; one combine wave per row adds them in
// block order (deterministic) and stores the float32 area.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tea_kernels.h"

namespace tea {
namespace {

constexpr int kTT = 256;
constexpr int kTPer = 8;  // elements per thread per round (loads in flight)

__global__ __launch_bounds__(kTT) void trapz_partial_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                           int64_t n, int64_t span, double* __restrict__ part,
                                                           int blocks) {
  const int64_t row = blockIdx.y;
  const float* xr = x + row * n;
  const float* yr = y + row * n;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * span;
  const int64_t hi = min(n - 1, lo + span);  // segments [i, i + 1] with i < n - 1
  double acc = 0.0;
  for (int64_t base = lo; base < hi; base += static_cast<int64_t>(kTT) * kTPer) {
    float xa[kTPer], xb[kTPer], ya[kTPer], yb[kTPer];
#pragma unroll
    for (int u = 0; u < kTPer; ++u) {  // clamped (always valid) addresses, masked below
      const int64_t i = base + u * kTT + threadIdx.x;
      const int64_t ic = i < hi ? i : lo;
      xa[u] = xr[ic];
      xb[u] = xr[ic + 1];
      ya[u] = yr[ic];
      yb[u] = yr[ic + 1];
    }
#pragma unroll
    for (int u = 0; u < kTPer; ++u) {
      const int64_t i = base + u * kTT + threadIdx.x;
      const float dx = xb[u] - xa[u];
      const float sy = yb[u] + ya[u];
      acc += i < hi ? static_cast<double>(dx) * static_cast<double>(sy) : 0.0;
    }
  }
  // block sum: wave shuffles, then the 4 wave totals in order
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  __shared__ double w[kTT / 64];
  if ((threadIdx.x & 63) == 0) w[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[row * blocks + blockIdx.x] = ((w[0] + w[1]) + (w[2] + w[3]));
}

__global__ __launch_bounds__(64) void trapz_combine_kernel(const double* __restrict__ part, int blocks,
                                                          float* __restrict__ out) {
  const int64_t row = blockIdx.x;
  double acc = 0.0;
  for (int b = threadIdx.x; b < blocks; b += 64) acc += part[row * blocks + b];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (threadIdx.x == 0) out[row] = static_cast<float>(0.5 * acc);
}

}  // namespace

int trapz_blocks(int64_t n) {
  const int64_t per = static_cast<int64_t>(kTT) * kTPer;
  const int64_t b = (n + per - 1) / per;
  return static_cast<int>(b < 1 ? 1 : (b > 256 ? 256 : b));
}

int launch_trapz_sorted(const float* x, const float* y, int64_t rows, int64_t n, double* part, float* out,
                        hipStream_t stream) {
  if (rows <= 0) return 0;
  const int blocks = trapz_blocks(n);
  const int64_t per = static_cast<int64_t>(kTT) * kTPer;
  const int64_t segs = n > 1 ? n - 1 : 0;
  const int64_t span = ((segs + blocks - 1) / blocks + per - 1) / per * per;
  hipLaunchKernelGGL(trapz_partial_kernel, dim3(blocks, static_cast<unsigned>(rows)), dim3(kTT), 0, stream, x, y,
                     n, span > 0 ? span : per, part, blocks);
  hipLaunchKernelGGL(trapz_combine_kernel, dim3(static_cast<unsigned>(rows)), dim3(64), 0, stream, part, blocks, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea
