// Standalone A/B harness for K8 (fid_cov.hip) at 1000 x 2048 and 50000 x 2048: times the
// production launcher; build with -DTEA_K8_NO_STAGE_LOADS to time the K loop without its
// per-stage global loads / LDS commits (numerically meaningless; isolates MFMA + LDS +
// barrier cost from load latency), -DTEA_K8_SCHED=0 for the compiler's default schedule.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include csrc/bench/k8_variants.hip -o k8v
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../kernels/fid_cov.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int64_t d = 2048;
  const int64_t ns[] = {1000, 8192, 50000};
  for (int64_t n : ns) {
    float *act, *cov, *cs;
    CK(hipMalloc(&act, n * d * 4));
    CK(hipMalloc(&cov, d * d * 4));
    CK(hipMalloc(&cs, d * 4));
    std::vector<float> h(n * d);
    uint64_t st = 0x9e3779b97f4a7c15ull;  // full-mantissa uniform values in [-1, 1)
    for (size_t i = 0; i < h.size(); ++i) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      h[i] = static_cast<float>(static_cast<int32_t>(st >> 32)) * 4.656612873e-10f;
    }
    CK(hipMemcpy(act, h.data(), n * d * 4, hipMemcpyHostToDevice));
    CK(hipMemset(cov, 0, d * d * 4));
    tea::FidCovArgs a;
    a.act = act;
    a.n = n;
    a.d = d;
    a.row_stride = d;
    a.cov = cov;
    a.colsum = cs;
    a.split = 1;
    a.ld = d;
    float* zeros;
    CK(hipMalloc(&zeros, 64));
    CK(hipMemset(zeros, 0, 64));
    a.zeros = zeros;
    for (int i = 0; i < 3; ++i) CK(static_cast<hipError_t>(tea::launch_fid_cov(a, 0)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = n > 10000 ? 10 : 50;
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < reps; ++i) CK(static_cast<hipError_t>(tea::launch_fid_cov(a, 0)));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / reps;
    const double T = (d + 95) / 96;
    const double flops = 2.0 * n * 96 * 96 * T * (T + 1) / 2;
    printf("{\"n\": %ld, \"d\": %ld, \"us\": %.2f, \"tflops_tri\": %.1f}\n", (long)n, (long)d, us, flops / us / 1e6);
    CK(hipFree(act));
    CK(hipFree(cov));
    CK(hipFree(cs));
  }
  return 0;
}
