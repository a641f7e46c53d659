// Standalone A/B harness for K5b (rowsums.hip): Sum / PSNR-auto / CTR-64 shapes, grid kernel
// with different block counts per row vs the one-launch fold, all in one process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc/include csrc/bench/k5b_variants.hip -o k5bv
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../kernels/rowsums.hip"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

using namespace tea;

static double time_us(RowSumsArgs a, int reps) {
  for (int i = 0; i < 5; ++i) CK(static_cast<hipError_t>(launch_row_sums(a, 0)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; ++i) CK(static_cast<hipError_t>(launch_row_sums(a, 0)));
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3 / reps;
}

int main() {
  const int64_t N = 8192 * 1000;
  float *x, *t, *w;
  double *out, *ws;
  unsigned* ticket;
  CK(hipMalloc(&x, N * 4));
  CK(hipMalloc(&t, N * 4));
  CK(hipMalloc(&w, N * 4));
  CK(hipMalloc(&out, 64 * 8 * 4));
  CK(hipMalloc(&ws, 64 << 20));
  CK(hipMalloc(&ticket, 4096));
  CK(hipMemset(ticket, 0, 4096));
  std::vector<float> h(N);
  for (int64_t i = 0; i < N; ++i) h[i] = static_cast<float>((i * 2654435761u) % 1000) / 1000.f;
  CK(hipMemcpy(x, h.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(t, h.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, h.data(), N * 4, hipMemcpyHostToDevice));
  struct Case { const char* name; int64_t rows; bool has_t, has_w; int need; int nout; int stats[3]; int ops[3]; };
  const Case cases[] = {
      {"sum 8192x1000", 1, false, false, 1 << kWX, 1, {kWX, 0, 0}, {kAdd, 0, 0}},
      {"psnr-auto 8192x1000", 1, true, false, (1 << kSSE) | (1 << kTMIN) | (1 << kTMAX), 3, {kSSE, kTMIN, kTMAX}, {kAdd, kMin, kMax}},
      {"ctr 64x128000 weighted", 64, true, true, (1 << kWX) | (1 << kW), 2, {kWX, kW, 0}, {kAdd, kAdd, 0}},
      {"ctr 64x128000 unweighted", 64, false, false, 1 << kWX, 1, {kWX, 0, 0}, {kAdd, 0, 0}},
      {"weighted sum 1x8.2M", 1, false, true, (1 << kWX) | (1 << kW), 2, {kWX, kW, 0}, {kAdd, kAdd, 0}},
  };
  for (const Case& c : cases) {
    RowSumsArgs a;
    a.x = x;
    a.x_rs = N / c.rows;
    a.t = c.has_t ? t : nullptr;
    a.t_rs = N / c.rows;
    a.w = c.has_w ? w : nullptr;
    a.w_rs = N / c.rows;
    a.rows = c.rows;
    a.n = N / c.rows;
    a.need = c.need;
    a.nout = c.nout;
    for (int k = 0; k < c.nout; ++k) {
      a.out[k].p = out + k * 64;
      a.out[k].dt = DType::f64;
      a.out[k].stride = 1;
      a.out[k].stat = c.stats[k];
      a.out[k].op = c.ops[k];
    }
    a.ws = ws;
    const int64_t chunks = (a.n + 4095) / 4096;
    for (int cap : {2048, 512}) {
      a.ticket = nullptr;
      a.blocks = static_cast<int>(std::min<int64_t>(chunks, std::max<int64_t>(2, cap / c.rows)));
      printf("{\"case\": \"%s\", \"variant\": \"grid+combine\", \"blocks_per_row\": %d, \"us\": %.2f}\n", c.name, a.blocks,
             time_us(a, 200));
    }
    a.ticket = ticket;
    a.blocks = row_sums_fold_blocks(a.rows, a.n);
    printf("{\"case\": \"%s\", \"variant\": \"fold\", \"blocks_per_row\": %d, \"us\": %.2f}\n", c.name, a.blocks, time_us(a, 200));
  }
  return 0;
}
