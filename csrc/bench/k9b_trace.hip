// K9b per-phase timeline: builds csrc/kernels/symeig.hip with TEA_SYMEIG_TRACE, runs the
// D = 2048 tridiagonalisation on a dense symmetric matrix and prints, for workgroups 0 and 100
// and 16 consecutive columns, the cycles spent waiting for the hand-off and in each step.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Icsrc/include csrc/bench/k9b_trace.hip -o /tmp/k9b_trace
#define TEA_SYMEIG_TRACE 1
#include "../kernels/symeig.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main() {
  const int n = 2048;
  std::vector<double> h((size_t)n * n);
  unsigned long long st = 12345;
  auto rnd = [&]() {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return (double)((st >> 11) & ((1ull << 53) - 1)) / (double)(1ull << 53) * 2.0 - 1.0;
  };
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) h[(size_t)i * n + j] = h[(size_t)j * n + i] = rnd() + (i == j ? 4.0 : 0.0);
  tea::SymEigArgs a;
  a.n = n;
  a.ld = tea::symeig_slot_stride(n);
  double *dA, *dd, *de, *dl;
  unsigned long long *gran, *trace;
  unsigned* ctl;
  const size_t gbytes = (size_t)4 * (n - 2) * a.ld * 8;
  CK(hipMalloc(&dA, (size_t)n * n * 8));
  CK(hipMalloc(&dd, a.ld * 8));
  CK(hipMalloc(&de, a.ld * 8));
  CK(hipMalloc(&dl, n * 8));
  CK(hipMalloc(&gran, gbytes));
  CK(hipMalloc(&ctl, 2048));
  CK(hipMalloc(&trace, 2 * 16 * 8 * 8));
  int* grid = nullptr;  // Sturm-count grid of the eigenvalue search (round 3 on)
  CK(hipMalloc(&grid, tea::symeig_grid_bytes()));
  CK(hipMemset(gran, 0, gbytes));
  CK(hipMemset(trace, 0, 2 * 16 * 8 * 8));
  CK(hipMemcpy(dA, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tea::g_symeig_trace), &trace, sizeof(trace)));
  unsigned long long* col = nullptr;
  CK(hipMalloc(&col, n * 8));
  CK(hipMemset(col, 0, n * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tea::g_symeig_col), &col, sizeof(col)));
  unsigned long long* ttr = nullptr;
  CK(hipMalloc(&ttr, 16 * 8 * 8));
  CK(hipMemset(ttr, 0, 16 * 8 * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tea::g_symeig_tailtr), &ttr, sizeof(ttr)));
  double* tailbuf = nullptr;  // the one-workgroup tail's trailing block (TORCHEVAL_AMD_SYMEIG_TAIL)
  CK(hipMalloc(&tailbuf, tea::symeig_tail_bytes()));
  a.a = dA; a.d = dd; a.e = de; a.lam = dl; a.slots = gran; a.ctl = ctl; a.grid = grid; a.tail = tailbuf;
  for (int it = 0; it < 3; ++it) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    int rc = tea::launch_symeig(a, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned abort_word = 0;
    CK(hipMemcpy(&abort_word, ctl + 1, 4, hipMemcpyDeviceToHost));
    std::printf("run %d rc=%d abort=%u total %.3f ms\n", it, rc, abort_word, ms);
  }
  std::vector<unsigned long long> tr(2 * 16 * 8);
  CK(hipMemcpy(tr.data(), trace, tr.size() * 8, hipMemcpyDeviceToHost));
  const char* names[] = {"wait", "R1", "house", "pass", "R3", "publish"};
  for (int b = 0; b < 2; ++b) {
    std::printf("workgroup %d (cycles): wait R1 house(update + reflector) pass R3(row publish + reduction) publish | phase total\n",
                b ? 100 : 0);
    for (int j = 1; j < 16; ++j) {
      const unsigned long long* t = &tr[b * 128 + j * 8];
      const unsigned long long* p = &tr[b * 128 + (j - 1) * 8];
      std::printf("  j=%d: %llu %llu %llu(%llu + %llu) %llu %llu(%llu + %llu) %llu | %llu\n", 1000 + j, t[0] - p[5],
                  t[1] - t[0], t[2] - t[1], t[6] - t[1], t[2] - t[6], t[3] - t[2], t[4] - t[3], t[7] - t[3],
                  t[4] - t[7], t[5] - t[4], t[5] - p[5]);
    }
  }
  (void)names;
  // workgroup 0's column starts (100 MHz wall clock): mean us per column in blocks of 128
  std::vector<unsigned long long> cs(n);
  CK(hipMemcpy(cs.data(), col, n * 8, hipMemcpyDeviceToHost));
  std::printf("us per column, workgroup 0, blocks of 128 columns:\n");
  for (int b = 0; b + 128 <= n - 3; b += 128)
    std::printf("  columns %4d-%4d: %.2f\n", b, b + 127, (double)(cs[b + 128] - cs[b]) / 100.0 / 128.0);
  std::printf("  columns %4d-%4d: %.2f (total to last column %.3f ms)\n", (n - 3) / 128 * 128, n - 3,
              (double)(cs[n - 3] - cs[(n - 3) / 128 * 128]) / 100.0 / ((n - 3) % 128 ? (n - 3) % 128 : 1),
              (double)(cs[n - 3] - cs[0]) / 1e5);
  std::vector<unsigned long long> tt(16 * 8);
  CK(hipMemcpy(tt.data(), ttr, tt.size() * 8, hipMemcpyDeviceToHost));
  std::printf("tail kernel (cycles), columns 1-14: top->sigma, ->reflector, ->matvec+reduce, barrier, ->update | column\n");
  for (int j = 1; j < 15; ++j) {
    const unsigned long long* q = &tt[j * 8];
    std::printf("  j=%d: %llu %llu %llu %llu %llu | %llu\n", j, q[1] - q[0], q[2] - q[1], q[3] - q[2], q[4] - q[3],
                q[5] - q[4], tt[(j + 1) * 8] - q[0]);
  }
  return 0;
}
