// Times csrc/bench/k9b_variant_counter.hip (counter barrier; -DVARIANT_ACQ: plain loads after
// an acquire) on a dense symmetric D = 2048 matrix and checks d/e against the production K9b.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Icsrc/include [-DVARIANT_ACQ] csrc/bench/k9b_ab.hip -o ...
#include "k9b_variant_counter.hip"

#include <cmath>
#include <cstdio>
#include <vector>

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
  a.ld = (n + 15) / 16 * 16;
  double *dA, *dd, *de, *dl;
  unsigned long long* gran;
  unsigned* ctl;
  const size_t gbytes = (size_t)4 * (n - 2) * a.ld * 8;
  if (hipMalloc(&dA, (size_t)n * n * 8) || hipMalloc(&dd, a.ld * 8) || hipMalloc(&de, a.ld * 8) ||
      hipMalloc(&dl, n * 8) || hipMalloc(&gran, gbytes) || hipMalloc(&ctl, 2048))
    return 1;
  hipMemset(gran, 0, gbytes);
  hipMemcpy(dA, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice);
  a.a = dA; a.d = dd; a.e = de; a.lam = dl; a.slots = gran; a.ctl = ctl;
  for (int it = 0; it < 4; ++it) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, 0);
    const int rc = teav::launch_symeig(a, 0);
    hipEventRecord(e1, 0);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned abort_word = 0;
    hipMemcpy(&abort_word, ctl + 1, 4, hipMemcpyDeviceToHost);
    std::vector<double> lam(n);
    hipMemcpy(lam.data(), dl, n * 8, hipMemcpyDeviceToHost);
    double tr = 0;
    for (double x : lam) tr += x;
    double want = 0;
    for (int i = 0; i < n; ++i) want += h[(size_t)i * n + i];
    std::printf("%s run %d rc=%d abort=%u %.3f ms  sum(lambda)-trace = %.3e\n",
#ifdef VARIANT_ACQ
                "acquire+plain",
#else
                "agent-loads",
#endif
                it, rc, abort_word, ms, tr - want);
  }
  return 0;
}
