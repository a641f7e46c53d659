// K3a splitter-bucket mode per-phase timeline (radix.hip built with TEA_RADIX_TRACE): 1M uniform
// scores + int64 targets; the sample kernel's phases (start, sample loaded, sample sorted) and, per
// bucket block, start -> offset known -> keys in LDS -> key spread -> LDS sort -> stores issued.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -Icsrc/include csrc/bench/k3_bucket_trace.hip -o csrc/bench/k3_bucket_trace.bin
#define TEA_RADIX_TRACE 1
#include "../kernels/radix.hip"

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

int main() {
  setenv("TORCHEVAL_AMD_K3_BUCKET", "1", 1);  // the opt-in mode
  const int64_t n = 1000000, rows = 1;
  std::vector<float> hx(n);
  std::vector<int64_t> ht(n);
  unsigned long long st = 987654321ull;
  for (int64_t i = 0; i < n; ++i) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    hx[i] = static_cast<float>((st >> 40) & 0xffffff) / 16777216.0f;
    ht[i] = (st >> 20) & 1;
  }
  tea::RadixArgs a;
  a.rows = rows;
  a.n = n;
  a.tiles = tea::radix_sort_tiles(rows, n);
  a.ngroups = tea::radix_sort_groups(a.tiles);
  if (!tea::radix_onesweep_ok(rows, n) || a.tiles > 4096) {
    std::printf("shape outside the onesweep tiling\n");
    return 1;
  }
  float *dx, *sorted;
  int64_t* dt;
  int32_t* order;
  uint32_t *ws, *groups, *hdr, *status;
  unsigned long long *gacc, *trace;
  const int64_t sw = tea::radix_onesweep_status_words(rows, n), gw = tea::radix_onesweep_group_words(rows, n);
  const int64_t region = rows * a.ngroups * 256;
  CK(hipMalloc(&dx, n * 4));
  CK(hipMalloc(&dt, n * 8));
  CK(hipMalloc(&sorted, n * 4));
  CK(hipMalloc(&order, n * 4));
  CK(hipMalloc(&ws, (4 * n + rows * 256 * a.tiles + rows * 512) * 4));
  CK(hipMalloc(&groups, (4 + 4 * region) * 4));
  CK(hipMalloc(&hdr, (16 + rows * 8 * 4 * 256) * 4));
  CK(hipMalloc(&status, 2 * sw * 4));
  CK(hipMalloc(&gacc, 2 * gw * 8));
  CK(hipMalloc(&trace, 16 * 4096 * 8 * 8));
  CK(hipMemset(groups, 0, (4 + 4 * region) * 4));
  CK(hipMemset(hdr, 0, (16 + rows * 8 * 4 * 256) * 4));
  CK(hipMemset(status, 0, 2 * sw * 4));
  CK(hipMemset(gacc, 0, 2 * gw * 8));
  CK(hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), n * 8, hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(tea::g_radix_trace), &trace, sizeof(trace)));
  a.in = dx;
  a.in_row_stride = n;
  a.keys0 = ws;
  a.vals0 = ws + n;
  a.keys1 = ws + 2 * n;
  a.vals1 = ws + 3 * n;
  a.hist = ws + 4 * n;
  a.dirty = groups;
  a.groups = groups + 4;
  a.region = region;
  a.out_sorted = sorted;
  a.out_order = order;
  a.payload_kind = 1;
  a.payload = dt;
  a.payload_dt = tea::DType::i64;
  a.payload_row_stride = 0;
  a.os_hdr = hdr;
  a.os_g = hdr + 16;
  a.os_status = status;
  a.os_splane = sw;
  a.os_gacc = gacc;
  a.os_gplane = gw;
  a.bkt_spl = ws + 4 * n + rows * 256 * a.tiles;
  a.bkt_cnt = a.bkt_spl + rows * 256;
  for (int it = 0; it < 6; ++it) {
    if (it == 5) CK(hipMemset(trace, 0, 16 * 4096 * 8 * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    const int rc = tea::launch_radix_sort_desc(a, 0);
    CK(hipEventRecord(e1, 0));
    CK(hipDeviceSynchronize());
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::printf("run %d rc=%d sort %.1f us\n", it, rc, ms * 1e3);
  }
  uint32_t timeout_flag = 0;
  CK(hipMemcpy(&timeout_flag, hdr + 8, 4, hipMemcpyDeviceToHost));
  std::vector<float> hs(n);
  CK(hipMemcpy(hs.data(), sorted, n * 4, hipMemcpyDeviceToHost));
  bool desc = true;
  for (int64_t i = 1; i < n; ++i) desc = desc && !(hs[i] > hs[i - 1]);
  std::printf("descending %s, look-back timeout flag %u\n", desc ? "yes" : "NO", timeout_flag);
  std::vector<unsigned long long> tr(16 * 4096 * 8);
  CK(hipMemcpy(tr.data(), trace, tr.size() * 8, hipMemcpyDeviceToHost));
  const unsigned long long* sp = &tr[(6 * 4096) * 8];
  std::printf("sample kernel: load %.2f us, spread + LDS radix %.2f us\n", (sp[1] - sp[0]) * 0.01, (sp[2] - sp[1]) * 0.01);
  std::vector<double> d[5];
  std::vector<int> nbits;
  unsigned long long t0 = ~0ull, t1 = 0;
  for (int b = 0; b < 256; ++b) {
    const unsigned long long* t = &tr[(5 * 4096 + b) * 8];
    if (t[0]) t0 = std::min(t0, t[0]);
    if (t[5]) t1 = std::max(t1, t[5]);
    for (int i = 0; i < 5; ++i)
      if (t[i] && t[i + 1]) d[i].push_back((t[i + 1] - t[i]) * 0.01);
    nbits.push_back(static_cast<int>(tr[(7 * 4096 + b) * 8]));
  }
  const char* names[] = {"start->offset", "offset->in_lds", "in_lds->spread", "spread->sorted", "sorted->stored"};
  std::printf("bucket kernel: first start to last store %.2f us; per-block median / max:\n", (t1 - t0) * 0.01);
  for (int i = 0; i < 5; ++i) {
    std::sort(d[i].begin(), d[i].end());
    if (!d[i].empty()) std::printf("  %-16s %7.2f %7.2f\n", names[i], d[i][d[i].size() / 2], d[i].back());
  }
  std::sort(nbits.begin(), nbits.end());
  std::printf("key bits sorted per bucket: median %d max %d\n", nbits[128], nbits.back());
  std::vector<double> q[3];
  for (int b = 0; b < 4096; ++b) {  // first LSD pass of the blocks (bucket blocks < 256, the sample block 0 too)
    const unsigned long long* t = &tr[(8 * 4096 + b) * 8];
    for (int i = 0; i < 3; ++i)
      if (t[i] && t[i + 1]) q[i].push_back((t[i + 1] - t[i]) * 0.01);
  }
  const char* qn[] = {"zero->ranked", "ranked->bases", "bases->scattered"};
  for (int i = 0; i < 3; ++i) {
    std::sort(q[i].begin(), q[i].end());
    if (!q[i].empty()) std::printf("  first LSD pass %-18s median %.2f max %.2f us\n", qn[i], q[i][q[i].size() / 2], q[i].back());
  }
  return desc && timeout_flag == 0 ? 0 : 1;
}
