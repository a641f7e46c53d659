// K3b probe: runs launch_bucket_auc (csrc/kernels/bucketauc.hip built with BK_PROBE) on a
// uniform / normal row of n samples with int64 targets and prints, per kernel, the spread of
// block start / end times and the per-phase block durations from s_memrealtime stamps
// (100 MHz), plus event-timed whole calls.  Usage: k3b_probe.bin n [normal]
#define BK_PROBE 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../kernels/bucketauc.hip"

using namespace tea;

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

static double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, static_cast<size_t>(p * (v.size() - 1)))];
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 1000000;
  const bool normal = argc > 2;
  std::mt19937 rng(1);
  std::vector<float> hx(n);
  std::vector<int64_t> ht(n);
  std::uniform_real_distribution<float> U(0.f, 1.f);
  std::normal_distribution<float> Nd(0.f, 1.f);
  for (int64_t i = 0; i < n; ++i) {
    hx[i] = normal ? Nd(rng) : U(rng);
    ht[i] = rng() & 1;
  }
  BucketAucArgs a;
  a.n = n;
  a.B = bucket_auc_buckets(n);
  a.S = 4 * a.B;
  a.nbins = 2 * a.B + 2;
  a.t_dt = DType::i64;
  const int64_t tiles = bucket_auc_tiles(n);
  float* dx;
  int64_t* dt;
  CK(hipMalloc(&dx, n * 4));
  CK(hipMalloc(&dt, n * 8));
  CK(hipMemcpy(dx, hx.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, ht.data(), n * 8, hipMemcpyHostToDevice));
  a.x = dx;
  a.t = dt;
  char* z;
  CK(hipMalloc(&z, 4096 * 12 + 64));
  CK(hipMemset(z, 0, 4096 * 12 + 64));
  a.cursor = reinterpret_cast<uint32_t*>(z);
  a.posmass = reinterpret_cast<double*>(z + 4096 * 4);
  a.done = reinterpret_cast<unsigned*>(z + 4096 * 12);
  const int64_t stack_bytes = bucket_auc_stack_items(n) * 16;
  const int64_t bytes = stack_bytes + 5 * n * 4 + a.B * 4 + a.nbins * 16 + tiles * 12 + tiles * a.nbins * 4 + 256;
  char* ws;
  CK(hipMalloc(&ws, bytes));
  a.stack = ws;
  ws += stack_bytes;
  a.slots = reinterpret_cast<double*>(ws);
  ws += ((a.nbins * 16 + 15) / 16) * 16;
  a.keys_out = reinterpret_cast<uint32_t*>(ws);
  a.t_out = reinterpret_cast<float*>(a.keys_out + n);
  a.keys_tmp = reinterpret_cast<uint32_t*>(a.t_out + n);
  a.t_tmp = reinterpret_cast<float*>(a.keys_tmp + n);
  a.sp = reinterpret_cast<uint32_t*>(a.t_tmp + n);
  a.spc = a.sp + a.B;
  a.tileoff = a.spc + tiles * 3;
  a.binrank = a.tileoff + tiles * a.nbins;
  double* out;
  CK(hipMalloc(&out, 16));
  a.out_roc = out;
  a.out_pr = out + 1;
  unsigned long long* dbg;
  const size_t dbg_n = 4 * 4096 * 8;
  CK(hipMalloc(&dbg, dbg_n * 8));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_bk_dbg), &dbg, sizeof(dbg)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 20; ++w) CK(static_cast<hipError_t>(launch_bucket_auc(a, 0)));
  CK(hipDeviceSynchronize());
  const int iters = 200;
  CK(hipEventRecord(e0, 0));
  for (int w = 0; w < iters; ++w) launch_bucket_auc(a, 0);
  CK(hipEventRecord(e1, 0));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipMemset(dbg, 0, dbg_n * 8));
  CK(hipDeviceSynchronize());
  launch_bucket_auc(a, 0);
  CK(hipDeviceSynchronize());
  std::vector<unsigned long long> h(dbg_n);
  CK(hipMemcpy(h.data(), dbg, dbg_n * 8, hipMemcpyDeviceToHost));
  double ho[2];
  CK(hipMemcpy(ho, out, 16, hipMemcpyDeviceToHost));
  printf("n=%lld B=%d nbins=%d tiles=%lld %s: %.2f us/call (events, %d calls)  auroc=%.9f auprc=%.9f\n",
         static_cast<long long>(n), a.B, a.nbins, static_cast<long long>(tiles), normal ? "normal" : "uniform",
         ms * 1000.0 / iters, iters, ho[0], ho[1]);
  const char* names[4] = {"hist", "scatter", "local", "sample"};
  const int blocks[4] = {static_cast<int>(tiles), static_cast<int>(tiles), a.B, 1};  // local: per wave unit
  unsigned long long t_origin = ~0ull;
  for (int k = 0; k < 4; ++k)
    for (int b = 0; b < blocks[k]; ++b) t_origin = std::min(t_origin, h[(k * 4096 + b) * 8]);
  const int order[4] = {3, 0, 1, 2};
  for (int oi = 0; oi < 4; ++oi) {
    const int k = order[oi];
    unsigned long long s0 = ~0ull, s1 = 0, e1v = 0;
    std::vector<double> dur, ph[3];
    for (int b = 0; b < blocks[k]; ++b) {
      const unsigned long long* r = &h[(k * 4096 + b) * 8];
      s0 = std::min(s0, r[0]);
      s1 = std::max(s1, r[0]);
      e1v = std::max(e1v, r[3]);
      dur.push_back((r[3] - r[0]) * 0.01);
      for (int q = 0; q < 3; ++q)
        if (r[q + 1] && r[q]) ph[q].push_back((static_cast<double>(r[q + 1]) - static_cast<double>(r[q])) * 0.01);
    }
    {  // extra stamps 4..7: time from stamp 1 (p50 over blocks)
      for (int x = 4; x < 8; ++x) {
        std::vector<double> v;
        for (int b = 0; b < blocks[k]; ++b) {
          const unsigned long long* r = &h[(k * 4096 + b) * 8];
          if (r[x] && r[1]) v.push_back((static_cast<double>(r[x]) - static_cast<double>(r[1])) * 0.01);
        }
        if (!v.empty()) printf("   [%s stamp %d - stamp 1: p50 %.2f us]\n", names[k], x, pct(v, 0.5));
      }
    }
    printf("%-8s blocks=%5d first_start=%8.2f last_start=%8.2f last_end=%8.2f us | block us p50=%.2f p90=%.2f max=%.2f",
           names[k], blocks[k], (s0 - t_origin) * 0.01, (s1 - t_origin) * 0.01, (e1v - t_origin) * 0.01,
           pct(dur, 0.5), pct(dur, 0.9), pct(dur, 1.0));
    for (int q = 0; q < 3; ++q) printf(" | ph%d p50=%.2f max=%.2f", q, pct(ph[q], 0.5), pct(ph[q], 1.0));
    printf("\n");
  }
  // the slowest local blocks
  std::vector<std::pair<double, int>> sl;
  for (int b = 0; b < a.B; ++b) {
    const unsigned long long* r = &h[(2 * 4096 + b) * 8];
    sl.push_back({(r[3] - r[0]) * 0.01, b});
  }
  std::sort(sl.rbegin(), sl.rend());
  for (int i = 0; i < 6 && i < static_cast<int>(sl.size()); ++i) {
    const unsigned long long* r = &h[(2 * 4096 + sl[i].second) * 8];
    printf("  local block %5d: %.2f us (prefix %.2f, body %.2f, fold %.2f) start at %.2f\n", sl[i].second, sl[i].first,
           (r[1] - r[0]) * 0.01, (r[2] - r[1]) * 0.01, (r[3] - r[2]) * 0.01, (r[0] - t_origin) * 0.01);
  }
  return 0;
}
