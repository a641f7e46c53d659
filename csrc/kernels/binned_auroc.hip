// K4b: the reference-default multiclass binned AUROC, one value per SAMPLE
// (reference torcheval/metrics/functional/classification/binned_auroc.py:189-215).
//
// The reference builds a [T, N, C] boolean tensor (input >= threshold), sums the one-hot
// product over the CLASS dim, so each curve is one sample: tp_t = [x_true >= thr_t],
// fp_t = #{c != true : x_c >= thr_t}, a trapezoid over the descending-threshold points with a
// leading 0, divided by tp_0 * fp_0 (0.5 where that is 0).  With b(x) = #{t : thr_t <= x}
// (the bin; thresholds ascending) every trapezoid segment is one class whose bin is b, so the
// area collapses to a rank statistic of the sample's own scores:
//
//   area  = #{c != true : 1 <= b_c < b_true} + 0.5 #{c != true : b_c == b_true}
//   auroc = area / #{c != true : b_c >= 1}   if b_true >= 1 and that count > 0, else 0.5
//
// and the comparisons against bins reduce to comparisons against three thresholds of the
// sample (thr_0, thr[b_true - 1], thr[b_true]): b_c >= 1 <=> x_c >= thr_0, b_c < b_true <=>
// x_c < thr[b_true - 1], b_c == b_true <=> thr[b_true - 1] <= x_c < thr[b_true].  So one
// binary search per SAMPLE (of its true score, in LDS), no per-class search, no histogram,
// one streaming read of the scores.  NaN scores compare false (bin 0), as `>=` does there.
//
// Layout: G lanes per sample (G = the next power of two >= C / 4, at most 64), 16-B loads at
// 4-B alignment (tea_common.h load_f4u; any width, any row stride); U = 8 samples per lane
// group in flight; counts folded by xor shuffles inside the group.  Labels outside [0, C) set
// bit 0 of `err` (the caller raises the reference's one_hot error after one flag read).
#include <algorithm>

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kU = 8;
constexpr int kLdsT = 4096;  // thresholds staged in LDS (larger T: searched in global memory)

__device__ __forceinline__ int upper_bound_f32(const float* thr, int T, float x) {
  // #{t : thr_t <= x}: fixed-trip branchless search (NaN: 0)
  int b = 0;
  int step = 1;
  while (step <= T) step <<= 1;
  for (step >>= 1; step > 0; step >>= 1) {
    const int nb = b + step;
    b = (nb <= T && thr[nb - 1] <= x) ? nb : b;
  }
  return b;
}

// NARROW (c < 4): G = 4 lanes per sample, lane j reads column j (scalar, clamped)
template <int G, typename TGT, bool NARROW = false>
__global__ __launch_bounds__(kB) void sample_binned_auroc_kernel(SampleAurocArgs a) {
  __shared__ float s_thr[kLdsT];
  const int T = a.T;
  const bool in_lds = T <= kLdsT;
  if (in_lds)
    for (int i = threadIdx.x; i < T; i += kB) s_thr[i] = a.thr[i];
  __syncthreads();
  const float* thr = in_lds ? s_thr : a.thr;
  const float t0 = thr[0];
  const int C = static_cast<int>(a.c);
  const int gl = threadIdx.x & (G - 1);
  const int64_t ngroups = static_cast<int64_t>(gridDim.x) * (kB / G);
  const int64_t grp = static_cast<int64_t>(blockIdx.x) * (kB / G) + threadIdx.x / G;
  const TGT* tgt = static_cast<const TGT*>(a.target);

  for (int64_t s0 = grp; s0 < a.n; s0 += ngroups * kU) {
    int64_t row[kU];
    TGT tg[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t r = s0 + static_cast<int64_t>(u) * ngroups;
      row[u] = r < a.n ? r : s0;  // clamped: every load valid, results masked below
      tg[u] = tgt[row[u] * a.tg_stride];
    }
    // the first pass of every sample's row (4 G columns), issued before anything waits
    float4 q[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if constexpr (NARROW) {
        const float v = a.input[row[u] * a.row_stride + (gl < C ? gl : 0)];
        q[u] = make_float4(v, v, v, v);
      } else {
        const int col = 4 * gl;
        const int lc = col + 4 <= C ? col : (col < C ? C - 4 : 0);
        q[u] = load_f4u(a.input + row[u] * a.row_stride + lc);
      }
    }
    // true scores (L1 / L2 hits: the row is in flight), then each sample's three thresholds
    float xt[kU], lo[kU], hi[kU];
    int bt[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t t = static_cast<int64_t>(tg[u]);
      const bool ok = t >= 0 && t < C;
      xt[u] = a.input[row[u] * a.row_stride + (ok ? t : 0)];
      if (!ok && gl == 0 && s0 + static_cast<int64_t>(u) * ngroups < a.n) atomicOr(a.err, 1);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      bt[u] = upper_bound_f32(thr, T, xt[u]);
      lo[u] = bt[u] >= 1 ? thr[bt[u] - 1] : __builtin_inff();
      hi[u] = bt[u] < T ? thr[bt[u]] : __builtin_inff();
    }
    int less[kU], eq[kU], pos[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      less[u] = eq[u] = pos[u] = 0;
    }
    // count one pass (shifted tail lane: the first sh values repeat earlier columns)
    auto count = [&](int u, float4 v, int col) {
      const int sh = (col < C && col + 4 > C) ? col + 4 - C : 0;
      const float f[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool in = col < C && e >= sh;
        const float x = f[e];
        const bool p = in && x >= t0;
        pos[u] += p;
        less[u] += p && x < lo[u];
        eq[u] += in && x >= lo[u] && x < hi[u];
      }
    };
    if constexpr (NARROW) {
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const bool in = gl < C;
        const float x = q[u].x;
        const bool p = in && x >= t0;
        pos[u] += p;
        less[u] += p && x < lo[u];
        eq[u] += in && x >= lo[u] && x < hi[u];
      }
    } else {
#pragma unroll
      for (int u = 0; u < kU; ++u) count(u, q[u], 4 * gl);
    }
    for (int base = 4 * G; !NARROW && base < C; base += 4 * G) {  // rows wider than 4 G columns
      float4 r[kU];
      const int col = base + 4 * gl;
      const int lc = col + 4 <= C ? col : (col < C ? C - 4 : 0);
#pragma unroll
      for (int u = 0; u < kU; ++u) r[u] = load_f4u(a.input + row[u] * a.row_stride + lc);
#pragma unroll
      for (int u = 0; u < kU; ++u) count(u, r[u], col);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) {
        less[u] += __shfl_xor(less[u], o, kWave);
        eq[u] += __shfl_xor(eq[u], o, kWave);
        pos[u] += __shfl_xor(pos[u], o, kWave);
      }
      const int64_t s = s0 + static_cast<int64_t>(u) * ngroups;
      if (gl == 0 && s < a.n) {
        // the true class sits in eq and pos (x_true >= thr[b - 1] >= thr_0, < thr[b])
        const int e = eq[u] - 1, p = pos[u] - 1;
        const float area = static_cast<float>(less[u]) + 0.5f * static_cast<float>(e);
        a.out[s] = (bt[u] >= 1 && p > 0) ? area / static_cast<float>(p) : 0.5f;
      }
    }
  }
}

template <int G, bool NARROW = false>
void launch_g(const SampleAurocArgs& a, hipStream_t s) {
  const int64_t groups = (a.n + kU - 1) / kU;
  const int grid = stream_grid(groups, kB / G, 2048);
  if (a.tg_dt == DType::i32)
    hipLaunchKernelGGL((sample_binned_auroc_kernel<G, int32_t, NARROW>), dim3(grid), dim3(kB), 0, s, a);
  else
    hipLaunchKernelGGL((sample_binned_auroc_kernel<G, int64_t, NARROW>), dim3(grid), dim3(kB), 0, s, a);
}

}  // namespace

int launch_sample_binned_auroc(const SampleAurocArgs& a, hipStream_t stream) {
  if (a.n <= 0) return 0;
  if (a.c < 1 || a.T < 1 || (a.tg_dt != DType::i64 && a.tg_dt != DType::i32) || !a.err) return -1;
  const int64_t need = (a.c + 3) / 4;
  if (a.c < 4) launch_g<4, true>(a, stream);
  else if (need <= 4) launch_g<4>(a, stream);
  else if (need <= 8) launch_g<8>(a, stream);
  else if (need <= 16) launch_g<16>(a, stream);
  else if (need <= 32) launch_g<32>(a, stream);
  else launch_g<64>(a, stream);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
