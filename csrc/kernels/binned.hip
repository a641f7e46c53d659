// K4: binned threshold histograms -> TP / FP / FN per (threshold, class).
//
// Replaces
//   binned_precision_recall_curve.py:84-110  searchsorted -> 2*idx+target -> histc -> suffix cumsum
//   binned_precision_recall_curve.py:214-236, 406-431  "vectorized": a [T, N, C] bool tensor
//   binned_precision_recall_curve.py:239-291, 434-486  "memory": histc over 2*T*C bins
//   binned_auroc.py:111-215  [T, tasks, N] bool tensor
// with two launches and O(T*C) memory:
//   1 hist   : every (sample, class) element finds its bin by binary search over the sorted
//              thresholds held in LDS (bin = #thresholds <= x, exactly searchsorted(right=True))
//              and increments an LDS-privatised [bin][class-chunk][pos/neg] histogram; blocks
//              flush non-zero bins with one float atomic each.  Classes are chunked across
//              grid.y so the private histogram fits in 48 KB of LDS.
//   2 suffix : one thread per class walks bins T..1 accumulating the suffix sums and adds
//              tp / fp / fn (fn = positives - tp) straight into the metric states.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kLdsBytes = 48 * 1024;

__device__ __forceinline__ int upper_bound_lds(const float* thr, int T, float x) {
  int lo = 0, hi = T;  // first index with thr > x
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (thr[mid] <= x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kB) void binned_hist_kernel(BinnedArgs a, int cb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s_thr = reinterpret_cast<float*>(smem);
  const int thr_bytes = ((a.T * 4 + 15) / 16) * 16;
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem + thr_bytes);
  const int c0 = blockIdx.y * cb;
  const int ncls = static_cast<int>(min(static_cast<int64_t>(cb), a.c - c0));
  const int hsize = (a.T + 1) * ncls * 2;
  for (int k = threadIdx.x; k < a.T; k += kB) s_thr[k] = a.thr[k];
  for (int k = threadIdx.x; k < hsize; k += kB) s_hist[k] = 0u;
  __syncthreads();

  const int64_t total = a.n * ncls;
  const bool class_fast = a.in_col_stride == 1;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x; e < total;
       e += static_cast<int64_t>(gridDim.x) * kB) {
    int64_t i;
    int jj;
    if (class_fast) {
      i = e / ncls;
      jj = static_cast<int>(e - i * ncls);
    } else {
      jj = static_cast<int>(e / a.n);
      i = e - static_cast<int64_t>(jj) * a.n;
    }
    const int64_t j = c0 + jj;
    const float x = load_as_f32(a.input, a.in_dt, i * a.in_row_stride + j * a.in_col_stride);
    bool pos;
    if (a.mode == 1) {
      pos = load_as_i64(a.target, a.tg_dt, i * a.tg_row_stride) == j;
    } else {
      pos = load_as_f32(a.target, a.tg_dt, i * a.tg_row_stride + j * a.tg_col_stride) == 1.f;
    }
    const int bin = upper_bound_lds(s_thr, a.T, x);  // 0 .. T
    atomicAdd(&s_hist[(bin * ncls + jj) * 2 + (pos ? 1 : 0)], 1u);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < hsize; k += kB) {
    const unsigned v = s_hist[k];
    if (v) {
      const int bin = k / (ncls * 2);
      const int rem = k - bin * ncls * 2;
      const int jj = rem >> 1;
      const int p = rem & 1;
      atomicAdd(&a.hist[(static_cast<int64_t>(bin) * a.c + c0 + jj) * 2 + p], static_cast<float>(v));
    }
  }
}

__global__ __launch_bounds__(kB) void binned_suffix_kernel(BinnedArgs a) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x;
  if (j >= a.c) return;
  double pos_total = 0.0;
  for (int b = 0; b <= a.T; ++b) pos_total += a.hist[(static_cast<int64_t>(b) * a.c + j) * 2 + 1];
  double tp = 0.0, fp = 0.0;
  for (int b = a.T; b >= 1; --b) {
    tp += a.hist[(static_cast<int64_t>(b) * a.c + j) * 2 + 1];
    fp += a.hist[(static_cast<int64_t>(b) * a.c + j) * 2 + 0];
    const int64_t o = static_cast<int64_t>(b - 1) * a.out_k_stride + j * a.out_c_stride;
    if (a.tp) a.tp[o] += static_cast<float>(tp);
    if (a.fp) a.fp[o] += static_cast<float>(fp);
    if (a.fn) a.fn[o] += static_cast<float>(pos_total - tp);
  }
}

}  // namespace

int launch_binned(const BinnedArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.c <= 0 || a.T <= 0) return 0;
  const int thr_bytes = ((a.T * 4 + 15) / 16) * 16;
  int cb = static_cast<int>((kLdsBytes - thr_bytes) / ((a.T + 1) * 2 * 4));
  if (cb < 1) return -1;  // too many thresholds for the LDS histogram
  if (cb > a.c) cb = static_cast<int>(a.c);
  const int chunks = static_cast<int>((a.c + cb - 1) / cb);
  const int64_t per_chunk = a.n * cb;
  int64_t want = (per_chunk + kB * 8 - 1) / (kB * 8);
  const int64_t cap = 1024 / chunks + 1;
  int gx = static_cast<int>(want < cap ? want : cap);
  if (gx < 1) gx = 1;
  const size_t smem = thr_bytes + static_cast<size_t>((a.T + 1) * cb * 2 * 4);
  hipLaunchKernelGGL(binned_hist_kernel, dim3(gx, chunks), dim3(kB), smem, stream, a, cb);
  hipLaunchKernelGGL(binned_suffix_kernel, dim3(static_cast<unsigned>((a.c + kB - 1) / kB)), dim3(kB),
                     0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
