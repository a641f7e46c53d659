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
//              flush non-zero bins with one u32 atomic each into one of kReplicas global
//              replicas (blockIdx % kReplicas: 16x less same-address contention than one
//              shared histogram - v1's single float histogram cost ~55 us at 1M samples).
//              Classes are chunked across grid.y so the private histogram fits in 48 KB.
//   2 suffix : one block per class sums the replicas per bin into LDS (and re-zeroes them:
//              the workspace is self-cleaning, no memset launch), then a block-parallel
//              suffix scan from the top bin writes tp / fp / fn (fn = positives - tp)
//              straight into the metric states (v1 walked the bins serially in one thread
//              per class: ~98 us for the binary case).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kLdsBytes = 48 * 1024;
constexpr int kReplicas = 16;

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
  unsigned* rep = a.ws + static_cast<int64_t>(blockIdx.x % kReplicas) * (a.T + 1) * a.c * 2;
  for (int k = threadIdx.x; k < hsize; k += kB) {
    const unsigned v = s_hist[k];
    if (v) {
      const int bin = k / (ncls * 2);
      const int rem = k - bin * ncls * 2;
      const int jj = rem >> 1;
      const int p = rem & 1;
      atomicAdd(&rep[(static_cast<int64_t>(bin) * a.c + c0 + jj) * 2 + p], v);
    }
  }
}

__device__ __forceinline__ unsigned long long wave_incl_sum_u64(unsigned long long v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// one block per class: replica sum per bin (self-cleaning) -> block-parallel suffix scan
__global__ __launch_bounds__(kB) void binned_suffix_kernel(BinnedArgs a, int replicas) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned* s_neg = reinterpret_cast<unsigned*>(smem);
  unsigned* s_pos = s_neg + (a.T + 1);
  __shared__ unsigned long long s_w[2][kB / 64];
  __shared__ unsigned long long s_total;
  const int64_t j = blockIdx.x;
  const int64_t rstride = static_cast<int64_t>(a.T + 1) * a.c * 2;
  unsigned long long pos_local = 0;
  for (int b = threadIdx.x; b <= a.T; b += kB) {
    unsigned ng = 0, ps = 0;
    for (int r = 0; r < replicas; ++r) {
      unsigned* cell = a.ws + r * rstride + (static_cast<int64_t>(b) * a.c + j) * 2;
      ng += cell[0];
      ps += cell[1];
      cell[0] = 0u;
      cell[1] = 0u;
    }
    s_neg[b] = ng;
    s_pos[b] = ps;
    pos_local += ps;
  }
  pos_local = wave_sum(pos_local);
  if (lane_id() == 0) s_w[0][threadIdx.x >> 6] = pos_local;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kB / 64; ++w) t += s_w[0][w];
    s_total = t;
  }
  __syncthreads();
  const double pos_total = static_cast<double>(s_total);
  // suffix sums over bins T..1, 256 bins per chunk, thread t -> bin (start - t)
  unsigned long long carry_tp = 0, carry_fp = 0;
  for (int start = a.T; start >= 1; start -= kB) {
    const int b = start - static_cast<int>(threadIdx.x);
    const unsigned long long p = b >= 1 ? s_pos[b] : 0ull;
    const unsigned long long f = b >= 1 ? s_neg[b] : 0ull;
    const unsigned long long ip = wave_incl_sum_u64(p);
    const unsigned long long ifp = wave_incl_sum_u64(f);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if (lane_id() == 63) {
      s_w[0][w] = ip;
      s_w[1][w] = ifp;
    }
    __syncthreads();
    unsigned long long op = carry_tp, of = carry_fp, tp_all = 0, fp_all = 0;
    for (int q = 0; q < kB / 64; ++q) {
      if (q < w) {
        op += s_w[0][q];
        of += s_w[1][q];
      }
      tp_all += s_w[0][q];
      fp_all += s_w[1][q];
    }
    if (b >= 1) {
      const double tp = static_cast<double>(op + ip), fp = static_cast<double>(of + ifp);
      const int64_t o = static_cast<int64_t>(b - 1) * a.out_k_stride + j * a.out_c_stride;
      if (a.tp) a.tp[o] += static_cast<float>(tp);
      if (a.fp) a.fp[o] += static_cast<float>(fp);
      if (a.fn) a.fn[o] += static_cast<float>(pos_total - tp);
    }
    carry_tp += tp_all;
    carry_fp += fp_all;
  }
}

// one block per row: AUROC (trapezoid over the binned ROC points) and AUPRC (Riemann sum over
// the binned PR points with the (precision 1, recall 0) end point) from [T, R] counts - the
// ~20 small ATen ops of the reference compute (binned_auroc.py:111-138,
// binned_auprc.py:86-112) in one launch.
__global__ __launch_bounds__(kB) void binned_finalize_kernel(BinnedFinalizeArgs a) {
  const int64_t r = blockIdx.x;
  const int T = a.T;
  auto at = [&](const float* p, int k) -> double { return static_cast<double>(p[k * a.k_stride + r * a.r_stride]); };
  double area = 0.0, riem = 0.0;
  bool riem_nan = false;
  for (int k = threadIdx.x; k < T; k += kB) {
    const double tp = at(a.tp, k), fp = at(a.fp, k);
    const double tpn = k + 1 < T ? at(a.tp, k + 1) : 0.0, fpn = k + 1 < T ? at(a.fp, k + 1) : 0.0;
    area += (fp - fpn) * (tp + tpn) * 0.5;
    if (a.out_auprc) {
      const double fn = at(a.fn, k);
      double prec = tp / (tp + fp);
      if (prec != prec) prec = 1.0;
      const double rec = tp / (tp + fn);
      double recn = 0.0;
      if (k + 1 < T) recn = at(a.tp, k + 1) / (at(a.tp, k + 1) + at(a.fn, k + 1));
      const double term = (recn - rec) * prec;
      if (term != term) riem_nan = true;
      else riem -= term;
    }
  }
  __shared__ double s[2][kB / 64];
  __shared__ int s_nan;
  if (threadIdx.x == 0) s_nan = 0;
  area = wave_sum(area);
  riem = wave_sum(riem);
  __syncthreads();
  if (riem_nan) s_nan = 1;
  if (lane_id() == 0) {
    s[0][threadIdx.x >> 6] = area;
    s[1][threadIdx.x >> 6] = riem;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ar = 0.0, rm = 0.0;
    for (int w = 0; w < kB / 64; ++w) {
      ar += s[0][w];
      rm += s[1][w];
    }
    if (a.out_auroc) {
      const double factor = at(a.tp, 0) * at(a.fp, 0);
      a.out_auroc[r] = factor == 0.0 ? 0.5 : ar / factor;
    }
    if (a.out_auprc) a.out_auprc[r] = s_nan ? 0.f : static_cast<float>(rm);
  }
}

}  // namespace

int launch_binned_finalize(const BinnedFinalizeArgs& a, hipStream_t stream) {
  if (a.rows <= 0 || a.T <= 0) return 0;
  hipLaunchKernelGGL(binned_finalize_kernel, dim3(static_cast<unsigned>(a.rows)), dim3(kB), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

int64_t binned_workspace_words(int T, int64_t c) { return static_cast<int64_t>(kReplicas) * (T + 1) * c * 2; }

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
  const size_t smem2 = static_cast<size_t>(a.T + 1) * 2 * sizeof(unsigned);
  hipLaunchKernelGGL(binned_suffix_kernel, dim3(static_cast<unsigned>(a.c)), dim3(kB), smem2, stream, a,
                     gx < kReplicas ? gx : kReplicas);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
