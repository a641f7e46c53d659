// K4: binned threshold histograms -> TP / FP / FN per (threshold, class).
//
// Replaces
//   binned_precision_recall_curve.py:84-110  searchsorted -> 2*idx+target -> histc -> suffix cumsum
//   binned_precision_recall_curve.py:214-236, 406-431  "vectorized": a [T, N, C] bool tensor
//   binned_precision_recall_curve.py:239-291, 434-486  "memory": histc over 2*T*C bins
//   binned_auroc.py:111-215  [T, tasks, N] bool tensor
// with two launches and O(T*C) memory:
//   1 hist   : every (sample, class) element finds its bin over the sorted thresholds held in
//              LDS (bin = #thresholds <= x, exactly searchsorted(right=True)): a uniform-grid
//              guess verified by two LDS reads, binary search only when the guess is wrong;
//              v3 issues kUnroll elements' loads per thread before any bin work
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
#include <algorithm>

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

// bin = #thresholds <= x.  Guess from the uniform grid (linspace(0, 1, T), the int-threshold
// case) and verify with two LDS reads; only a wrong guess (arbitrary thresholds, NaN) pays for
// the binary search.  v2 always searched: ~8 dependent LDS round trips per element.
__device__ __forceinline__ int find_bin(const float* thr, int T, float x) {
  if (x != x) return T;  // NaN sorts above every threshold, as in torch.searchsorted
  const float gf = x * static_cast<float>(T - 1);
  const int g = gf >= 0.f ? (gf < static_cast<float>(T - 1) ? static_cast<int>(gf) + 1 : T) : 0;
  const bool lo_ok = g == 0 || thr[g - 1] <= x;
  const bool hi_ok = g == T || thr[g] > x;
  if (lo_ok && hi_ok) return g;
  return upper_bound_lds(thr, T, x);
}

// typed loads: f32 scores / int64 targets are the common case and get straight-line loads;
// everything else goes through the dtype switch (a uniform branch per element)
template <bool F32>
__device__ __forceinline__ float ld_x(const BinnedArgs& a, int64_t off) {
  if constexpr (F32) return static_cast<const float*>(a.input)[off];
  return load_as_f32(a.input, a.in_dt, off);
}

template <bool I64>
__device__ __forceinline__ bool ld_pos(const BinnedArgs& a, int64_t i, int64_t j) {
  if (a.mode == 1) {
    const int64_t lab = I64 ? static_cast<const int64_t*>(a.target)[i * a.tg_row_stride]
                            : load_as_i64(a.target, a.tg_dt, i * a.tg_row_stride);
    return lab == j;
  }
  const int64_t off = i * a.tg_row_stride + j * a.tg_col_stride;
  if constexpr (I64) return static_cast<const int64_t*>(a.target)[off] == 1;
  return load_as_f32(a.target, a.tg_dt, off) == 1.f;
}

constexpr int kUnroll = 8;  // elements per thread per round, all loads issued before any bin

template <bool XF32, bool YI64>
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
  const bool small = total <= 0xffffffffll;  // 32-bit index split (no 64-bit division)
  const int64_t step = static_cast<int64_t>(gridDim.x) * kB * kUnroll;
  for (int64_t base = static_cast<int64_t>(blockIdx.x) * kB * kUnroll + threadIdx.x; base < total;
       base += step) {
    float x[kUnroll];
    bool pos[kUnroll];
    int jj[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int64_t e = base + u * kB;
      int64_t i = 0;
      int c = 0;
      if (ncls == 1) {
        i = e;
      } else if (small) {
        const uint32_t e32 = static_cast<uint32_t>(e);
        if (class_fast) {
          const uint32_t q = e32 / static_cast<uint32_t>(ncls);
          i = q;
          c = static_cast<int>(e32 - q * static_cast<uint32_t>(ncls));
        } else {
          const uint32_t q = e32 / static_cast<uint32_t>(a.n);
          c = static_cast<int>(q);
          i = e32 - q * static_cast<uint32_t>(a.n);
        }
      } else if (class_fast) {
        i = e / ncls;
        c = static_cast<int>(e - i * ncls);
      } else {
        c = static_cast<int>(e / a.n);
        i = e - static_cast<int64_t>(c) * a.n;
      }
      jj[u] = e < total ? c : -1;
      if (e < total) {
        x[u] = ld_x<XF32>(a, i * a.in_row_stride + (c0 + c) * a.in_col_stride);
        pos[u] = ld_pos<YI64>(a, i, c0 + c);
      }
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      if (jj[u] >= 0) {
        const int bin = find_bin(s_thr, a.T, x[u]);  // 0 .. T
        atomicAdd(&s_hist[(bin * ncls + jj[u]) * 2 + (pos[u] ? 1 : 0)], 1u);
      }
    }
  }
  __syncthreads();
  unsigned* rep = a.ws + static_cast<int64_t>(blockIdx.x % kReplicas) * (a.T + 1) * a.c * 2;
  for (int k = threadIdx.x; k < hsize; k += kB) {
    const unsigned v = s_hist[k];
    if (v) {
      const int bin = k / (ncls * 2);
      const int rem = k - bin * ncls * 2;
      const int c = rem >> 1;
      const int p = rem & 1;
      atomicAdd(&rep[(static_cast<int64_t>(bin) * a.c + c0 + c) * 2 + p], v);
    }
  }
}

// ---- dense path (v4): the whole [T+1][C] histogram of one block fits in LDS as packed
// u32 counters (negatives in the low 16 bits, positives in the high 16 bits; a block never
// sees more than 65535 elements, so neither half can carry).  Blocks FLUSH WITH PLAIN
// COALESCED STORES into their own slab row, and a reduce kernel folds the slab with a few
// coalesced atomics.  The v2/v3 path flushed every non-zero bin with a global atomic: with
// [101 x 100] bins and ~20k elements per block that was ~one atomic per element (80-112 us
// for 100k x 100 classes).
constexpr int kDB = 1024;
constexpr int kDenseMaxWords = 16384;  // 64 KB of LDS
constexpr int kDenseMaxBlocks = 512;
constexpr int64_t kDenseBlockElems = 65535;
constexpr int kReduceRows = 16;
constexpr int kDU = 16;  // dense path: elements per thread per round (16 loads in flight)

template <bool YI64, int MODE>
__device__ __forceinline__ bool ld_pos_at(const BinnedArgs& a, int64_t off, uint32_t c) {
  if constexpr (MODE == 1) {
    const int64_t lab = YI64 ? static_cast<const int64_t*>(a.target)[off] : load_as_i64(a.target, a.tg_dt, off);
    return lab == static_cast<int64_t>(c);
  } else if constexpr (YI64) {
    return static_cast<const int64_t*>(a.target)[off] == 1;
  } else {
    return load_as_f32(a.target, a.tg_dt, off) == 1.f;
  }
}

// Dense-path kernel flavours.  FAST: f32 scores, int64 targets, every byte offset of the slab
// below 2^30 - the walker then keeps 32-bit BYTE offsets, so each load is a saddr + 32-bit
// voffset global load with no per-element 64-bit address math.  UNIFORM: the thresholds are
// the cached linspace(0, 1, T) (an int ``threshold``); the bin is then floor(x * (T - 1)) + 1
// whenever x * (T - 1) is not within ``margin`` of an integer (bounded by the fp32 error of
// linspace and of the product), with no LDS reads; only near-boundary elements verify.
template <bool FAST>
struct DenseTypes {
  using Off = int64_t;
};
template <>
struct DenseTypes<true> {
  using Off = uint32_t;
};

template <bool XF32, bool YI64, int MODE, bool FAST>
__device__ __forceinline__ void dense_load(const BinnedArgs& a, typename DenseTypes<FAST>::Off ox,
                                           typename DenseTypes<FAST>::Off ot, uint32_t c, float& x, bool& pos) {
  if constexpr (FAST) {
    x = *reinterpret_cast<const float*>(static_cast<const char*>(a.input) + ox);
    const int64_t v = *reinterpret_cast<const int64_t*>(static_cast<const char*>(a.target) + ot);
    pos = MODE == 1 ? v == static_cast<int64_t>(c) : v == 1;
  } else {
    x = ld_x<XF32>(a, ox);
    pos = ld_pos_at<YI64, MODE>(a, ot, c);
  }
}

template <bool UNIFORM>
__device__ __forceinline__ int dense_bin(const float* thr, int T, float x, float tm1, float margin, bool& ok) {
  if constexpr (UNIFORM) {
    const float gf = x * tm1;
    const float fl = floorf(gf);
    const float fr = gf - fl;
    int g = static_cast<int>(fl) + 1;
    ok = gf >= 0.f && gf < tm1 && fr > margin && fr < 1.f - margin;
    if (x >= 1.f) {  // thr[T-1] == 1 exactly
      g = T;
      ok = true;
    } else if (x < 0.f) {  // thr[0] == 0 exactly
      g = 0;
      ok = true;
    }
    return g;
  } else {
    const float gf = x * tm1;
    const int g = gf >= 0.f ? (gf < tm1 ? static_cast<int>(gf) + 1 : T) : 0;
    const float below = thr[max(g - 1, 0)];
    const float above = thr[min(g, T - 1)];
    ok = (g == 0 || below <= x) & (g == T || above > x);
    return g;
  }
}

// Element walker: e = major * M + minor with incremental offsets (one division per thread).
template <typename OffT>
struct DenseWalk {
  uint32_t mn, maj;
  OffT ox, ot;
};

template <typename OffT>
struct DenseStep {
  uint32_t M, dmin, dmaj;
  OffT sx, st, wx, wt;
};

// One round of kDU elements per thread: all loads first, then bins (wrong / unsafe guesses -
// arbitrary thresholds, near-boundary values, NaN - in one wave-uniform slow path), then the
// LDS atomics.
template <bool XF32, bool YI64, int MODE, bool FAST, bool UNIFORM, bool TAIL>
__device__ __forceinline__ void dense_round(const BinnedArgs& a, DenseWalk<typename DenseTypes<FAST>::Off>& w,
                                            const DenseStep<typename DenseTypes<FAST>::Off>& sp, uint32_t left,
                                            bool cf, float tm1, float margin, const float* s_thr,
                                            unsigned* s_hist, int C, uint32_t c0) {
  float x[kDU];
  bool pos[kDU];
  int cc[kDU];
#pragma unroll
  for (int u = 0; u < kDU; ++u) {
    const uint32_t c = cf ? w.mn : w.maj;
    cc[u] = static_cast<int>(c);
    if (!TAIL || static_cast<uint32_t>(u) < left) dense_load<XF32, YI64, MODE, FAST>(a, w.ox, w.ot, c0 + c, x[u], pos[u]);
    w.mn += sp.dmin;
    w.maj += sp.dmaj;
    w.ox += sp.sx;
    w.ot += sp.st;
    if (w.mn >= sp.M) {
      w.mn -= sp.M;
      w.maj += 1;
      w.ox += sp.wx;
      w.ot += sp.wt;
    }
  }
  int bin[kDU];
  uint32_t bad = 0;
#pragma unroll
  for (int u = 0; u < kDU; ++u) {
    bool ok = true;
    bin[u] = (!TAIL || static_cast<uint32_t>(u) < left) ? dense_bin<UNIFORM>(s_thr, a.T, x[u], tm1, margin, ok) : 0;
    bad |= ok ? 0u : (1u << u);
  }
  if (__builtin_expect(__any(bad != 0), 0)) {
#pragma unroll
    for (int u = 0; u < kDU; ++u)
      if (bad & (1u << u)) bin[u] = find_bin(s_thr, a.T, x[u]);
  }
#pragma unroll
  for (int u = 0; u < kDU; ++u)
    if (!TAIL || static_cast<uint32_t>(u) < left) atomicAdd(&s_hist[bin[u] * C + cc[u]], pos[u] ? 0x10000u : 1u);
}

// v4 dense histogram.  Each thread walks e = lo + tid + k * kDB; full rounds carry no bounds
// checks.  History at 100k x 100 classes, T=100 (MI355X): v4a per-element 64-bit div/mul and
// branches 34 us (VALU-bound, ~68 VALU per element); incremental walker + templated mode 21.5 us.
template <bool XF32, bool YI64, int MODE, bool FAST, bool UNIFORM>
__global__ __launch_bounds__(kDB) void binned_hist_dense_kernel(BinnedArgs a, unsigned* slab, int cb) {
  // grid.y walks class chunks of cb classes: chunk y owns classes [c0, c0 + C) and its own
  // [T+1][C] LDS histogram (v4 required the whole [T+1][classes] histogram in one block: more
  // than 16k bins fell back to the sparse atomic-flush path, 0.6 TB/s at 1000 classes)
  using OffT = typename DenseTypes<FAST>::Off;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* s_thr = reinterpret_cast<float*>(smem);
  const int thr_bytes = ((a.T * 4 + 15) / 16) * 16;
  unsigned* s_hist = reinterpret_cast<unsigned*>(smem + thr_bytes);
  const uint32_t c0 = blockIdx.y * static_cast<uint32_t>(cb);
  const int C = static_cast<int>(min(static_cast<int64_t>(cb), a.c - c0));
  const int W = (a.T + 1) * C;
  for (int k = threadIdx.x; k < a.T; k += kDB) s_thr[k] = a.thr[k];
  for (int k = threadIdx.x; k < W; k += kDB) s_hist[k] = 0u;
  __syncthreads();
  const uint32_t total = static_cast<uint32_t>(a.n * C);  // host slabs keep this < 2^26
  // element e = major * M + minor; (row, class) = cf ? (major, minor) : (minor, major)
  const bool cf = a.in_col_stride == 1 || C == 1;
  constexpr bool lab = MODE == 1;
  const int64_t xu = FAST ? 4 : 1, tu = FAST ? 8 : 1;  // offset units (bytes when FAST)
  const int64_t xs_min = (cf ? a.in_col_stride : a.in_row_stride) * xu;
  const int64_t xs_maj = (cf ? a.in_row_stride : a.in_col_stride) * xu;
  const int64_t ts_min = (lab ? (cf ? 0 : a.tg_row_stride) : (cf ? a.tg_col_stride : a.tg_row_stride)) * tu;
  const int64_t ts_maj = (lab ? (cf ? a.tg_row_stride : 0) : (cf ? a.tg_row_stride : a.tg_col_stride)) * tu;
  DenseStep<OffT> sp;
  sp.M = cf ? static_cast<uint32_t>(C) : static_cast<uint32_t>(a.n);
  sp.dmaj = kDB / sp.M;
  sp.dmin = kDB - sp.dmaj * sp.M;
  sp.sx = static_cast<OffT>(sp.dmaj * xs_maj + sp.dmin * xs_min);
  sp.st = static_cast<OffT>(sp.dmaj * ts_maj + sp.dmin * ts_min);
  sp.wx = static_cast<OffT>(xs_maj - static_cast<int64_t>(sp.M) * xs_min);
  sp.wt = static_cast<OffT>(ts_maj - static_cast<int64_t>(sp.M) * ts_min);
  // a contiguous element range per block (<= kDenseBlockElems, so the 16-bit halves are safe)
  const uint32_t per = (total + gridDim.x - 1) / gridDim.x;
  const uint32_t lo = blockIdx.x * per;
  const uint32_t hi = min(total, lo + per);
  const uint32_t e0 = lo + threadIdx.x;
  DenseWalk<OffT> w;
  w.maj = e0 / sp.M;
  w.mn = e0 - w.maj * sp.M;
  // offsets relative to the chunk's first class column
  const int64_t xc0 = static_cast<int64_t>(c0) * a.in_col_stride * xu;
  const int64_t tc0 = lab ? 0 : static_cast<int64_t>(c0) * a.tg_col_stride * tu;
  w.ox = static_cast<OffT>(xc0 + w.maj * xs_maj + w.mn * xs_min);
  w.ot = static_cast<OffT>(tc0 + w.maj * ts_maj + w.mn * ts_min);
  const float tm1 = static_cast<float>(a.T - 1);
  const float margin = 4e-7f * static_cast<float>(a.T) + 1e-6f;
  const uint32_t cnt = e0 < hi ? (hi - e0 + kDB - 1) / kDB : 0;
  uint32_t done = 0;
  for (; done + kDU <= cnt; done += kDU)
    dense_round<XF32, YI64, MODE, FAST, UNIFORM, false>(a, w, sp, kDU, cf, tm1, margin, s_thr, s_hist, C, c0);
  if (done < cnt)
    dense_round<XF32, YI64, MODE, FAST, UNIFORM, true>(a, w, sp, cnt - done, cf, tm1, margin, s_thr, s_hist, C, c0);
  __syncthreads();
  const int64_t wc = static_cast<int64_t>(a.T + 1) * cb;  // slab row stride
  unsigned* row = slab + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * wc;
  for (int k = threadIdx.x; k < W; k += kDB) row[k] = s_hist[k];
}

// slab [chunk][G][(T+1) x cb] packed -> acc[((bin * classes) + c0 + c) * 2 + {0: neg, 1: pos}]
// (u32, zero on entry; the suffix kernel consumes and re-zeroes it as replica 0)
__global__ __launch_bounds__(256) void binned_dense_reduce_kernel(const unsigned* slab, int G, int T, int64_t classes,
                                                                  int cb, unsigned* acc) {
  const int c0 = blockIdx.z * cb;
  const int C = static_cast<int>(min(static_cast<int64_t>(cb), classes - c0));
  const int W = (T + 1) * C;
  const int w = blockIdx.x * 256 + threadIdx.x;
  if (w >= W) return;
  const int64_t wc = static_cast<int64_t>(T + 1) * cb;
  const unsigned* base = slab + static_cast<int64_t>(blockIdx.z) * G * wc;
  const int g0 = blockIdx.y * kReduceRows;
  unsigned v[kReduceRows];
#pragma unroll
  for (int r = 0; r < kReduceRows; ++r)
    v[r] = g0 + r < G ? base[static_cast<int64_t>(g0 + r) * wc + w] : 0u;
  unsigned neg = 0, pos = 0;
#pragma unroll
  for (int r = 0; r < kReduceRows; ++r) {
    neg += v[r] & 0xffffu;
    pos += v[r] >> 16;
  }
  const int b = w / C, c = w - b * C;
  const int64_t o = (static_cast<int64_t>(b) * classes + c0 + c) * 2;
  if (neg) atomicAdd(&acc[o], neg);
  if (pos) atomicAdd(&acc[o + 1], pos);
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
    // all replica loads in flight before the sum (v2 alternated load / zero-store per
    // replica: one HBM round trip each), then the self-cleaning zero stores
    uint2 v[kReplicas];
    unsigned* cell0 = a.ws + (static_cast<int64_t>(b) * a.c + j) * 2;
#pragma unroll
    for (int r = 0; r < kReplicas; ++r)
      v[r] = r < replicas ? *reinterpret_cast<const uint2*>(cell0 + r * rstride) : make_uint2(0u, 0u);
    unsigned ng = 0, ps = 0;
#pragma unroll
    for (int r = 0; r < kReplicas; ++r) {
      ng += v[r].x;
      ps += v[r].y;
    }
#pragma unroll
    for (int r = 0; r < kReplicas; ++r)
      if (r < replicas) *reinterpret_cast<uint2*>(cell0 + r * rstride) = make_uint2(0u, 0u);
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

// binned PR curve points: precision = nan_to_num(tp / (tp + fp), nan=1), recall = tp / (tp +
// fn), each row closed with (1, 0) - the div / add / nan_to_num / cat / new_ones chain of the
// reference (binned_precision_recall_curve.py:113-131) as one elementwise launch, same fp32
// arithmetic so the values are bit-identical.
__global__ __launch_bounds__(kB) void binned_curve_kernel(BinnedFinalizeArgs a) {
  const int64_t idx = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x;
  const int64_t per = a.T + 1;
  if (idx >= a.rows * per) return;
  const int64_t r = idx / per;
  const int k = static_cast<int>(idx - r * per);
  float prec = 1.f, rec = 0.f;
  if (k < a.T) {
    const int64_t o = k * a.k_stride + r * a.r_stride;
    const float tp = a.tp[o], fp = a.fp[o], fn = a.fn[o];
    prec = tp / (tp + fp);
    if (prec != prec) prec = 1.f;
    rec = tp / (tp + fn);
  }
  a.out_prec[idx] = prec;
  a.out_rec[idx] = rec;
}

}  // namespace

int launch_binned_finalize(const BinnedFinalizeArgs& a, hipStream_t stream) {
  if (a.rows <= 0 || a.T <= 0) return 0;
  if (a.out_prec && a.out_rec) {
    const int64_t n = a.rows * (a.T + 1);
    hipLaunchKernelGGL(binned_curve_kernel, dim3(static_cast<unsigned>((n + kB - 1) / kB)), dim3(kB), 0, stream, a);
  }
  if (!a.out_auroc && !a.out_auprc) return static_cast<int>(hipGetLastError());
  hipLaunchKernelGGL(binned_finalize_kernel, dim3(static_cast<unsigned>(a.rows)), dim3(kB), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

namespace {
// classes per dense chunk: a [T+1][cb] histogram plus the thresholds in 64 KB of LDS
int dense_chunk(int T, int64_t c) {
  const int64_t thr_words = ((T * 4 + 15) / 16) * 4;
  const int64_t cb = (kDenseMaxWords - thr_words) / (T + 1);
  return static_cast<int>(cb < c ? cb : c);
}

bool dense_eligible(int T, int64_t c) {
  return (T + 1) * c >= 256 && dense_chunk(T, c) >= 1;
}
int dtype_bytes(DType d) {
  switch (d) {
    case DType::f64: case DType::i64: return 8;
    case DType::f32: case DType::i32: return 4;
    case DType::f16: case DType::bf16: case DType::i16: return 2;
    default: return 1;
  }
}
}  // namespace

int64_t binned_workspace_words(int T, int64_t c) { return static_cast<int64_t>(kReplicas) * (T + 1) * c * 2; }

int64_t binned_slab_words(int T, int64_t c) {
  if (!dense_eligible(T, c)) return 0;
  const int64_t cb = dense_chunk(T, c), chunks = (c + cb - 1) / cb;
  return std::max<int64_t>(kDenseMaxBlocks, chunks) * (T + 1) * cb;  // G * chunks <= this many rows
}

namespace {
template <bool XF32, bool YI64, int MODE, bool FAST, bool UNIFORM>
void dense_go(const BinnedArgs& s, dim3 grid, size_t smem, hipStream_t stream, unsigned* slab, int cb) {
  hipLaunchKernelGGL((binned_hist_dense_kernel<XF32, YI64, MODE, FAST, UNIFORM>), grid, dim3(kDB), smem, stream, s, slab, cb);
}

template <int MODE>
void launch_dense_mode(const BinnedArgs& s, dim3 grid, size_t smem, hipStream_t stream, unsigned* slab, bool xf32,
                       bool yi64, bool fast, int cb) {
  if (fast) {
    if (s.uniform) dense_go<true, true, MODE, true, true>(s, grid, smem, stream, slab, cb);
    else dense_go<true, true, MODE, true, false>(s, grid, smem, stream, slab, cb);
  } else if (xf32 && yi64) {
    dense_go<true, true, MODE, false, false>(s, grid, smem, stream, slab, cb);
  } else if (xf32) {
    dense_go<true, false, MODE, false, false>(s, grid, smem, stream, slab, cb);
  } else if (yi64) {
    dense_go<false, true, MODE, false, false>(s, grid, smem, stream, slab, cb);
  } else {
    dense_go<false, false, MODE, false, false>(s, grid, smem, stream, slab, cb);
  }
}

// largest element offset a [n, c] view with these strides can reach (strides >= 0 from torch)
int64_t max_offset(int64_t n, int64_t c, int64_t rs, int64_t cs) {
  return (n > 0 ? (n - 1) * std::abs(rs) : 0) + (c > 0 ? (c - 1) * std::abs(cs) : 0);
}

void launch_dense(const BinnedArgs& s, dim3 grid, size_t smem, hipStream_t stream, unsigned* slab, bool xf32,
                  bool yi64, int cb) {
  // byte offsets in 32 bits: the walker can step one kDB stride past the range before the
  // bound check stops it, so keep 2^30 of headroom
  const int64_t lim = (int64_t{1} << 30);
  const bool fast = xf32 && yi64 && 4 * max_offset(s.n, s.c, s.in_row_stride, s.in_col_stride) < lim &&
                    8 * max_offset(s.n, s.mode == 1 ? 1 : s.c, s.tg_row_stride, s.tg_col_stride) < lim;
  if (s.mode == 1) launch_dense_mode<1>(s, grid, smem, stream, slab, xf32, yi64, fast, cb);
  else launch_dense_mode<0>(s, grid, smem, stream, slab, xf32, yi64, fast, cb);
}
}  // namespace

int launch_binned(const BinnedArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.c <= 0 || a.T <= 0) return 0;
  if (dense_eligible(a.T, a.c)) {
    const int cb = dense_chunk(a.T, a.c);
    const int chunks = static_cast<int>((a.c + cb - 1) / cb);
    const int64_t wc = static_cast<int64_t>(a.T + 1) * cb;
    unsigned* acc = a.ws;    // [T+1][classes][2], replica 0 of the suffix kernel (zero contract)
    unsigned* slab = a.slab;  // [chunks][G][wc], fully overwritten per launch (separate scratch)
    if (slab == nullptr) return -2;
    const int thr_bytes = ((a.T * 4 + 15) / 16) * 16;
    const size_t smem = thr_bytes + static_cast<size_t>(wc) * 4;
    const bool xf32 = a.in_dt == DType::f32, yi64 = a.tg_dt == DType::i64;
    // <= kDenseMaxBlocks blocks over all chunks; row slabs keep every block <= 65535 elements
    const int64_t gmax = std::max<int64_t>(1, kDenseMaxBlocks / chunks);
    const int64_t rows_per = std::max<int64_t>(1, gmax * kDenseBlockElems / cb);
    for (int64_t r0 = 0; r0 < a.n; r0 += rows_per) {
      BinnedArgs s = a;
      s.n = std::min(rows_per, a.n - r0);
      s.input = static_cast<const char*>(a.input) + r0 * a.in_row_stride * dtype_bytes(a.in_dt);
      s.target = static_cast<const char*>(a.target) + r0 * a.tg_row_stride * dtype_bytes(a.tg_dt);
      const int64_t E = s.n * cb;  // elements of a full chunk
      // ~one round of kDU elements per thread, never more than 65535 per block, and a flush
      // (G * wc words written and read back) of at most ~half the input's own bytes
      int64_t lo = (E + kDenseBlockElems - 1) / kDenseBlockElems;
      int64_t hi = std::max<int64_t>(lo, std::min<int64_t>(gmax, E / (4 * wc)));
      int64_t G = std::min(std::max((E + kDB * kDU - 1) / (kDB * kDU), lo), hi);
      if (G < 1) G = 1;
      const dim3 grid(static_cast<unsigned>(G), static_cast<unsigned>(chunks));
      launch_dense(s, grid, smem, stream, slab, xf32, yi64, cb);
      const dim3 rgrid(static_cast<unsigned>((wc + 255) / 256), static_cast<unsigned>((G + kReduceRows - 1) / kReduceRows),
                       static_cast<unsigned>(chunks));
      hipLaunchKernelGGL(binned_dense_reduce_kernel, rgrid, dim3(256), 0, stream, slab, static_cast<int>(G), a.T, a.c,
                         cb, acc);
    }
    const size_t smem2 = static_cast<size_t>(a.T + 1) * 2 * sizeof(unsigned);
    hipLaunchKernelGGL(binned_suffix_kernel, dim3(static_cast<unsigned>(a.c)), dim3(kB), smem2, stream, a, 1);
    return static_cast<int>(hipGetLastError());
  }
  const int thr_bytes = ((a.T * 4 + 15) / 16) * 16;
  int cb = static_cast<int>((kLdsBytes - thr_bytes) / ((a.T + 1) * 2 * 4));
  if (cb < 1) return -1;  // too many thresholds for the LDS histogram
  if (cb > a.c) cb = static_cast<int>(a.c);
  const int chunks = static_cast<int>((a.c + cb - 1) / cb);
  // ~one round of kUnroll elements per thread, <= ~4 blocks per CU over all chunks
  const int64_t per_chunk = a.n * cb;
  int64_t want = (per_chunk + kB * kUnroll - 1) / (kB * kUnroll);
  const int64_t cap = 1024 / chunks + 1;
  int gx = static_cast<int>(want < cap ? want : cap);
  if (gx < 1) gx = 1;
  const size_t smem = thr_bytes + static_cast<size_t>((a.T + 1) * cb * 2 * 4);
  const bool xf32 = a.in_dt == DType::f32, yi64 = a.tg_dt == DType::i64;
  const dim3 grid(gx, chunks);
  if (xf32 && yi64) hipLaunchKernelGGL((binned_hist_kernel<true, true>), grid, dim3(kB), smem, stream, a, cb);
  else if (xf32) hipLaunchKernelGGL((binned_hist_kernel<true, false>), grid, dim3(kB), smem, stream, a, cb);
  else if (yi64) hipLaunchKernelGGL((binned_hist_kernel<false, true>), grid, dim3(kB), smem, stream, a, cb);
  else hipLaunchKernelGGL((binned_hist_kernel<false, false>), grid, dim3(kB), smem, stream, a, cb);
  const size_t smem2 = static_cast<size_t>(a.T + 1) * 2 * sizeof(unsigned);
  hipLaunchKernelGGL(binned_suffix_kernel, dim3(static_cast<unsigned>(a.c)), dim3(kB), smem2, stream, a,
                     gx < kReplicas ? gx : kReplicas);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
