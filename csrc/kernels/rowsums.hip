// K5b: per-row weighted sums merged straight into metric states.
//
// Replaces the eager chains of
//   functional/aggregation/sum.py / mean.py         (input * weight).sum() / torch.sum + numel
//   functional/image/psnr.py:68-85 + image/psnr.py   sum((x - t)^2), numel, target min / max,
//                                                    then three out-of-place state updates
//   functional/ranking/click_through_rate.py         (input * weights).sum(-1), weights.sum(-1)
//   functional/ranking/weighted_calibration.py       sum(w x, -1), sum(w t, -1)
//   regression MSE / R2 small-batch updates, metrics/window/* (+ the ring-slot index_copy and
//   the lifetime +=)
// with ONE launch for rows of <= kSingle elements (one block each; the common per-batch case)
// or two for longer rows (a grid of FP64 partials, then an ordered per-row combine).
//
// The statistic set is a template parameter (NEED): the FP64 VALU work per element is only
// what the metric asks for - computing every statistic for every element made the kernel
// FP64-bound (2.2 TB/s at 8192 x 1000 measured).  A scalar weight is applied once per row
// at the end (sum w x = w sum x) instead of per element.  Every input is read once, in 16-B
// vectors when rows are unit-stride f32.  Each output applies its own op (= / += / min / max)
// in its own dtype.  Deterministic: fixed partition and combine order.
#include <algorithm>
#include <cstdlib>

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kNStat = kRowRaw;        // raw stats (6 sums, 2 extrema)
constexpr int kVecPerThread = 4;       // float4 loads in flight per operand per thread
constexpr int64_t kPerBlock = kB * kVecPerThread * 4;  // 4096 elements per grid block
constexpr int64_t kSingle = 32768;     // rows up to this long: one block per row
constexpr int kCB = 1024;              // combine block

constexpr int bit(int s) { return 1 << s; }
constexpr int kNeedT = bit(kWT) | bit(kSSE) | bit(kWSSE) | bit(kWTT) | bit(kTMIN) | bit(kTMAX);
constexpr int kAll = 0xff;

struct Acc {
  double v[kNStat];
};

__device__ __forceinline__ void acc_init(Acc& a) {
#pragma unroll
  for (int k = 0; k < kRowSums; ++k) a.v[k] = 0.0;
  a.v[kTMIN] = __builtin_inf();
  a.v[kTMAX] = -__builtin_inf();
}

// torch.minimum / maximum propagate NaN
__device__ __forceinline__ double nmin(double a, double b) { return (a != a || b != b) ? __builtin_nan("") : fmin(a, b); }
__device__ __forceinline__ double nmax(double a, double b) { return (a != a || b != b) ? __builtin_nan("") : fmax(a, b); }

// NEED is compile time except for the generic instantiation (kAll), which tests g.need
template <int NEED, bool HAS_W>
__device__ __forceinline__ void acc_elem(Acc& a, int need, double x, double t, double w, bool valid = true) {
  auto want = [&](int s) { return (NEED & bit(s)) && (NEED != kAll || (need & bit(s))); };
  // HAS_W: per-element weights; otherwise the sums are unweighted here and scaled by w_scalar
  // once per row (finish_row)
  if (want(kWX)) a.v[kWX] += HAS_W ? w * x : x;
  if (want(kWT)) a.v[kWT] += HAS_W ? w * t : t;
  if (HAS_W && want(kW)) a.v[kW] += w;
  if (want(kSSE) || want(kWSSE)) {
    const double d = x - t;
    if (want(kSSE)) a.v[kSSE] += d * d;
    if (want(kWSSE)) a.v[kWSSE] += HAS_W ? w * d * d : d * d;
  }
  if (want(kWTT)) a.v[kWTT] += HAS_W ? w * t * t : t * t;
  // (an invalid lane arrives with x = t = w = 0: every sum above adds 0; the extrema select)
  if (want(kTMIN)) a.v[kTMIN] = valid ? nmin(a.v[kTMIN], t) : a.v[kTMIN];
  if (want(kTMAX)) a.v[kTMAX] = valid ? nmax(a.v[kTMAX], t) : a.v[kTMAX];
}

template <int NEED>
__device__ __forceinline__ void acc_merge(Acc& a, const Acc& b) {
#pragma unroll
  for (int k = 0; k < kRowSums; ++k)
    if (NEED & bit(k)) a.v[k] += b.v[k];
  if (NEED & bit(kTMIN)) a.v[kTMIN] = nmin(a.v[kTMIN], b.v[kTMIN]);
  if (NEED & bit(kTMAX)) a.v[kTMAX] = nmax(a.v[kTMAX], b.v[kTMAX]);
}

template <int NEED>
__device__ __forceinline__ Acc wave_merge(Acc a) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    Acc b;
#pragma unroll
    for (int k = 0; k < kNStat; ++k) b.v[k] = (NEED & bit(k)) ? __shfl_xor(a.v[k], o, kWave) : 0.0;
    acc_merge<NEED>(a, b);
  }
  return a;
}

// block reduction; the result is valid in thread 0
template <int NEED, int BS = kB>
__device__ Acc block_merge(Acc a) {
  __shared__ double lds[BS / kWave][kNStat];
  a = wave_merge<NEED>(a);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
#pragma unroll
    for (int k = 0; k < kNStat; ++k) lds[w][k] = a.v[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int j = 1; j < BS / kWave; ++j) {
      Acc b;
#pragma unroll
      for (int k = 0; k < kNStat; ++k) b.v[k] = lds[j][k];
      acc_merge<NEED>(a, b);
    }
  }
  return a;
}

// [lo, hi) of row r; VEC: f32 rows with unit stride (x, t, w as present; any 4-B alignment)
template <int NEED, bool HAS_W, bool VEC, int BS = kB, int VPT = kVecPerThread>
__device__ Acc reduce_range(const RowSumsArgs& g, int64_t r, int64_t lo, int64_t hi) {
  constexpr int64_t kChunk = static_cast<int64_t>(BS) * VPT * 4;
  constexpr bool HAS_T = (NEED & kNeedT) != 0;
  Acc a;
  acc_init(a);
  const int need = g.need;
  if constexpr (VEC) {
    // target extrema of f32 rows: fminf / fmaxf in f32 (exact) plus a NaN flag, merged into the
    // FP64 accumulator once at the end - the NaN-propagating FP64 min / max per element made PSNR
    // (auto range) 2.6 us slower than its fixed-range form at 8192 x 1000
    constexpr bool FX = NEED != kAll && (NEED & (bit(kTMIN) | bit(kTMAX))) != 0;
    constexpr int NB = FX ? (NEED & ~(bit(kTMIN) | bit(kTMAX))) : NEED;
    float fmn = __builtin_inff(), fmx = -__builtin_inff();
    bool fnan = false;
    auto fx = [&](float t, bool ok) {
      if constexpr (FX) {
        fmn = fminf(fmn, ok ? t : fmn);
        fmx = fmaxf(fmx, ok ? t : fmx);
        fnan |= ok && t != t;
      }
    };
    const float* xr = static_cast<const float*>(g.x) + r * g.x_rs;
    const float* tr = HAS_T ? static_cast<const float*>(g.t) + r * g.t_rs : nullptr;
    const float* wr = HAS_W ? static_cast<const float*>(g.w) + r * g.w_rs : nullptr;
    // 16-B loads at any 4-B alignment: the body is every whole group of 4 from lo
    const int64_t vlo = lo, vhi = lo + (hi - lo) / 4 * 4;
    // every float4 of the chunk is issued before any arithmetic: one memory round trip
    for (int64_t base = vlo; base < vhi; base += kChunk) {
      float4 xv[VPT], tv[VPT], wv[VPT];
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      // unconditional loads from a clamped (always valid) address: a per-lane `ok ? load : 0`
      // makes hipcc branch around each load and wait vmcnt(0) after it - one serial memory
      // round trip per float4 (the consumers below skip the out-of-range lanes)
#pragma unroll
      for (int u = 0; u < VPT; ++u) {
        const int64_t i = base + 4 * (static_cast<int64_t>(u) * BS + threadIdx.x);
        const int64_t ic = i < vhi ? i : vlo;
        xv[u] = load_f4u(xr + ic);  // 4-B alignment suffices (tea_common.h)
        tv[u] = HAS_T ? load_f4u(tr + ic) : z;
        wv[u] = HAS_W ? load_f4u(wr + ic) : z;
      }
      if (base + kChunk <= vhi) {  // whole chunk in range (block-uniform): no per-lane branch
#pragma unroll
        for (int u = 0; u < VPT; ++u) {
          acc_elem<NB, HAS_W>(a, need, xv[u].x, tv[u].x, wv[u].x);
          acc_elem<NB, HAS_W>(a, need, xv[u].y, tv[u].y, wv[u].y);
          acc_elem<NB, HAS_W>(a, need, xv[u].z, tv[u].z, wv[u].z);
          acc_elem<NB, HAS_W>(a, need, xv[u].w, tv[u].w, wv[u].w);
          fx(tv[u].x, true);
          fx(tv[u].y, true);
          fx(tv[u].z, true);
          fx(tv[u].w, true);
        }
      } else {
        // the row's last, partial chunk: the same loads, out-of-range lanes zeroed by selects
        // (a per-lane `if` here let hipcc sink the loads into the branch and wait on each -
        // every row's last block ran ~4 serial round trips: CTR 64 x 128000 took 17.7 us
        // against 8.1 us for the same bytes in one row)
#pragma unroll
        for (int u = 0; u < VPT; ++u) {
          const int64_t i = base + 4 * (static_cast<int64_t>(u) * BS + threadIdx.x);
          const bool ok = i < vhi;
          const float4 xm = make_float4(ok ? xv[u].x : 0.f, ok ? xv[u].y : 0.f, ok ? xv[u].z : 0.f, ok ? xv[u].w : 0.f);
          const float4 tm = make_float4(ok ? tv[u].x : 0.f, ok ? tv[u].y : 0.f, ok ? tv[u].z : 0.f, ok ? tv[u].w : 0.f);
          const float4 wm = make_float4(ok ? wv[u].x : 0.f, ok ? wv[u].y : 0.f, ok ? wv[u].z : 0.f, ok ? wv[u].w : 0.f);
          acc_elem<NB, HAS_W>(a, need, xm.x, tm.x, wm.x, ok);
          acc_elem<NB, HAS_W>(a, need, xm.y, tm.y, wm.y, ok);
          acc_elem<NB, HAS_W>(a, need, xm.z, tm.z, wm.z, ok);
          acc_elem<NB, HAS_W>(a, need, xm.w, tm.w, wm.w, ok);
          fx(tv[u].x, ok);
          fx(tv[u].y, ok);
          fx(tv[u].z, ok);
          fx(tv[u].w, ok);
        }
      }
    }
    if constexpr (FX) {
      const double nan = __builtin_nan("");
      if (NEED & bit(kTMIN)) a.v[kTMIN] = nmin(a.v[kTMIN], fnan ? nan : static_cast<double>(fmn));
      if (NEED & bit(kTMAX)) a.v[kTMAX] = nmax(a.v[kTMAX], fnan ? nan : static_cast<double>(fmx));
    }
    // ragged head / tail (< 4 elements each side)
    for (int64_t i = lo + threadIdx.x; i < min(vlo, hi); i += BS)
      acc_elem<NEED, HAS_W>(a, need, xr[i], HAS_T ? tr[i] : 0.f, HAS_W ? wr[i] : 0.f);
    for (int64_t i = max(vhi, vlo) + threadIdx.x; i < hi; i += BS)
      acc_elem<NEED, HAS_W>(a, need, xr[i], HAS_T ? tr[i] : 0.f, HAS_W ? wr[i] : 0.f);
  } else {
    for (int64_t i = lo + threadIdx.x; i < hi; i += BS) {
      const double x = load_as_f64(g.x, g.x_dt, r * g.x_rs + i * g.x_cs);
      const double t = HAS_T ? load_as_f64(g.t, g.t_dt, r * g.t_rs + i * g.t_cs) : 0.0;
      const double w = HAS_W ? load_as_f64(g.w, g.w_dt, r * g.w_rs + i * g.w_cs) : 0.0;
      acc_elem<NEED, HAS_W>(a, need, x, t, w);
    }
  }
  return a;
}

__device__ __forceinline__ double load_out(const RowSumsOut& o, int64_t r) {
  return load_as_f64(o.p, o.dt, r * o.stride);
}

// v rounded to the output dtype, combined in that dtype (as `state op tensor` would be)
__device__ void store_out(const RowSumsOut& o, int64_t r, double v) {
  const int64_t i = r * o.stride;
  if (o.dt == DType::f64) {
    double* p = static_cast<double*>(o.p) + i;
    switch (o.op) {
      case kSet: *p = v; break;
      case kAdd: *p = *p + v; break;
      case kMin: *p = nmin(*p, v); break;
      default: *p = nmax(*p, v); break;
    }
  } else {  // f32 states
    float* p = static_cast<float*>(o.p) + i;
    const float f = static_cast<float>(v);
    switch (o.op) {
      case kSet: *p = f; break;
      case kAdd: *p = *p + f; break;
      case kMin: *p = static_cast<float>(nmin(*p, f)); break;
      default: *p = static_cast<float>(nmax(*p, f)); break;
    }
  }
}

// thread 0: scale by a scalar weight, derive COUNT / W / RANGE, apply every output of row r
template <bool HAS_W>
__device__ void finish_row(const RowSumsArgs& g, int64_t r, Acc a) {
  const double n = static_cast<double>(g.n);
  if (!HAS_W) {
    const double w = g.w_scalar;
    a.v[kWX] *= w;
    a.v[kWT] *= w;
    a.v[kWSSE] *= w;
    a.v[kWTT] *= w;
    a.v[kW] = w * n;
  }
  double merged_min = 0.0, merged_max = 0.0;
  for (int k = 0; k < g.nout; ++k) {
    const RowSumsOut& o = g.out[k];
    if (o.first_row_only && r != 0) continue;
    double v;
    if (o.stat == kCOUNT) v = n;
    else if (o.stat == kRANGE) v = merged_max - merged_min;
    else v = a.v[o.stat];
    store_out(o, r, v);
    if (o.stat == kTMIN) merged_min = load_out(o, r);
    if (o.stat == kTMAX) merged_max = load_out(o, r);
  }
}

template <int NEED, bool HAS_W, bool VEC>
__global__ __launch_bounds__(kB) void row_sums_single_kernel(RowSumsArgs g) {
  const int64_t r = blockIdx.x;
  const Acc a = block_merge<NEED>(reduce_range<NEED, HAS_W, VEC>(g, r, 0, g.n));
  if (threadIdx.x == 0) finish_row<HAS_W>(g, r, a);
}

// grid blocks: each folds `span` elements (whole 4096-element chunks) of its row into FP64
// partials -> ws, stored stat-major ([row][stat][block]) so the combine reads only the NEEDed
// stats, contiguously (combined by row_sums_combine_kernel in block order: deterministic).
// A last-block-combines variant (agent release per block + ticket) was measured at 46 us for
// 8192 x 1000 (2000 release fences) against 14.6 + 10 us for two launches.
template <int NEED, bool HAS_W, bool VEC, int VPT = kVecPerThread>
__global__ __launch_bounds__(kB) void row_sums_grid_kernel(RowSumsArgs g, int64_t span) {
  const int64_t r = blockIdx.y;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * span;
  const int64_t hi = min(g.n, lo + span);
  const Acc a = block_merge<NEED>(reduce_range<NEED, HAS_W, VEC, kB, VPT>(g, r, lo, hi));
  if (g.pend) {
    // deferred mode: this block's slot, pre-scaled (a scalar weight differs per update), ADDED
    if (threadIdx.x == 0) {
      double* p = g.pend + r * kRowPendStats * g.pend_blocks + blockIdx.x;
      const double cnt = static_cast<double>(hi > lo ? hi - lo : 0);
      const double ws = HAS_W ? 1.0 : g.w_scalar;
#pragma unroll
      for (int k = 0; k < kRowSums; ++k) {
        if (k == kW) {
          if (NEED & bit(kW) || !HAS_W) pend_add(p + k * g.pend_blocks, HAS_W ? a.v[kW] : ws * cnt);
        } else if (NEED & bit(k)) {
          pend_add(p + k * g.pend_blocks, k == kSSE ? a.v[k] : ws * a.v[k]);
        }
      }
      if constexpr ((NEED & (bit(kTMIN) | bit(kTMAX))) != 0) {
        // the extrema slots are this block's own (plain read-modify-write, stream-ordered across
        // launches); a slot whose COUNT is still 0 holds no extrema yet (the buffer is zeroed)
        const bool fresh = p[kRowSums * g.pend_blocks] == 0.0;
        double* pmin = p + (kRowSums + 1) * g.pend_blocks;
        double* pmax = p + (kRowSums + 2) * g.pend_blocks;
        if (NEED & bit(kTMIN)) *pmin = fresh ? a.v[kTMIN] : nmin(*pmin, a.v[kTMIN]);
        if (NEED & bit(kTMAX)) *pmax = fresh ? a.v[kTMAX] : nmax(*pmax, a.v[kTMAX]);
      }
      pend_add(p + kRowSums * g.pend_blocks, cnt);
    }
    return;
  }
  if (threadIdx.x == 0) {
    double* p = g.ws + r * kNStat * g.blocks + blockIdx.x;
#pragma unroll
    for (int k = 0; k < kNStat; ++k)
      if (NEED & bit(k)) p[k * g.blocks] = a.v[k];
  }
}

// one block per row: every thread folds a strided subset of the partials, then a block merge
template <int NEED, bool HAS_W>
__global__ __launch_bounds__(kCB) void row_sums_combine_kernel(RowSumsArgs g) {
  const int64_t r = blockIdx.x;
  Acc m;
  acc_init(m);
  const double* src = g.ws + r * kNStat * g.blocks;
  for (int b = threadIdx.x; b < g.blocks; b += kCB) {
    Acc q;
    acc_init(q);
#pragma unroll
    for (int k = 0; k < kNStat; ++k)
      if (NEED & bit(k)) q.v[k] = src[k * g.blocks + b];
    acc_merge<NEED>(m, q);
  }
  m = block_merge<NEED, kCB>(m);
  if (threadIdx.x == 0) finish_row<HAS_W>(g, r, m);
}

// many rows: one wave per row (lane b folds partials b, b + 64, ...; shuffle merge; lane 0
// applies the outputs).  A 1024-thread block per row took 12.8 us for 64 rows of 8 partials
// (a 16-wave block merge and a serial tail per row) against 4.5 us for one row.
template <int NEED, bool HAS_W>
__global__ __launch_bounds__(kB) void row_sums_combine_rows_kernel(RowSumsArgs g) {
  const int64_t r = static_cast<int64_t>(blockIdx.x) * (kB / kWave) + (threadIdx.x >> 6);
  if (r >= g.rows) return;  // whole wave
  const int lane = threadIdx.x & (kWave - 1);
  Acc m;
  acc_init(m);
  const double* src = g.ws + r * kNStat * g.blocks;
  for (int b = lane; b < g.blocks; b += kWave) {
    Acc q;
    acc_init(q);
#pragma unroll
    for (int k = 0; k < kNStat; ++k)
      if (NEED & bit(k)) q.v[k] = src[k * g.blocks + b];
    acc_merge<NEED>(m, q);
  }
  m = wave_merge<NEED>(m);
  if (lane == 0) finish_row<HAS_W>(g, r, m);
}

// one launch for long rows: <= 256 fat blocks (1024 threads, ~one per CU) each fold a span
// of the row; each publishes its FP64 partial (plain store -> agent release -> ticket), and
// the block that draws the row's last ticket acquires, combines the partials in block order
// (deterministic) and applies the outputs.  With one block per CU the release costs one
// L2 write-back per CU (the 2000-block variant of this protocol paid 2000 and took 46 us).
// The ticket resets itself, so the zeroed workspace stays zeroed between calls.
constexpr int kFB = 1024;
constexpr int64_t kFoldChunk = static_cast<int64_t>(kFB) * kVecPerThread * 4;

template <int NEED, bool HAS_W, bool VEC>
__global__ __launch_bounds__(kFB) void row_sums_fold_kernel(RowSumsArgs g, int64_t span) {
  const int64_t r = blockIdx.y;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * span;
  const int64_t hi = min(g.n, lo + span);
  const Acc a = block_merge<NEED, kFB>(reduce_range<NEED, HAS_W, VEC, kFB>(g, r, lo, hi));
  __shared__ int s_last;
  if (threadIdx.x == 0) {
    double* p = g.ws + (r * g.blocks + blockIdx.x) * kNStat;
#pragma unroll
    for (int k = 0; k < kNStat; ++k) p[k] = a.v[k];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the partial reached L2 ...
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // ... is written back chip-wide ...
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(g.ticket + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == static_cast<unsigned>(g.blocks - 1)) ? 1 : 0;  // ... before the ticket
  }
  __syncthreads();
  if (!s_last) return;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  Acc m;
  acc_init(m);
  for (int b = threadIdx.x; b < g.blocks; b += kFB) {
    Acc q;
    const double* src = g.ws + (r * g.blocks + b) * kNStat;
#pragma unroll
    for (int k = 0; k < kNStat; ++k) q.v[k] = src[k];
    acc_merge<NEED>(m, q);
  }
  m = block_merge<NEED, kFB>(m);
  if (threadIdx.x == 0) {
    finish_row<HAS_W>(g, r, m);
    __hip_atomic_store(g.ticket + r, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// one launch for long rows (the default): grid blocks fold their span with 8 x 16-B loads per
// operand per thread in flight, store their FP64 partials WRITE-THROUGH and take a ticket; the
// row's last arriving block reads the partials back (sc1 loads), combines them in a fixed
// order (deterministic) and applies the outputs (tea_common.h wt_*: no release / acquire
// fence, whose buffer_wbl2 made the fat-block fold above no faster than two launches).
constexpr int kWtVPT = 8;
constexpr int64_t kWtChunk = static_cast<int64_t>(kB) * kWtVPT * 4;

template <int NEED, bool HAS_W, bool VEC>
__global__ __launch_bounds__(kB) void row_sums_wt_kernel(RowSumsArgs g, int64_t span) {
  const int64_t r = blockIdx.y;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * span;
  const int64_t hi = min(g.n, lo + span);
  const Acc a = block_merge<NEED>(reduce_range<NEED, HAS_W, VEC, kB, kWtVPT>(g, r, lo, hi));
  double* p = g.ws + r * kNStat * g.blocks + blockIdx.x;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < kNStat; ++k)
      if (NEED & bit(k)) wt_store(p + k * g.blocks, a.v[k]);
  }
  if (!wt_arrive_last(g.ticket + r, static_cast<unsigned>(g.blocks))) return;
  const double* src = g.ws + r * kNStat * g.blocks;
  Acc m;
  acc_init(m);
  for (int b0 = threadIdx.x; b0 < g.blocks; b0 += 2 * kB) {  // two partials' loads in flight
    const int b1 = b0 + kB;
    Acc q0, q1;
    acc_init(q0);
    acc_init(q1);
#pragma unroll
    for (int k = 0; k < kNStat; ++k) {
      if (!(NEED & bit(k))) continue;
      q0.v[k] = wt_load(src + k * g.blocks + b0);
      if (b1 < g.blocks) q1.v[k] = wt_load(src + k * g.blocks + b1);
    }
    acc_merge<NEED>(m, q0);
    if (b1 < g.blocks) acc_merge<NEED>(m, q1);
  }
  m = block_merge<NEED>(m);
  if (threadIdx.x == 0) finish_row<HAS_W>(g, r, m);
}

// deferred-mode fold: one block per row; every thread folds a strided share of the slots of
// each statistic (fixed partition + fixed LDS tree: deterministic), zeroes them, and thread 0
// applies the outputs as finish_row does (sums / COUNT added, extrema min / max-merged with the
// states, RANGE set from the merged extrema)
__global__ __launch_bounds__(kB) void row_sums_pend_fold_kernel(RowSumsArgs g, int used) {
  const int64_t r = blockIdx.x;
  __shared__ double lds[kRowPendStats][kB];
  double* base = g.pend + r * kRowPendStats * g.pend_blocks;
  {  // extrema first, while the COUNT slots still tell which slots hold any
    double mn = __builtin_inf(), mx = -__builtin_inf();
    double* cnt = base + kRowSums * g.pend_blocks;
    double* pmin = base + (kRowSums + 1) * g.pend_blocks;
    double* pmax = base + (kRowSums + 2) * g.pend_blocks;
    for (int b = threadIdx.x; b < used; b += kB) {
      if (cnt[b] != 0.0) {
        mn = nmin(mn, pmin[b]);
        mx = nmax(mx, pmax[b]);
      }
      pmin[b] = 0.0;
      pmax[b] = 0.0;
    }
    lds[kRowSums + 1][threadIdx.x] = mn;
    lds[kRowSums + 2][threadIdx.x] = mx;
  }
  for (int k = 0; k <= kRowSums; ++k) {
    double v = 0.0;
    for (int b = threadIdx.x; b < used; b += kB) {
      v += base[k * g.pend_blocks + b];
      base[k * g.pend_blocks + b] = 0.0;
    }
    lds[k][threadIdx.x] = v;
  }
  __syncthreads();
  for (int h = kB / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) {
      for (int k = 0; k <= kRowSums; ++k) lds[k][threadIdx.x] += lds[k][threadIdx.x + h];
      lds[kRowSums + 1][threadIdx.x] = nmin(lds[kRowSums + 1][threadIdx.x], lds[kRowSums + 1][threadIdx.x + h]);
      lds[kRowSums + 2][threadIdx.x] = nmax(lds[kRowSums + 2][threadIdx.x], lds[kRowSums + 2][threadIdx.x + h]);
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  double merged_min = 0.0, merged_max = 0.0;
  for (int k = 0; k < g.nout; ++k) {
    const RowSumsOut& o = g.out[k];
    if (o.first_row_only && r != 0) continue;
    double v;
    if (o.stat == kCOUNT) v = lds[kRowSums][0];
    else if (o.stat == kTMIN) v = lds[kRowSums + 1][0];
    else if (o.stat == kTMAX) v = lds[kRowSums + 2][0];
    else if (o.stat == kRANGE) v = merged_max - merged_min;
    else v = lds[o.stat][0];
    store_out(o, r, v);
    if (o.stat == kTMIN) merged_min = load_out(o, r);
    if (o.stat == kTMAX) merged_max = load_out(o, r);
  }
}

// the outputs a deferred update can fold: sums / COUNT added, extrema min / max, RANGE set
bool pend_outputs_ok(const RowSumsArgs& a) {
  for (int k = 0; k < a.nout; ++k) {
    const RowSumsOut& o = a.out[k];
    const bool ok = o.stat == kTMIN ? o.op == kMin : o.stat == kTMAX ? o.op == kMax
                  : o.stat == kRANGE ? o.op == kSet : o.op == kAdd;
    if (!ok) return false;
  }
  return true;
}

bool vec_ok(const void* p, DType dt, int64_t /*rs*/, int64_t cs) {
  return p == nullptr || (dt == DType::f32 && cs == 1);  // 16-B loads need only 4-B alignment
}

template <int NEED, bool HAS_W>
int launch_need(const RowSumsArgs& a, bool vec, hipStream_t stream) {
  if (a.blocks <= 1) {
    if (vec) hipLaunchKernelGGL((row_sums_single_kernel<NEED, HAS_W, true>), dim3(a.rows), dim3(kB), 0, stream, a);
    else hipLaunchKernelGGL((row_sums_single_kernel<NEED, HAS_W, false>), dim3(a.rows), dim3(kB), 0, stream, a);
  } else if (a.ticket && a.wt) {  // one launch: write-through partials + last-block combine
    const int64_t chunks = (a.n + kWtChunk - 1) / kWtChunk;
    const int64_t span = (chunks + a.blocks - 1) / a.blocks * kWtChunk;
    const dim3 grid(static_cast<unsigned>(a.blocks), static_cast<unsigned>(a.rows));
    if (vec) hipLaunchKernelGGL((row_sums_wt_kernel<NEED, HAS_W, true>), grid, dim3(kB), 0, stream, a, span);
    else hipLaunchKernelGGL((row_sums_wt_kernel<NEED, HAS_W, false>), grid, dim3(kB), 0, stream, a, span);
  } else if (a.ticket) {  // one launch: fat blocks + last-block combine
    const int64_t span = (a.n + a.blocks - 1) / a.blocks;
    const int64_t span_c = (span + kFoldChunk - 1) / kFoldChunk * kFoldChunk;
    const dim3 grid(static_cast<unsigned>(a.blocks), static_cast<unsigned>(a.rows));
    if (vec) hipLaunchKernelGGL((row_sums_fold_kernel<NEED, HAS_W, true>), grid, dim3(kFB), 0, stream, a, span_c);
    else hipLaunchKernelGGL((row_sums_fold_kernel<NEED, HAS_W, false>), grid, dim3(kFB), 0, stream, a, span_c);
  } else {
    const int64_t chunks = (a.n + kPerBlock - 1) / kPerBlock;
    const int64_t span = (chunks + a.blocks - 1) / a.blocks * kPerBlock;
    const dim3 grid(static_cast<unsigned>(a.blocks), static_cast<unsigned>(a.rows));
    if (a.pend) {  // deferred: no combine launch; 8 x 16-B loads per operand in flight per thread
      static const int vpt = [] {
        const char* e = std::getenv("TORCHEVAL_AMD_K5B_PEND_VPT");
        const int v = e != nullptr ? std::atoi(e) : 8;
        return v == 4 || v == 16 ? v : 8;
      }();
      if (vpt == 16) {
        if (vec) hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, true, 16>), grid, dim3(kB), 0, stream, a, span);
        else hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, false, 16>), grid, dim3(kB), 0, stream, a, span);
      } else if (vpt == 8) {
        if (vec) hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, true, 8>), grid, dim3(kB), 0, stream, a, span);
        else hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, false, 8>), grid, dim3(kB), 0, stream, a, span);
      } else {
        if (vec) hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, true>), grid, dim3(kB), 0, stream, a, span);
        else hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, false>), grid, dim3(kB), 0, stream, a, span);
      }
      return static_cast<int>(hipGetLastError());
    }
    if (vec) hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, true>), grid, dim3(kB), 0, stream, a, span);
    else hipLaunchKernelGGL((row_sums_grid_kernel<NEED, HAS_W, false>), grid, dim3(kB), 0, stream, a, span);
    if (a.rows == 1) {
      hipLaunchKernelGGL((row_sums_combine_kernel<NEED, HAS_W>), dim3(1), dim3(kCB), 0, stream, a);
    } else {
      const unsigned cb = static_cast<unsigned>((a.rows + kB / kWave - 1) / (kB / kWave));
      hipLaunchKernelGGL((row_sums_combine_rows_kernel<NEED, HAS_W>), dim3(cb), dim3(kB), 0, stream, a);
    }
  }
  return static_cast<int>(hipGetLastError());
}

template <int NEED>
int launch_w(const RowSumsArgs& a, bool vec, hipStream_t stream) {
  return a.w ? launch_need<NEED, true>(a, vec, stream) : launch_need<NEED, false>(a, vec, stream);
}

}  // namespace

int row_sums_blocks(int64_t rows, int64_t n) {
  if (n <= kSingle) return 1;
  // about 512 blocks over all rows (each folds whole 4096-element chunks): enough bytes in
  // flight per CU without thousands of one-chunk blocks and partials (csrc/bench/
  // k5b_variants.hip, Sum 8192 x 1000: 2000 blocks 9.1 us, 1024 8.4, 512 7.95, 256 9.1)
  int64_t cap = 512;
  if (const char* e = std::getenv("TORCHEVAL_AMD_K5B_GRID")) cap = std::max(1, std::atoi(e));
  const int64_t chunks = (n + kPerBlock - 1) / kPerBlock;
  const int64_t per_row = std::max<int64_t>(2, cap / std::max<int64_t>(rows, 1));
  return static_cast<int>(std::min(chunks, per_row));
}

int row_sums_wt_blocks(int64_t rows, int64_t n) {
  if (n <= kSingle) return 1;
  int64_t cap = 512;
  if (const char* e = std::getenv("TORCHEVAL_AMD_K5B_GRID")) cap = std::max(1, std::atoi(e));
  const int64_t chunks = (n + kWtChunk - 1) / kWtChunk;
  const int64_t per_row = std::max<int64_t>(2, cap / std::max<int64_t>(rows, 1));
  return static_cast<int>(std::min(chunks, per_row));
}

int row_sums_fold_blocks(int64_t rows, int64_t n) {
  if (n <= kSingle) return 1;
  const int64_t per_row = std::max<int64_t>(2, 256 / std::max<int64_t>(rows, 1));
  return static_cast<int>(std::min<int64_t>(per_row, (n + kFoldChunk - 1) / kFoldChunk));
}

int launch_row_sums_fold(const RowSumsArgs& a, int blocks_used, hipStream_t stream) {
  if (a.rows <= 0 || blocks_used <= 0 || !a.pend) return 0;
  if (blocks_used > a.pend_blocks || !pend_outputs_ok(a)) return -2;
  hipLaunchKernelGGL(row_sums_pend_fold_kernel, dim3(static_cast<unsigned>(a.rows)), dim3(kB), 0, stream, a,
                     blocks_used);
  return static_cast<int>(hipGetLastError());
}

int launch_row_sums(const RowSumsArgs& a, hipStream_t stream) {
  if (a.rows <= 0) return 0;
  if (a.pend) {  // deferred mode: grid blocks only, within the slots, sums / W / COUNT ADD outputs
    if (a.blocks < 2 || a.blocks > a.pend_blocks || a.ticket || !pend_outputs_ok(a)) return -2;
  }
  if ((a.n > 0 && a.x == nullptr) || (a.blocks > 1 && !a.ws && !a.pend)) return -2;  // empty rows: outputs only
  if (a.ticket && a.blocks < 2) return -2;
  const bool vec = vec_ok(a.x, a.x_dt, a.x_rs, a.x_cs) && vec_ok(a.t, a.t_dt, a.t_rs, a.t_cs) &&
                   vec_ok(a.w, a.w_dt, a.w_rs, a.w_cs);
  // the statistic sets the metrics use; W is derived when the weight is a scalar
  const int need = a.w ? a.need : (a.need & ~bit(kW));
  switch (need) {
    case bit(kWX): return launch_w<bit(kWX)>(a, vec, stream);                               // Sum, Mean, CTR
    case bit(kWX) | bit(kW): return launch_w<bit(kWX) | bit(kW)>(a, vec, stream);           // weighted Mean, CTR
    case bit(kWX) | bit(kWT): return launch_w<bit(kWX) | bit(kWT)>(a, vec, stream);         // WC
    case bit(kSSE): return launch_w<bit(kSSE)>(a, vec, stream);                             // PSNR (fixed range)
    case bit(kSSE) | bit(kTMIN) | bit(kTMAX):                                               // PSNR (auto range)
      return launch_w<bit(kSSE) | bit(kTMIN) | bit(kTMAX)>(a, vec, stream);
    case bit(kWSSE): return launch_w<bit(kWSSE)>(a, vec, stream);                           // MSE
    case bit(kWSSE) | bit(kW): return launch_w<bit(kWSSE) | bit(kW)>(a, vec, stream);       // weighted MSE
    case bit(kWT) | bit(kSSE) | bit(kWTT):                                                  // R2
      return launch_w<bit(kWT) | bit(kSSE) | bit(kWTT)>(a, vec, stream);
    default: return launch_w<kAll>(a, vec, stream);
  }
}

}  // namespace tea
