// K5 / K6: fused weighted reductions for regression, aggregation and normalized entropy.
//
// K5 column_moments: one pass over x [N, D], t [N, D] (optional w [N]) accumulating any of
//   sse[j] = sum_i w_i (t_ij - x_ij)^2, st[j] = sum_i w_i t_ij, stt[j] = sum_i w_i t_ij^2,
//   sx[j] = sum_i w_i x_ij, sw = sum_i w_i
//   replacing mean_squared_error.py:81-97 (square, mul, sum x2), r2_score.py:97-106 (square x2,
//   sum x3, torch.tensor(N)), aggregation sum/mean and the ranking CTR / calibration sums.
//   Threads own a fixed column (tid % Dt) and stride over rows, accumulate in FP64, reduce
//   through LDS per column and add one float atomic per (block, column).
// K6 ne_sums: per task row: sum w*BCE(x, t) (or BCE-with-logits), sum w, sum w*t in FP64,
//   plus a device-side range flag for probabilities outside [0, 1]
//   (binary_normalized_entropy.py:86-117 and the host-synchronising check at :145-147).
#include <algorithm>
#include <cstdlib>

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;

// ---------------------------------------------------------------- K5 column moments
// Two deterministic passes, no atomics:
//   A) grid (P row-chunks) x (column tiles of 64 column groups).  A thread owns V consecutive
//      columns (V = 4 with 16-B loads for contiguous f32 inputs, else 1) and walks its chunk's
//      rows with a U-row unroll so 2 x U independent loads are in flight; FP64 accumulators.
//      The block folds its row lanes through LDS and writes only the requested statistics to
//      ws[chunk][slot][col] (compact slots: MSE writes 1 stat, R2 3).
//   B) 16 columns x 16 partial groups per block sum the P partials and add the FP64 total to
//      the float32 output once (single writer per column: deterministic, no same-address
//      atomics - v1 issued P x d float atomics, 256-way contended per column).
constexpr int kStats = 4;  // sse, st, stt, sx
constexpr int kColGroups = 64;

struct Slots {
  int s[kStats];
  int n;
};

__device__ __forceinline__ Slots slots_of(const MomentsArgs& a) {
  Slots r;
  const float* outs[kStats] = {a.sse, a.st, a.stt, a.sx};
  r.n = 0;
#pragma unroll
  for (int k = 0; k < kStats; ++k) r.s[k] = outs[k] ? r.n++ : -1;
  return r;
}

template <int V>
__device__ __forceinline__ void load_v(const void* p, DType dt, int64_t off, int64_t cstride, float (&v)[V]) {
  if constexpr (V == 4) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + off);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = static_cast<float>(load_as_f64(p, dt, off + e * cstride));
  }
}

template <int V>
__global__ __launch_bounds__(kB) void moments_partial_kernel(MomentsArgs a) {
  constexpr int U = 4;
  const int64_t d = a.d;
  const int64_t dv = (d + V - 1) / V;
  const int64_t c0 = static_cast<int64_t>(blockIdx.y) * kColGroups;
  const int CG = static_cast<int>(dv - c0 < kColGroups ? dv - c0 : kColGroups);
  const int RPP = kB / CG;
  const int cg = threadIdx.x % CG;
  const int rl = threadIdx.x / CG;
  const bool active = rl < RPP;
  const int64_t chunk = (a.n + gridDim.x - 1) / gridDim.x;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * chunk;
  const int64_t r1 = r0 + chunk < a.n ? r0 + chunk : a.n;
  const bool want_x = a.sse || a.sx, want_t = a.sse || a.st || a.stt;
  const Slots sl = slots_of(a);
  const int64_t stride = sl.n * d + 1;
  __shared__ double lds[kStats * V][kB];
  __shared__ double lds_w[kB];
  double* ws = a.ws + static_cast<int64_t>(blockIdx.x) * stride;

  double acc[kStats][V];
#pragma unroll
  for (int k = 0; k < kStats; ++k)
#pragma unroll
    for (int e = 0; e < V; ++e) acc[k][e] = 0.0;
  double wsum = 0.0;
  const int64_t col = (c0 + cg) * V;
  const int nv = static_cast<int>(d - col < V ? d - col : V);
  if (active) {
    for (int64_t i = r0 + rl; i < r1; i += static_cast<int64_t>(RPP) * U) {
      float xv[U][V], tv[U][V], wv[U];
      if constexpr (V == 4) {
        // f32 rows (launch_column_moments checked dtype, unit stride, alignment): every load
        // from a clamped valid row, masked after - guarded loads through the dtype dispatch
        // compiled to a branch + vmcnt(0) per load
        // both operands always loaded (an absent one aliases the other; masked below)
        const float* xp = static_cast<const float*>(want_x ? a.x : a.t);
        const float* tp = static_cast<const float*>(want_t ? a.t : a.x);
        const int64_t xrs = want_x ? a.x_row_stride : a.t_row_stride;
        const int64_t trs = want_t ? a.t_row_stride : a.x_row_stride;
        float4 xq[U], tq[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int64_t row = i + static_cast<int64_t>(u) * RPP;
          const int64_t rc = row < r1 ? row : i;
          xq[u] = *reinterpret_cast<const float4*>(xp + rc * xrs + col);
          tq[u] = *reinterpret_cast<const float4*>(tp + rc * trs + col);
          wv[u] = a.w ? static_cast<float>(load_as_f64(a.w, a.w_dt, rc * a.w_stride)) : 1.f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const bool ok = i + static_cast<int64_t>(u) * RPP < r1;
          const bool okx = ok && want_x, okt = ok && want_t;
          wv[u] = ok ? wv[u] : 0.f;
          xv[u][0] = okx ? xq[u].x : 0.f;
          xv[u][1] = okx ? xq[u].y : 0.f;
          xv[u][2] = okx ? xq[u].z : 0.f;
          xv[u][3] = okx ? xq[u].w : 0.f;
          tv[u][0] = okt ? tq[u].x : 0.f;
          tv[u][1] = okt ? tq[u].y : 0.f;
          tv[u][2] = okt ? tq[u].z : 0.f;
          tv[u][3] = okt ? tq[u].w : 0.f;
        }
      } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t row = i + static_cast<int64_t>(u) * RPP;
        const bool ok = row < r1;
#pragma unroll
        for (int e = 0; e < V; ++e) xv[u][e] = tv[u][e] = 0.f;
        wv[u] = ok ? (a.w ? static_cast<float>(load_as_f64(a.w, a.w_dt, row * a.w_stride)) : 1.f) : 0.f;
        if (ok && V == 4 && nv == 4) {
          if (want_x) load_v<V>(a.x, a.x_dt, row * a.x_row_stride + col, 1, xv[u]);
          if (want_t) load_v<V>(a.t, a.t_dt, row * a.t_row_stride + col, 1, tv[u]);
        } else if (ok) {
          for (int e = 0; e < nv; ++e) {
            if (want_x) xv[u][e] = static_cast<float>(load_as_f64(a.x, a.x_dt, row * a.x_row_stride + (col + e) * a.x_col_stride));
            if (want_t) tv[u][e] = static_cast<float>(load_as_f64(a.t, a.t_dt, row * a.t_row_stride + (col + e) * a.t_col_stride));
          }
        }
      }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const double w = wv[u];
        wsum += w;
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const double x = xv[u][e], t = tv[u][e], r = t - x;
          acc[0][e] += w * r * r;
          acc[1][e] += w * t;
          acc[2][e] += w * t * t;
          acc[3][e] += w * x;
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kStats; ++k)
#pragma unroll
    for (int e = 0; e < V; ++e) lds[k * V + e][threadIdx.x] = acc[k][e];
  lds_w[threadIdx.x] = (cg == 0 && active) ? wsum : 0.0;  // one column group counts weights
  __syncthreads();
  if (a.mse_mode == 2) {
    // functional MSE, uniform average: with per-row weights every column divides by the same
    // weight total, so mean_j(sse_j / sw) = (sum_j sse_j) / (d sw) and the block only hands
    // on {its sse summed over its columns, its weight total} - no per-column partials, no
    // per-column finalize (mse_scalar_kernel folds these pairs)
    double tot = 0.0;
    if (threadIdx.x < CG) {  // CG <= 64: wave 0
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double s = 0.0;
        for (int r = 0; r < RPP; ++r) s += lds[e][r * CG + threadIdx.x];
        tot += (c0 + threadIdx.x) * V + e < d ? s : 0.0;
      }
    }
    if (threadIdx.x < 64) {
      tot = wave_sum(tot);
      if (threadIdx.x == 0) {
        double sw = 0.0;
        if (blockIdx.y == 0)
          for (int r = 0; r < kB; ++r) sw += lds_w[r];
        double* pair = a.ws + 2 * (static_cast<int64_t>(blockIdx.x) * gridDim.y + blockIdx.y);
        pair[0] = tot;
        pair[1] = sw;
      }
    }
    return;
  }
  if (threadIdx.x < CG) {
#pragma unroll
    for (int k = 0; k < kStats; ++k) {
      if (sl.s[k] < 0) continue;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        double s = 0.0;
        for (int r = 0; r < RPP; ++r) s += lds[k * V + e][r * CG + threadIdx.x];
        const int64_t cc = (c0 + threadIdx.x) * V + e;
        if (cc < d) ws[sl.s[k] * d + cc] = s;
      }
    }
  }
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    double s = 0.0;
    for (int r = 0; r < kB; ++r) s += lds_w[r];
    ws[sl.n * d] = s;
  }
}

// B) G partial groups x C columns per block: each thread sums P/G partials (independent loads,
// unrolled), the groups fold through an LDS tree (v1 summed the 32 groups of all 5 stats in
// ONE thread per column: a ~4 us serial tail), then one thread per column writes.  Every block
// also folds the weight total, so the functional MSE compute (divide by the clamped signed
// weight total, then the column mean via a deterministic last-block-done fold) happens here
// instead of as ~6 ATen launches (the column mean is one more single-block launch: a
// last-block-done fold would need an agent-scope release fence per block, which
// tea_fold.h measured at +47 us for a 2048-block grid).
constexpr int kFG = 64, kFC = kB / kFG;  // 4 columns x 64 partial groups: 250 blocks at d = 1000 (32 x 8: 125)

// functional MSE (uniform average): fold the partial kernel's {sse, weight} pairs in a fixed
// order, then the reference's float32 sse / (clamp(|sw|, eps) sign(sw)) averaged over columns
// (mean_squared_error.py:100-111), as one quotient
__global__ __launch_bounds__(kB) void mse_scalar_kernel(const double* pairs, int64_t npairs, int64_t d,
                                                        float* out) {
  __shared__ double lds[2][kB / 64];
  double s = 0.0, w = 0.0;
  for (int64_t p = threadIdx.x; p < npairs; p += kB) {
    s += pairs[2 * p];
    w += pairs[2 * p + 1];
  }
  s = wave_sum(s);
  w = wave_sum(w);
  if (lane_id() == 0) {
    lds[0][threadIdx.x >> 6] = s;
    lds[1][threadIdx.x >> 6] = w;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double st = 0.0, wt = 0.0;
    for (int q = 0; q < kB / 64; ++q) {
      st += lds[0][q];
      wt += lds[1][q];
    }
    const float sw = static_cast<float>(wt);
    const float eps = 2.220446049250313e-16f;
    const float sgn = sw > 0.f ? 1.f : (sw < 0.f ? -1.f : 0.f);
    const double den = static_cast<double>(fmaxf(fabsf(sw), eps) * sgn) * static_cast<double>(d);
    *out = static_cast<float>(st / den);
  }
}

// final scalar of the fused functional computes, in a fixed order (per-thread strided sums +
// LDS tree): MSE / R2 uniform mean (modes 2, 4), R2 variance-weighted sum (mode 5); then the
// adjusted-R2 correction when num_regressors != 0
__device__ __forceinline__ float adjust_r2(float r2, int64_t n, int k) {
  // reference r2_score.py:_compute: 1 - (1 - r2) * (n - 1) / (n - k - 1) in float32
  return 1.f - (1.f - r2) * static_cast<float>(n - 1) / static_cast<float>(n - k - 1);
}

__global__ __launch_bounds__(kB) void post_reduce_kernel(const float* vals, const float* tss, int64_t d, int mode,
                                                          int64_t n, int k, float* out) {
  __shared__ double lds[2][kB];
  double s = 0.0, st = 0.0;
  for (int64_t j = threadIdx.x; j < d; j += kB) {
    if (mode == 5) {
      s += static_cast<double>(vals[j]) * tss[j];
      st += tss[j];
    } else {
      s += vals[j];
    }
  }
  lds[0][threadIdx.x] = s;
  lds[1][threadIdx.x] = st;
  __syncthreads();
  for (int h = kB / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h) {
      lds[0][threadIdx.x] += lds[0][threadIdx.x + h];
      lds[1][threadIdx.x] += lds[1][threadIdx.x + h];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    float r = mode == 5 ? static_cast<float>(lds[0][0] / lds[1][0]) : static_cast<float>(lds[0][0] / static_cast<double>(d));
    if (mode >= 3 && k != 0) r = adjust_r2(r, n, k);
    *out = r;
  }
}

__global__ __launch_bounds__(kB) void moments_finalize_kernel(MomentsArgs a, int P) {
  const int64_t d = a.d;
  const int c = threadIdx.x % kFC, grp = threadIdx.x / kFC;
  const int64_t col = static_cast<int64_t>(blockIdx.x) * kFC + c;
  const Slots sl = slots_of(a);
  const int64_t stride = sl.n * d + 1;
  __shared__ double lds[kFG][kStats + 1][kFC];
  double s[kStats + 1] = {0, 0, 0, 0, 0};
#pragma unroll 8
  for (int p = grp; p < P; p += kFG) {  // independent loads: the unroll keeps 8 in flight
    const double* ws = a.ws + p * stride;
    if (col < d) {
#pragma unroll
      for (int k = 0; k < kStats; ++k)
        if (sl.s[k] >= 0) s[k] += ws[sl.s[k] * d + col];
    }
    if (c == 0) s[kStats] += ws[sl.n * d];
  }
#pragma unroll
  for (int k = 0; k <= kStats; ++k) lds[grp][k][c] = s[k];
  __syncthreads();
#pragma unroll
  for (int h = kFG / 2; h >= 1; h >>= 1) {  // fixed-order tree: deterministic
    if (grp < h) {
#pragma unroll
      for (int k = 0; k <= kStats; ++k)
        if (k == kStats ? c == 0 : sl.s[k] >= 0) lds[grp][k][c] += lds[grp + h][k][c];
    }
    __syncthreads();
  }
  if (grp == 0) {
    const double w_tot = lds[0][kStats][0];
    if (col < d) {
      float* outs[kStats] = {a.sse, a.st, a.stt, a.sx};
#pragma unroll
      for (int k = 0; k < kStats; ++k) {
        if (!outs[k]) continue;
        float& o = outs[k][col * a.out_stride];
        o = a.overwrite ? static_cast<float>(lds[0][k][c]) : o + static_cast<float>(lds[0][k][c]);
      }
      if (a.mse_mode == 1 || a.mse_mode == 2) {
        // reference mean_squared_error.py:100-111 in float32: sse / (clamp(|sw|, eps) * sign(sw))
        const float sse = a.sse[col * a.out_stride];
        const float sw = a.sw ? (a.overwrite ? static_cast<float>(w_tot) : *a.sw + static_cast<float>(w_tot))
                              : static_cast<float>(w_tot);
        const float eps = 2.220446049250313e-16f;
        const float sgn = sw > 0.f ? 1.f : (sw < 0.f ? -1.f : 0.f);
        const float raw = sse / (fmaxf(fabsf(sw), eps) * sgn);
        (a.mse_mode == 1 ? a.mse_out : a.mse_part_f)[col] = raw;
      } else if (a.mse_mode >= 3) {
        // reference r2_score.py:_compute in float32: tss = stt - st^2 / n, r2 = 1 - rss / tss
        const float rss = a.sse[col * a.out_stride], so = a.st[col * a.out_stride];
        const float sso = a.stt[col * a.out_stride];
        const float tss = sso - (so * so) / static_cast<float>(a.num_obs);
        const float r2 = 1.f - rss / tss;
        if (a.mse_mode == 3) {
          a.mse_out[col] = a.num_regressors != 0 ? adjust_r2(r2, a.num_obs, a.num_regressors) : r2;
        } else {
          a.mse_part_f[col] = r2;
          a.mse_part_f[d + col] = tss;
        }
      }
    }
    if (blockIdx.x == 0 && c == 0 && a.sw) {
      *a.sw = a.overwrite ? static_cast<float>(w_tot) : *a.sw + static_cast<float>(w_tot);
    }
  }
}

// ---------------------------------------------------------------- K5 v2: one launch
// f32 x / t with unit column stride and d >= 4 (any row stride, any 4-B alignment: the 16-B
// loads need only 4-B alignment on gfx950, tea_common.h load_f4u), optional f32 row weights.
//   grid (R row chunks) x (column tiles of CG groups of 4 columns); 256 threads = CG column
//   groups x RPP = 256 / CG row lanes.  A thread owns 4 columns and walks its row lane with
//   U = 8 rows unrolled: 8 (16 with both operands) 16-B loads in flight, FP64 accumulation.
//   The tail group of a width that is not a multiple of 4 loads the row's LAST 4 columns
//   (shifted back by sh = 1..3) and drops its first sh lanes: every column is read once by
//   16-B loads whatever d % 4 (the v1 kernel fell back to scalar loads: 2.6x slower at 1001).
//   Block epilogue: row lanes fold through LDS; each column's FP64 partial is stored
//   write-through; the tile's LAST arriving block (ticket) sums the R partials in chunk
//   order (deterministic) and applies the outputs / the fused MSE / R2 compute - no second
//   launch (v1: partial + finalize (+ a scalar fold) = 2-3 launches).  The scalar modes
//   (uniform / variance-weighted averages) hand per-tile sums to the last tile the same way.
constexpr int kU2 = 8;

template <int NEED>
struct NeedInfo {
  static constexpr bool sse = NEED & 1, st = NEED & 2, stt = NEED & 4, sx = NEED & 8;
  static constexpr int ns = int(sse) + int(st) + int(stt) + int(sx);
  static constexpr bool want_x = sse || sx, want_t = sse || st || stt;
  // slot of each statistic in the compact partial layout
  static constexpr int s_sse = 0, s_st = int(sse), s_stt = int(sse) + int(st), s_sx = int(sse) + int(st) + int(stt);
};

struct V2Layout {
  int64_t tiles, tc;  // tiles, columns per tile
  __device__ __forceinline__ int64_t part(int tile, int slot, int ns, int R, int rc) const {
    return ((static_cast<int64_t>(tile) * ns + slot) * R + rc) * tc;
  }
  __device__ __forceinline__ int64_t wpart(int ns, int R) const { return tiles * ns * R * tc; }  // [tiles][R]
  __device__ __forceinline__ int64_t tscal(int ns, int R) const { return wpart(ns, R) + tiles * R; }  // [tiles][4]
};

__device__ __forceinline__ float4 f4_select(bool ok, float4 v) {
  return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

// one unrolled batch of kU2 rows of a row lane: loads from clamped valid rows (a guarded load
// compiles to a branch and a vmcnt(0) per load), masked when accumulated
template <int NEED, bool HAS_W>
struct V2Batch {
  float4 xq[kU2], tq[kU2];
  float wv[kU2];
  __device__ __forceinline__ void load(const float* xp, const float* tp, const float* wp, int64_t xrs, int64_t trs,
                                       int64_t ws, int64_t i, int64_t r1, int rpp) {
    using NI = NeedInfo<NEED>;
#pragma unroll
    for (int u = 0; u < kU2; ++u) {
      const int64_t row = i + static_cast<int64_t>(u) * rpp;
      const int64_t rr = row < r1 ? row : i;
      if (NI::want_x) xq[u] = load_f4u(xp + rr * xrs);
      if (NI::want_t) tq[u] = load_f4u(tp + rr * trs);
      if (HAS_W) wv[u] = wp[rr * ws];
    }
  }
  __device__ __forceinline__ void accumulate(double (&acc)[4][4], double& wsum, int64_t i, int64_t r1, int rpp) const {
    using NI = NeedInfo<NEED>;
#pragma unroll
    for (int u = 0; u < kU2; ++u) {
      const bool ok = i + static_cast<int64_t>(u) * rpp < r1;
      const float4 x4 = NI::want_x ? f4_select(ok, xq[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 t4 = NI::want_t ? f4_select(ok, tq[u]) : make_float4(0.f, 0.f, 0.f, 0.f);
      const double w = HAS_W ? (ok ? static_cast<double>(wv[u]) : 0.0) : 1.0;
      if (HAS_W) wsum += w;
      const float xs[4] = {x4.x, x4.y, x4.z, x4.w}, ts[4] = {t4.x, t4.y, t4.z, t4.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double x = xs[e], t = ts[e];
        if (NI::sse) {
          const double r = t - x;
          acc[0][e] += HAS_W ? w * r * r : r * r;
        }
        if (NI::st) acc[1][e] += HAS_W ? w * t : t;
        if (NI::stt) acc[2][e] += HAS_W ? w * t * t : t * t;
        if (NI::sx) acc[3][e] += HAS_W ? w * x : x;
      }
    }
  }
};

// sum over r = q, q + step, ... < R of src[r * stride] with every load of the share issued
// before the first add (16 at a time)
__device__ __forceinline__ double wt_strided_sum(const double* src, int q, int step, int R, int64_t stride) {
  double v = 0.0;
  for (int r0 = q; r0 < R; r0 += 16 * step) {
    double t[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int r = r0 + j * step;
      t[j] = r < R ? wt_load(src + static_cast<int64_t>(r) * stride) : 0.0;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) v += t[j];
  }
  return v;
}

// eps-clamped signed weight total of the reference (mean_squared_error.py:100-111), float32
__device__ __forceinline__ float mse_den(double w_tot) {
  const float sw = static_cast<float>(w_tot);
  const float eps = 2.220446049250313e-16f;
  const float sgn = sw > 0.f ? 1.f : (sw < 0.f ? -1.f : 0.f);
  return fmaxf(fabsf(sw), eps) * sgn;
}

template <int CG, int NEED, bool HAS_W, bool PIPE>
__global__ __launch_bounds__(kB) void moments_v2_kernel(MomentsArgs a) {
  using NI = NeedInfo<NEED>;
  constexpr int RPP = kB / CG, TC = CG * 4, NS = NI::ns, TP = kB / TC;
  const int cg = threadIdx.x % CG, rl = threadIdx.x / CG;
  const int rc = blockIdx.x, tile = blockIdx.y, R = gridDim.x;
  const int64_t d = a.d, n = a.n;
  const int64_t tbase = static_cast<int64_t>(tile) * TC;
  const int64_t col = tbase + cg * 4;
  const bool active = col < d;
  const int64_t lcol = col + 4 <= d ? col : d - 4;  // d >= 4 (launcher)
  const int sh = active ? static_cast<int>(col - lcol) : 0;
  const int64_t r0 = static_cast<int64_t>(rc) * a.v2_chunk;
  const int64_t r1 = r0 + a.v2_chunk < n ? r0 + a.v2_chunk : n;
  const float* xp = static_cast<const float*>(NI::want_x ? a.x : a.t) + lcol;
  const float* tp = static_cast<const float*>(NI::want_t ? a.t : a.x) + lcol;
  const int64_t xrs = NI::want_x ? a.x_row_stride : a.t_row_stride;
  const int64_t trs = NI::want_t ? a.t_row_stride : a.x_row_stride;
  const float* wp = static_cast<const float*>(a.w);
  const int mode = a.mse_mode;

  double acc[4][4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[k][e] = 0.0;
  double wsum = 0.0;
  constexpr int64_t kStep = static_cast<int64_t>(RPP) * kU2;
  int64_t i = r0 + rl;
  if (active && i < r1) {
    if constexpr (PIPE) {
      // two batches in flight: the next batch's loads are issued before this one is consumed
      V2Batch<NEED, HAS_W> b0, b1;
      b0.load(xp, tp, wp, xrs, trs, a.w_stride, i, r1, RPP);
      for (;;) {
        const int64_t i1 = i + kStep;
        if (i1 < r1) b1.load(xp, tp, wp, xrs, trs, a.w_stride, i1, r1, RPP);
        b0.accumulate(acc, wsum, i, r1, RPP);
        if (i1 >= r1) break;
        const int64_t i2 = i1 + kStep;
        if (i2 < r1) b0.load(xp, tp, wp, xrs, trs, a.w_stride, i2, r1, RPP);
        b1.accumulate(acc, wsum, i1, r1, RPP);
        if (i2 >= r1) break;
        i = i2;
      }
    } else {
      for (; i < r1; i += kStep) {
        V2Batch<NEED, HAS_W> b;
        b.load(xp, tp, wp, xrs, trs, a.w_stride, i, r1, RPP);
        b.accumulate(acc, wsum, i, r1, RPP);
      }
    }
  }
  // row lanes -> LDS at the columns' tile positions (the tail group's first sh lanes are
  // copies of the previous group's columns: dropped; its last positions are past d: zero)
  __shared__ double lds[NS][RPP][TC];
  __shared__ double lds_w[RPP];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bool keep = active && e >= sh;
    const int pos = cg * 4 + (e >= sh ? e - sh : 4 - sh + e);
    int s = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool on = k == 0 ? NI::sse : k == 1 ? NI::st : k == 2 ? NI::stt : NI::sx;
      if (on) {
        lds[s][rl][pos] = keep ? acc[k][e] : 0.0;
        ++s;
      }
    }
  }
  if (HAS_W && cg == 0) lds_w[rl] = wsum;  // one column group counts each row's weight once
  __syncthreads();
  const V2Layout L{static_cast<int64_t>(gridDim.y), TC};
  double* wpart = a.part + L.wpart(NS, R);
  double* tsc = a.part + L.tscal(NS, R);
  if (mode == 2) {
    // MSE uniform average = sum_j sse_j / (d * clamp(sw)): a block hands on only its sse summed
    // over its columns (and its weight total); ONE ticket over the whole grid
    __shared__ double s_red[kB];
    double v = 0.0;
    for (int c = threadIdx.x; c < TC; c += kB)
      if (tbase + c < d)
#pragma unroll
        for (int r = 0; r < RPP; ++r) v += lds[NI::s_sse][r][c];
    s_red[threadIdx.x] = v;
    __syncthreads();
    for (int h = kB / 2; h >= 1; h >>= 1) {
      if (threadIdx.x < h) s_red[threadIdx.x] += s_red[threadIdx.x + h];
      __syncthreads();
    }
    const int64_t b = static_cast<int64_t>(tile) * R + rc;
    if (threadIdx.x == 0) {
      wt_store(tsc + 2 * b, s_red[0]);
      double w = 0.0;
      if (HAS_W)
        for (int r = 0; r < RPP; ++r) w += lds_w[r];
      wt_store(tsc + 2 * b + 1, w);
    }
    const unsigned nb = static_cast<unsigned>(R) * gridDim.y;
    if (!wt_arrive_last(a.tickets + gridDim.y, nb)) return;
    __shared__ double s_fin[2][kB];
    double s = 0.0, w = 0.0;
    for (unsigned q = threadIdx.x; q < nb; q += kB) {  // fixed partition + fixed tree: deterministic
      s += wt_load(tsc + 2 * q);
      w += wt_load(tsc + 2 * q + 1);
    }
    s_fin[0][threadIdx.x] = s;
    s_fin[1][threadIdx.x] = w;
    __syncthreads();
    for (int h = kB / 2; h >= 1; h >>= 1) {
      if (threadIdx.x < h) {
        s_fin[0][threadIdx.x] += s_fin[0][threadIdx.x + h];
        s_fin[1][threadIdx.x] += s_fin[1][threadIdx.x + h];
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      // every tile's blocks cover every row: the weight total is tile 0's blocks' sum
      const double w_tot = HAS_W ? 0.0 : static_cast<double>(n);
      double wt = w_tot;
      if (HAS_W) {
        wt = 0.0;
        for (int r = 0; r < R; ++r) wt += wt_load(tsc + 2 * r + 1);
      }
      *a.mse_out = static_cast<float>(s_fin[0][0] / (static_cast<double>(mse_den(wt)) * static_cast<double>(d)));
      if (a.sw) *a.sw = a.overwrite ? static_cast<float>(wt) : *a.sw + static_cast<float>(wt);
    }
    return;
  }
  if (a.pend) {
    // deferred mode: this block owns slot rc of every column of its tile; ADD the partials
    // (tea_common.h pend_add: one no-return atomic per slot, one writer per launch, launches
    // ordered by the stream: deterministic) - no ticket, no fold on the launch's tail
    // (launch_moments_fold runs when a state is read)
    for (int p = threadIdx.x; p < NS * TC; p += kB) {
      const int s = p / TC, c = p % TC;
      if (tbase + c >= d) continue;
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < RPP; ++r) v += lds[s][r][c];
      pend_add(a.pend + (static_cast<int64_t>(rc) * NS + s) * d + tbase + c, v);
    }
    if (tile == 0 && threadIdx.x == 0) {
      double v = 0.0;
      if (HAS_W) {
        for (int r = 0; r < RPP; ++r) v += lds_w[r];
      } else {
        v = static_cast<double>(r1 > r0 ? r1 - r0 : 0);
      }
      pend_add(a.pend + static_cast<int64_t>(a.pend_slots) * NS * d + rc, v);
    }
    return;
  }
  for (int p = threadIdx.x; p < NS * TC; p += kB) {
    const int s = p / TC, c = p % TC;
    if (tbase + c >= d) continue;
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < RPP; ++r) v += lds[s][r][c];
    wt_store(a.part + L.part(tile, s, NS, R, rc) + c, v);
  }
  if (HAS_W && threadIdx.x == 0) {
    double v = 0.0;
    for (int r = 0; r < RPP; ++r) v += lds_w[r];
    wt_store(wpart + static_cast<int64_t>(tile) * R + rc, v);
  }
  if (a.v2_skip_fold) return;  // A/B only (benchmarks/k5_v2_ab.py): the streaming part alone
  if (!wt_arrive_last(a.tickets + tile, static_cast<unsigned>(R))) return;

  // ---- the tile's last block: TP threads per column each sum a strided share of the R
  // partials (all loads of the share in flight), then a fixed-order fold of the TP shares
  __shared__ double s_part[NS][TP][TC];
  __shared__ double s_w[kB];
  {
    const int c = threadIdx.x % TC, q = threadIdx.x / TC;
#pragma unroll
    for (int s = 0; s < NS; ++s)
      s_part[s][q][c] = tbase + c < d ? wt_strided_sum(a.part + L.part(tile, s, NS, R, 0) + c, q, TP, R, TC) : 0.0;
    s_w[threadIdx.x] = HAS_W ? wt_strided_sum(wpart + static_cast<int64_t>(tile) * R, threadIdx.x, kB, R, 1) : 0.0;
  }
  __syncthreads();
  if (HAS_W) {
    for (int h = kB / 2; h >= 1; h >>= 1) {
      if (threadIdx.x < h) s_w[threadIdx.x] += s_w[threadIdx.x + h];
      __syncthreads();
    }
  }
  const double w_tot = HAS_W ? s_w[0] : static_cast<double>(n);
  double tsum[3] = {0.0, 0.0, 0.0};  // this thread's share of the tile's scalar-mode sums
  if (threadIdx.x < TC && tbase + threadIdx.x < d) {
    const int c = threadIdx.x;
    const int64_t cc = tbase + c;
    double v[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      v[s] = 0.0;
#pragma unroll
      for (int q = 0; q < TP; ++q) v[s] += s_part[s][q][c];
    }
    float* outs[4] = {a.sse, a.st, a.stt, a.sx};
    const int slot[4] = {NI::s_sse, NI::s_st, NI::s_stt, NI::s_sx};
    const bool on[4] = {NI::sse, NI::st, NI::stt, NI::sx};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!on[k] || !outs[k]) continue;
      float& o = outs[k][cc * a.out_stride];
      o = a.overwrite ? static_cast<float>(v[slot[k]]) : o + static_cast<float>(v[slot[k]]);
    }
    if (mode == 1) {
      // reference mean_squared_error.py:100-111 in float32: sse / (clamp(|sw|, eps) * sign(sw))
      a.mse_out[cc] = static_cast<float>(v[NI::s_sse]) / mse_den(w_tot);
    } else if (mode >= 3) {
      // reference r2_score.py:_compute in float32: tss = stt - st^2 / n, r2 = 1 - rss / tss
      const float rss = static_cast<float>(v[NI::s_sse]), so = static_cast<float>(v[NI::s_st]);
      const float sso = static_cast<float>(v[NI::s_stt]);
      const float tss = sso - (so * so) / static_cast<float>(a.num_obs);
      const float r2 = 1.f - rss / tss;
      if (mode == 3) {
        a.mse_out[cc] = a.num_regressors != 0 ? adjust_r2(r2, a.num_obs, a.num_regressors) : r2;
      } else {
        tsum[0] = r2;
        tsum[1] = static_cast<double>(r2) * tss;
        tsum[2] = tss;
      }
    }
  }
  if (tile == 0 && threadIdx.x == 0 && a.sw)
    *a.sw = a.overwrite ? static_cast<float>(w_tot) : *a.sw + static_cast<float>(w_tot);
  if (mode != 4 && mode != 5) return;
  // R2 averages: the tile's sums (fixed-order LDS tree) -> the last tile folds all tiles
  __shared__ double s_red3[3][kB];
#pragma unroll
  for (int q = 0; q < 3; ++q) s_red3[q][threadIdx.x] = tsum[q];
  __syncthreads();
  for (int h = kB / 2; h >= 1; h >>= 1) {
    if (threadIdx.x < h)
#pragma unroll
      for (int q = 0; q < 3; ++q) s_red3[q][threadIdx.x] += s_red3[q][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < 3) wt_store(tsc + tile * 4 + threadIdx.x, s_red3[threadIdx.x][0]);
  if (!wt_arrive_last(a.tickets + gridDim.y, gridDim.y)) return;
  if (threadIdx.x == 0) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0;
    for (unsigned t = 0; t < gridDim.y; ++t) {
      s0 += wt_load(tsc + t * 4);
      s1 += wt_load(tsc + t * 4 + 1);
      s2 += wt_load(tsc + t * 4 + 2);
    }
    float r = mode == 5 ? static_cast<float>(s1 / s2) : static_cast<float>(s0 / static_cast<double>(d));
    if (a.num_regressors != 0) r = adjust_r2(r, a.num_obs, a.num_regressors);
    *a.mse_out = r;
  }
}

// deferred-mode fold: thread per column, every slot's loads in flight 8 at a time, slots zeroed
__global__ __launch_bounds__(kB) void moments_pend_fold_kernel(MomentsArgs a, int R) {
  const int64_t d = a.d;
  const int ns = moments_ns(a);  // the binding admits only the sets whose layout this reads
  const int64_t col = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x;
  float* outs[4] = {a.sse, a.st, a.stt, a.sx};
  if (col < d) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (!outs[k]) continue;
      // statistic k sits in slot row k in every instantiation (NEED 1: sse; 7: sse, st, stt;
      // 15: all four)
      double* src = a.pend + static_cast<int64_t>(k) * d + col;
      const int64_t step = static_cast<int64_t>(ns) * d;
      double v = 0.0;
      int r = 0;
      for (; r + 8 <= R; r += 8) {
        double q[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) q[j] = src[(r + j) * step];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v += q[j];
          src[(r + j) * step] = 0.0;
        }
      }
      for (; r < R; ++r) {
        v += src[r * step];
        src[r * step] = 0.0;
      }
      float& o = outs[k][col * a.out_stride];
      o = o + static_cast<float>(v);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double* pw = a.pend + static_cast<int64_t>(a.pend_slots) * ns * d;
    double w = 0.0;
    for (int r = 0; r < R; ++r) {
      w += pw[r];
      pw[r] = 0.0;
    }
    if (a.sw) *a.sw = *a.sw + static_cast<float>(w);
  }
}

template <int CG, int NEED, bool PIPE>
void launch_v2_w(const MomentsArgs& a, dim3 grid, hipStream_t stream) {
  if (a.w) hipLaunchKernelGGL((moments_v2_kernel<CG, NEED, true, PIPE>), grid, dim3(kB), 0, stream, a);
  else hipLaunchKernelGGL((moments_v2_kernel<CG, NEED, false, PIPE>), grid, dim3(kB), 0, stream, a);
}

template <int NEED>
void launch_v2_need(const MomentsArgs& a, dim3 grid, hipStream_t stream) {
  const bool pipe = a.v2_pipe != 0;
  if (a.v2_cg == 4) pipe ? launch_v2_w<4, NEED, true>(a, grid, stream) : launch_v2_w<4, NEED, false>(a, grid, stream);
  else if (a.v2_cg == 16) pipe ? launch_v2_w<16, NEED, true>(a, grid, stream) : launch_v2_w<16, NEED, false>(a, grid, stream);
  else pipe ? launch_v2_w<64, NEED, true>(a, grid, stream) : launch_v2_w<64, NEED, false>(a, grid, stream);
}

int need_of(const MomentsArgs& a) {
  return (a.sse ? 1 : 0) | (a.st ? 2 : 0) | (a.stt ? 4 : 0) | (a.sx ? 8 : 0);
}

int launch_moments_v2(const MomentsArgs& a, hipStream_t stream) {
  const int64_t groups = (a.d + 3) / 4;
  const dim3 grid(static_cast<unsigned>(a.v2_r), static_cast<unsigned>((groups + a.v2_cg - 1) / a.v2_cg));
  switch (need_of(a)) {
    case 1: launch_v2_need<1>(a, grid, stream); break;   // MSE
    case 7: launch_v2_need<7>(a, grid, stream); break;   // R2
    default: launch_v2_need<15>(a, grid, stream); break;  // anything else: every statistic
  }
  return static_cast<int>(hipGetLastError());
}

__device__ __forceinline__ double bce(double x, double t, bool logits) {
  if (logits) {
    // max(x, 0) - x t + log(1 + exp(-|x|))
    const double ax = x < 0 ? -x : x;
    return (x > 0 ? x : 0.0) - x * t + log1p(exp(-ax));
  }
  const double lp = x > 0 ? log(x) : -INFINITY;
  const double lq = x < 1 ? log1p(-x) : -INFINITY;
  // torch clamps each log term at -100
  return -(t * (lp < -100.0 ? -100.0 : lp) + (1.0 - t) * (lq < -100.0 ? -100.0 : lq));
}

// order-preserving u64 key of a double (larger key = larger value)
__device__ __forceinline__ unsigned long long ord_key(double x) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  return (u >> 63) ? ~u : (u | (1ull << 63));
}

__global__ __launch_bounds__(kB) void ne_sums_kernel(NeArgs a) {
  const int r = blockIdx.y;
  double s_ce = 0, s_w = 0, s_pos = 0;
  double mn = INFINITY, mx = -INFINITY;
  bool bad = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x; i < a.n;
       i += static_cast<int64_t>(gridDim.x) * kB) {
    const double x = load_as_f64(a.x, a.x_dt, r * a.x_row_stride + i);
    const double t = load_as_f64(a.t, a.t_dt, r * a.t_row_stride + i);
    const double w = a.w ? load_as_f64(a.w, a.w_dt, r * a.w_row_stride + i) : 1.0;
    // the reference's check is max > 1 or min < 0: NaN passes it
    if (!a.from_logits && (x < 0.0 || x > 1.0)) bad = true;
    mn = fmin(mn, x);
    mx = fmax(mx, x);
    s_ce += w * bce(x, t, a.from_logits != 0);
    s_w += w;
    s_pos += w * t;
  }
  if (bad && a.err) atomicOr(a.err, 1);
  if (a.range && !a.from_logits) {  // one pair of atomics per block
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mn = fmin(mn, __shfl_xor(mn, o, 64));
      mx = fmax(mx, __shfl_xor(mx, o, 64));
    }
    if (lane_id() == 0 && mx >= mn) {
      atomicMax(a.range, ord_key(mx));
      atomicMax(a.range + 1, ~ord_key(mn));
    }
  }
  s_ce = wave_sum(s_ce);
  s_w = wave_sum(s_w);
  s_pos = wave_sum(s_pos);
  __shared__ double lds[3][kB / 64];
  if (lane_id() == 0) {
    lds[0][threadIdx.x >> 6] = s_ce;
    lds[1][threadIdx.x >> 6] = s_pos;
    lds[2][threadIdx.x >> 6] = s_w;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    double tot = 0;
    for (int k = 0; k < kB / 64; ++k) tot += lds[threadIdx.x][k];
    if (a.ordered_ws)  // deterministic: partial per block, folded in block order afterwards
      a.ordered_ws[(static_cast<int64_t>(r) * 3 + threadIdx.x) * gridDim.x + blockIdx.x] = tot;
    else
      atomicAdd(a.out + r * 3 + threadIdx.x, tot);
  }
}

__global__ __launch_bounds__(kB) void ordered_sum_kernel(const double* ws, int64_t nvals, int64_t parts,
                                                         double* out) {
  const int64_t v = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x;
  if (v >= nvals) return;
  double s = 0.0;
  for (int64_t p = 0; p < parts; ++p) s += ws[v * parts + p];
  out[v] += s;
}

}  // namespace

int column_moments_blocks(int64_t n, int64_t d) {
  // row chunks: ~32 rows each (>= 8 per row lane with the U = 4 unroll), at most 256 partials
  // per column so the finalize pass stays one latency round per thread
  int64_t p = (n + 31) / 32;
  if (d < 16) p = (n * d + 2047) / 2048;
  if (p > 256) p = 256;
  if (p < 1) p = 1;
  return static_cast<int>(p);
}

int column_moments_finalize_blocks(int64_t d) { return static_cast<int>((d + kFC - 1) / kFC); }

namespace {
int env_read(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return (e != nullptr && e[0] != '\0') ? std::atoi(e) : dflt;
}
// K5 geometry knobs: read once, or on every call when TORCHEVAL_AMD_AB_DYNAMIC=1 (A/B
// harnesses switch them inside one process)
struct K5Knobs {
  int v2, cg, blocks, maxr, pipe, skip;
  void read() {
    v2 = env_read("TORCHEVAL_AMD_K5_V2", 1);
    cg = env_read("TORCHEVAL_AMD_K5_CG", 0);
    blocks = env_read("TORCHEVAL_AMD_K5_BLOCKS", 0);
    maxr = env_read("TORCHEVAL_AMD_K5_MAXR", 64);
    pipe = env_read("TORCHEVAL_AMD_K5_PIPE", 0);
    skip = env_read("TORCHEVAL_AMD_K5_AB_SKIP_FOLD", 0);
  }
};
const K5Knobs& k5_knobs() {
  static K5Knobs fixed = [] {
    K5Knobs k;
    k.read();
    return k;
  }();
  thread_local K5Knobs live;
  if (std::getenv("TORCHEVAL_AMD_AB_DYNAMIC") == nullptr) return fixed;  // one getenv per call
  live.read();
  return live;
}
}  // namespace

bool column_moments_v2_plan(MomentsArgs& a, int64_t* ws_doubles, int64_t* tickets) {
  a.v2_cg = 0;
  const K5Knobs& kn = k5_knobs();
  if (a.n <= 0 || a.d < 4 || kn.v2 == 0) return false;
  const int need = need_of(a);
  const bool want_x = (need & 9) != 0, want_t = (need & 7) != 0;
  if (need == 0 || (want_x && !a.x) || (want_t && !a.t)) return false;
  auto f32_rows = [](const void* p, DType dt, int64_t cs) { return p == nullptr || (dt == DType::f32 && cs == 1); };
  if (!f32_rows(a.x, a.x_dt, a.x_col_stride) || !f32_rows(a.t, a.t_dt, a.t_col_stride)) return false;
  if (a.w && a.w_dt != DType::f32) return false;
  const int64_t groups = (a.d + 3) / 4;
  int cg = kn.cg;
  // measured (benchmarks/k5_v2_ab.py, profiles/k5_v2_ab_r5.jsonl): 16-group tiles with one
  // block per CU for widths up to 2048, 64-group tiles beyond
  if (cg != 4 && cg != 16 && cg != 64) cg = groups <= 4 ? 4 : groups <= 512 ? 16 : 64;
  const int64_t tiles = (groups + cg - 1) / cg;
  const int rpp = kB / cg;
  const int64_t target = kn.blocks > 0 ? kn.blocks : 256;
  int64_t r = std::max<int64_t>(1, (target + tiles - 1) / tiles);
  r = std::min<int64_t>(r, std::max(1, kn.maxr));
  if (a.pend) r = std::min<int64_t>(r, a.pend_slots);
  r = std::min<int64_t>(r, std::max<int64_t>(1, a.n / (static_cast<int64_t>(rpp) * kU2)));  // >= one unrolled pass each
  const int64_t chunk = (a.n + r - 1) / r;
  r = (a.n + chunk - 1) / chunk;
  if (r > 65535 || tiles > 65535) return false;
  const int ns = need == 1 ? 1 : need == 7 ? 3 : 4;
  a.v2_cg = cg;
  a.v2_pipe = kn.pipe != 0;
  a.v2_skip_fold = kn.skip != 0;
  a.v2_r = static_cast<int>(r);
  a.v2_chunk = chunk;
  // partials [tiles][ns][R][tc], weights [tiles][R], scalars max(4 per tile, 2 per block)
  *ws_doubles = tiles * ns * r * (cg * 4) + tiles * r + std::max<int64_t>(tiles * 4, 2 * tiles * r);
  *tickets = tiles + 1;
  return true;
}

int launch_moments_fold(const MomentsArgs& a, int rows_used, hipStream_t stream) {
  if (a.d <= 0 || rows_used <= 0 || !a.pend) return 0;
  if (rows_used > a.pend_slots) return -2;
  hipLaunchKernelGGL(moments_pend_fold_kernel, dim3(static_cast<unsigned>((a.d + kB - 1) / kB)), dim3(kB), 0, stream,
                     a, rows_used);
  return static_cast<int>(hipGetLastError());
}

int launch_column_moments(const MomentsArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.d <= 0) return 0;
  if (a.pend) {  // deferred mode: accumulate-only updates
    if (!a.v2_cg || a.mse_mode || a.overwrite || a.v2_r > a.pend_slots) return -2;
    return launch_moments_v2(a, stream);
  }
  if (a.v2_cg) {
    if (!a.part || !a.tickets) return -2;
    if (a.mse_mode && (!a.overwrite || !a.sse || !a.mse_out)) return -2;
    if (a.mse_mode >= 3 && (!a.st || !a.stt)) return -2;
    return launch_moments_v2(a, stream);
  }
  const int P = a.ws_blocks;
  const bool vec = (a.x == nullptr || (a.x_dt == DType::f32 && a.x_col_stride == 1 && a.x_row_stride % 4 == 0 &&
                                       reinterpret_cast<uintptr_t>(a.x) % 16 == 0)) &&
                   (a.t == nullptr || (a.t_dt == DType::f32 && a.t_col_stride == 1 && a.t_row_stride % 4 == 0 &&
                                       reinterpret_cast<uintptr_t>(a.t) % 16 == 0)) &&
                   a.d % 4 == 0;
  const int V = vec ? 4 : 1;
  const unsigned ct = static_cast<unsigned>(((a.d + V - 1) / V + kColGroups - 1) / kColGroups);
  if (vec)
    hipLaunchKernelGGL(moments_partial_kernel<4>, dim3(P, ct), dim3(kB), 0, stream, a);
  else
    hipLaunchKernelGGL(moments_partial_kernel<1>, dim3(P, ct), dim3(kB), 0, stream, a);
  if (a.mse_mode == 2) {  // the scalar MSE needs no per-column statistics (sse / sw left unwritten)
    hipLaunchKernelGGL(mse_scalar_kernel, dim3(1), dim3(kB), 0, stream, a.ws, static_cast<int64_t>(P) * ct, a.d,
                       a.mse_out);
    return static_cast<int>(hipGetLastError());
  }
  const unsigned fb = static_cast<unsigned>(column_moments_finalize_blocks(a.d));
  const bool scalar = a.mse_mode == 2 || a.mse_mode == 4 || a.mse_mode == 5;
  if (a.mse_mode && (!a.overwrite || !a.sse || (scalar && !a.mse_part_f))) return -2;
  if (a.mse_mode >= 3 && (!a.st || !a.stt)) return -2;
  hipLaunchKernelGGL(moments_finalize_kernel, dim3(fb), dim3(kB), 0, stream, a, P);
  if (scalar)
    hipLaunchKernelGGL(post_reduce_kernel, dim3(1), dim3(kB), 0, stream, a.mse_part_f, a.mse_part_f + a.d, a.d,
                       a.mse_mode, a.num_obs, a.num_regressors, a.mse_out);
  return static_cast<int>(hipGetLastError());
}

int ne_sums_blocks(int64_t n) {
  int64_t blocks = (n + kB * 16 - 1) / (kB * 16);
  if (blocks > 64) blocks = 64;
  if (blocks < 1) blocks = 1;
  return static_cast<int>(blocks);
}

int launch_ne_sums(const NeArgs& a, hipStream_t stream) {
  if (a.rows <= 0) return 0;
  const int blocks = ne_sums_blocks(a.n);
  hipLaunchKernelGGL(ne_sums_kernel, dim3(static_cast<unsigned>(blocks), static_cast<unsigned>(a.rows)),
                     dim3(kB), 0, stream, a);
  if (a.ordered_ws) return launch_ordered_sum(a.ordered_ws, a.rows * 3, blocks, a.out, stream);
  return static_cast<int>(hipGetLastError());
}

int launch_ordered_sum(const double* ws, int64_t nvals, int64_t parts, double* out, hipStream_t stream) {
  if (nvals <= 0) return 0;
  hipLaunchKernelGGL(ordered_sum_kernel, dim3(static_cast<unsigned>((nvals + kB - 1) / kB)), dim3(kB), 0,
                     stream, ws, nvals, parts, out);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
