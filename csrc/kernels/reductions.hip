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

int launch_column_moments(const MomentsArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.d <= 0) return 0;
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
