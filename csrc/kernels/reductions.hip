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

__global__ __launch_bounds__(kB) void column_moments_kernel(MomentsArgs a) {
  const int D = static_cast<int>(a.d);
  const int Dt = D < kB ? D : kB;           // columns per block pass
  const int rows_per_pass = kB / Dt;        // rows handled together
  const int my_col_in_tile = threadIdx.x % Dt;
  const int my_row_off = threadIdx.x / Dt;
  const bool active = my_row_off < rows_per_pass;
  __shared__ double lds[5][kB];
  __shared__ double s_w[kB];
  for (int c0 = 0; c0 < D; c0 += Dt) {
    const int j = c0 + my_col_in_tile;
    double sse = 0, st = 0, stt = 0, sx = 0, sw = 0;
    if (active && j < D) {
      for (int64_t i = static_cast<int64_t>(blockIdx.x) * rows_per_pass + my_row_off; i < a.n;
           i += static_cast<int64_t>(gridDim.x) * rows_per_pass) {
        const double x = a.x ? load_as_f64(a.x, a.x_dt, i * a.x_row_stride + j * a.x_col_stride) : 0.0;
        const double t = a.t ? load_as_f64(a.t, a.t_dt, i * a.t_row_stride + j * a.t_col_stride) : 0.0;
        const double w = a.w ? load_as_f64(a.w, a.w_dt, i * a.w_stride) : 1.0;
        const double r = t - x;
        sse += w * r * r;
        st += w * t;
        stt += w * t * t;
        sx += w * x;
        sw += w;
      }
    }
    lds[0][threadIdx.x] = sse;
    lds[1][threadIdx.x] = st;
    lds[2][threadIdx.x] = stt;
    lds[3][threadIdx.x] = sx;
    s_w[threadIdx.x] = (j == c0) ? sw : 0.0;  // count weights once (column c0 threads)
    __syncthreads();
    if (threadIdx.x < Dt && c0 + threadIdx.x < D) {
      double acc[4] = {0, 0, 0, 0};
      for (int r = 0; r < rows_per_pass; ++r) {
        const int src = r * Dt + threadIdx.x;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] += lds[k][src];
      }
      const int jj = c0 + threadIdx.x;
      if (a.sse && acc[0] != 0.0) atomicAdd(a.sse + jj * a.out_stride, static_cast<float>(acc[0]));
      if (a.st && acc[1] != 0.0) atomicAdd(a.st + jj * a.out_stride, static_cast<float>(acc[1]));
      if (a.stt && acc[2] != 0.0) atomicAdd(a.stt + jj * a.out_stride, static_cast<float>(acc[2]));
      if (a.sx && acc[3] != 0.0) atomicAdd(a.sx + jj * a.out_stride, static_cast<float>(acc[3]));
    }
    if (c0 == 0 && a.sw) {
      // reduce the weight sum over the whole block
      double v = s_w[threadIdx.x];
      v = wave_sum(v);
      __shared__ double s_ws[kB / 64];
      if (lane_id() == 0) s_ws[threadIdx.x >> 6] = v;
      __syncthreads();
      if (threadIdx.x == 0) {
        double tot = 0;
        for (int k = 0; k < kB / 64; ++k) tot += s_ws[k];
        if (tot != 0.0) atomicAdd(a.sw, static_cast<float>(tot));
      }
    }
    __syncthreads();
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

__global__ __launch_bounds__(kB) void ne_sums_kernel(NeArgs a) {
  const int r = blockIdx.y;
  double s_ce = 0, s_w = 0, s_pos = 0;
  bool bad = false;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kB + threadIdx.x; i < a.n;
       i += static_cast<int64_t>(gridDim.x) * kB) {
    const double x = load_as_f64(a.x, a.x_dt, r * a.x_row_stride + i);
    const double t = load_as_f64(a.t, a.t_dt, r * a.t_row_stride + i);
    const double w = a.w ? load_as_f64(a.w, a.w_dt, r * a.w_row_stride + i) : 1.0;
    if (!a.from_logits && !(x >= 0.0 && x <= 1.0)) bad = true;
    s_ce += w * bce(x, t, a.from_logits != 0);
    s_w += w;
    s_pos += w * t;
  }
  if (bad && a.err) atomicOr(a.err, 1);
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
    atomicAdd(a.out + r * 3 + threadIdx.x, tot);
  }
}

}  // namespace

int launch_column_moments(const MomentsArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.d <= 0) return 0;
  const int Dt = a.d < kB ? static_cast<int>(a.d) : kB;
  const int rows_per_pass = kB / Dt;
  int64_t blocks = (a.n + rows_per_pass * 16 - 1) / (rows_per_pass * 16);
  const int64_t cap = a.d == 1 ? 64 : 256;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(column_moments_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kB), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

int launch_ne_sums(const NeArgs& a, hipStream_t stream) {
  if (a.rows <= 0) return 0;
  int64_t blocks = (a.n + kB * 16 - 1) / (kB * 16);
  if (blocks > 64) blocks = 64;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ne_sums_kernel, dim3(static_cast<unsigned>(blocks), static_cast<unsigned>(a.rows)),
                     dim3(kB), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
