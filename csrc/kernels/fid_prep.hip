// FID compute glue around K9b / K9d (metrics/image/fid.py; reference torcheval/metrics/image/
// fid.py:239-262):
//   * cov_finalize: the FP64 symmetric covariance straight from the FP32 K8 states,
//       S[i][j] = ((C[i][j] + C[j][i]) / 2 - n mu_i mu_j) / (n - 1),  mu = colsum / n,
//     one pass per side - replacing the ATen chain .double() / outer / scale / sub / div and
//     frechet_distance's (S + S^T) / 2 (~10 full passes over a 32 MB FP64 matrix at D = 2048);
//   * sym_fill_upper: M[i][j] = M[j][i] above the diagonal, for the triangle-aware
//     L^T S2 L whose block products only fill the lower block triangle;
//   * fid_finish: |mu1 - mu2|^2 + tr S1 + tr S2 - 2 sum sqrt(max(lambda, 0)) from the FP32 state
//     sums, the covariances and the eigenvalues, as the FP32 result - one launch instead of the
//     ~12 small ATen kernels (each ~10-15 us of host time apart) that closed compute().
// Both walk 64 x 64 tiles through an LDS transpose (coalesced both ways).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tea_kernels.h"

namespace tea {
namespace {

constexpr int kPT = 64;
constexpr int kPThreads = 256;

// one workgroup per (tile row bi, tile column bj) pair with bj <= bi: reads tiles (bi, bj) and
// (bj, bi) of C ONCE each (every thread's 16 + 16 loads issued together), stages both through LDS
// transposed, one barrier, writes both tiles of S.  (The first form read each input tile twice
// around three barriers: 31 us per side at D = 2048, ~1.6 TB/s.)
__global__ __launch_bounds__(kPThreads) void cov_finalize_kernel(const float* __restrict__ C, const float* __restrict__ colsum,
                                                                double n, int d, double* __restrict__ S) {
  __shared__ float tt[kPT][kPT + 1];  // tile (bj, bi) transposed: tt[c][r] = C[bj + r][bi + c]
  __shared__ float ut[kPT][kPT + 1];  // tile (bi, bj) transposed: ut[c][r] = C[bi + r][bj + c]
  __shared__ double mu_r[kPT], mu_c[kPT];
  // decode the lower-triangle pair index
  int p = blockIdx.x, bi = 0;
  while (p > bi) {
    p -= bi + 1;
    ++bi;
  }
  const int bj = p;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  constexpr int kRows = kPT / (kPThreads / 64);  // 16 rows a thread
  const double inv_n = 1.0 / n, scale = 1.0 / (n - 1.0);
  if (threadIdx.x < kPT) {
    const int r = kPT * bi + threadIdx.x;
    mu_r[threadIdx.x] = r < d ? static_cast<double>(colsum[r]) * inv_n : 0.0;
  } else if (threadIdx.x < 2 * kPT) {
    const int c = kPT * bj + threadIdx.x - kPT;
    mu_c[threadIdx.x - kPT] = c < d ? static_cast<double>(colsum[c]) * inv_n : 0.0;
  }
  const bool diag = bi == bj;
  float a[kRows], b[kRows];
#pragma unroll
  for (int q = 0; q < kRows; ++q) {
    const int r = ty + q * (kPThreads / 64);
    const int ar = kPT * bi + r, ac = kPT * bj + tx;  // tile (bi, bj)
    const int br = kPT * bj + r, bc = kPT * bi + tx;  // tile (bj, bi)
    a[q] = (ar < d && ac < d) ? C[static_cast<int64_t>(ar) * d + ac] : 0.f;
    b[q] = (!diag && br < d && bc < d) ? C[static_cast<int64_t>(br) * d + bc] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < kRows; ++q) {
    const int r = ty + q * (kPThreads / 64);
    ut[tx][r] = a[q];
    tt[tx][r] = diag ? a[q] : b[q];
  }
  __syncthreads();
  // S tile (bi, bj): C[bi + r][bj + tx] (= a[q]) and C[bj + tx][bi + r] (= tt[r][tx])
#pragma unroll
  for (int q = 0; q < kRows; ++q) {
    const int r = ty + q * (kPThreads / 64);
    const int gr = kPT * bi + r, gc = kPT * bj + tx;
    if (gr < d && gc < d) {
      const double v = (0.5 * (static_cast<double>(a[q]) + static_cast<double>(tt[r][tx])) -
                        n * (mu_r[r] * mu_c[tx])) * scale;  // mu_i mu_j: commutative, so S is exactly symmetric
      S[static_cast<int64_t>(gr) * d + gc] = v;
    }
  }
  if (diag) return;
  // mirror tile (bj, bi): C[bj + r][bi + tx] (= b[q]) and C[bi + tx][bj + r] (= ut[r][tx])
#pragma unroll
  for (int q = 0; q < kRows; ++q) {
    const int r = ty + q * (kPThreads / 64);
    const int gr = kPT * bj + r, gc = kPT * bi + tx;
    if (gr < d && gc < d) {
      const double v = (0.5 * (static_cast<double>(ut[r][tx]) + static_cast<double>(b[q])) -
                        n * (mu_r[tx] * mu_c[r])) * scale;
      S[static_cast<int64_t>(gr) * d + gc] = v;
    }
  }
}

// M[i][j] = M[j][i] for j > i: workgroup per upper tile pair (bi < bj) and per diagonal tile
__global__ __launch_bounds__(kPThreads) void sym_fill_upper_kernel(double* M, int64_t ld, int n) {
  __shared__ double tt[kPT][kPT + 1];
  int p = blockIdx.x, bj = 0;
  while (p > bj) {
    p -= bj + 1;
    ++bj;
  }
  const int bi = p;  // bi <= bj: fill tile (bi, bj) from tile (bj, bi)
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < kPT; r += kPThreads / 64) {
    const int gr = kPT * bj + r, gc = kPT * bi + tx;
    tt[r][tx] = (gr < n && gc < n) ? M[static_cast<int64_t>(gr) * ld + gc] : 0.0;
  }
  __syncthreads();
  for (int r = ty; r < kPT; r += kPThreads / 64) {
    const int gr = kPT * bi + r, gc = kPT * bj + tx;
    if (gr < n && gc < n && gc > gr) M[static_cast<int64_t>(gr) * ld + gc] = tt[tx][r];
  }
}

// one block: FP64 partials per thread, then a fixed-order block tree (deterministic)
__global__ __launch_bounds__(1024) void fid_finish_kernel(const float* __restrict__ sum1, double n1,
                                                         const float* __restrict__ sum2, double n2, int d,
                                                         const double* __restrict__ s1, int64_t ld1,
                                                         const double* __restrict__ s2, int64_t ld2,
                                                         const double* __restrict__ lam, int r, float* out) {
  __shared__ double part[3][16];
  double a = 0.0, t = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < d; i += 1024) {
    const double diff = static_cast<double>(sum1[i]) / n1 - static_cast<double>(sum2[i]) / n2;
    a = fma(diff, diff, a);
    t += s1[static_cast<int64_t>(i) * ld1 + i] + s2[static_cast<int64_t>(i) * ld2 + i];
  }
  for (int i = threadIdx.x; i < r; i += 1024) q += sqrt(fmax(lam[i], 0.0));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    t += __shfl_xor(t, o, 64);
    q += __shfl_xor(q, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    part[0][threadIdx.x >> 6] = a;
    part[1][threadIdx.x >> 6] = t;
    part[2][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double v[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      double x = 0.0;
      for (int w = 0; w < 16; ++w) x += part[k][w];
      v[k] = x;
    }
    out[0] = static_cast<float>(v[0] + v[1] - 2.0 * v[2]);
  }
}

}  // namespace

int launch_fid_finish(const float* sum1, double n1, const float* sum2, double n2, int64_t d, const double* s1,
                      int64_t ld1, const double* s2, int64_t ld2, const double* lam, int64_t r, float* out,
                      hipStream_t stream) {
  hipLaunchKernelGGL(fid_finish_kernel, dim3(1), dim3(1024), 0, stream, sum1, n1, sum2, n2, static_cast<int>(d), s1, ld1,
                     s2, ld2, lam, static_cast<int>(r), out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int launch_cov_finalize(const float* C, const float* colsum, double n, int64_t d, double* S, hipStream_t stream) {
  if (d <= 0) return 0;
  const int64_t nb = (d + kPT - 1) / kPT;
  hipLaunchKernelGGL(cov_finalize_kernel, dim3(static_cast<unsigned>(nb * (nb + 1) / 2)), dim3(kPThreads), 0,
                     stream, C, colsum, n, static_cast<int>(d), S);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int launch_sym_fill_upper(double* M, int64_t ld, int64_t n, hipStream_t stream) {
  if (n <= 1) return 0;
  const int64_t nb = (n + kPT - 1) / kPT;
  hipLaunchKernelGGL(sym_fill_upper_kernel, dim3(static_cast<unsigned>(nb * (nb + 1) / 2)), dim3(kPThreads), 0,
                     stream, M, ld, static_cast<int>(n));
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea
