// K9b A/B (not built into _C.so): round-2's counter-barrier hand-off (write-through payload,
// 8 arrival counters) with the payload read by agent-scope loads (default) or, with
// -DVARIANT_ACQ, by plain loads behind one agent-scope acquire per phase (csrc/bench/k9b_ab.hip).
// K9b: eigenvalues of a symmetric FP64 matrix for the FID compute.
//
// FID's compute needs tr sqrt(S1 S2) = sum sqrt(lambda_i(L^T S2 L)) at D = 2048 (fid.py in the
// reference: torch.linalg.eigvals of the non-symmetric product, reference
// torcheval/metrics/image/fid.py:253-262).  Round 2's path ran rocSOLVER's eigvalsh: ~45 ms at
// D = 2048, and its rocprof breakdown (profiles/rocprof_suite_kernel_stats_r1.csv) is ~7000
// launches of ~5 us (latrd gemv / dot / update kernels, one group per column of the
// Householder reduction) plus the tridiagonal solver: the chip idles between tiny launches.
//
// MI355X design: the whole D x D FP64 matrix lives in LDS across the chip for the whole
// reduction (2048 x 2048 x 8 B = 32 MiB = 256 CUs x 128 KB of their 160 KB), one cooperative
// launch of one workgroup per CU.  Workgroup g owns R consecutive rows; the matrix never goes
// back to HBM.  Householder tridiagonalisation (unblocked, LAPACK sytd2 semantics) with ONE
// grid-wide hand-off per column:
//   phase j publishes p_j = tau_j A v_j for the owned rows (8 B each) and, from the owner of
//   row j+1, that row as updated through step j-1; after the barrier every workgroup holds
//   the full p_j and row j+1, forms w_j = p_j - (tau_j/2)(p_j . v_j) v_j, applies step j to
//   row j+1 itself (so row j+1 is never re-published), derives the next reflector v_{j+1}
//   redundantly, and then ONE LDS pass over its rows both applies A -= v_j w_j^T + w_j v_j^T
//   and accumulates the next p_{j+1} = tau_{j+1} A v_{j+1}.
// Hand-offs follow the guide's write-through form: payload stored with agent-scope
// (write-through) stores into a slot used by exactly one phase, drained, then one relaxed
// counter add per workgroup; consumers poll the counter and read the payload with agent-scope
// loads (L1 bypass), so no acquire fence per phase.  Every spin is bounded: a timed-out
// workgroup raises an abort word that every poller checks, the grid drains, and the host
// falls back to rocSOLVER when the status word is non-zero.
//
// The tridiagonal eigenvalues then come from ``tridiag_eigvals_kernel``: one wave per
// eigenvalue index, 64-point multisection of the Gershgorin interval with Sturm counts
// (LAPACK dstebz's count with pivmin), ~9 rounds to double precision.  Eigenvalues are written
// in ascending order; the caller sums sqrt(max(lambda, 0)).

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "tea_kernels.h"

namespace teav {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxCols = 10;   // columns per thread: n <= 2560
constexpr int kMaxRows = 10;   // rows per workgroup (LDS: R * n * 8 <= 160 KB)
constexpr unsigned kSpinLimit = 1u << 18;
constexpr size_t kCtlBytes = 128 * 9;  // top counter + abort, then one 128-B line per XCD

// every handed-off word is a GLOBAL (address space 1) agent-scope access, never flat
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

__device__ __forceinline__ void st_wt(double* p, double x) {
  __hip_atomic_store((gu64*)p,
                     static_cast<unsigned long long>(__double_as_longlong(x)), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double ld_wt(double* p) {
  return __longlong_as_double(static_cast<long long>(__hip_atomic_load(
      (gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), Ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), Ctrl, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double readlane_f64(double x, int lane) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), lane),
                          __builtin_amdgcn_readlane(__double2loint(x), lane));
}

// Wave64 sum, uniform result: DPP within each 16-lane row (quad swaps, half-row and row
// mirrors: a few cycles per step instead of an LDS-latency ds_bpermute), then the four row
// totals by readlane.
__device__ __forceinline__ double wave_sum(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f64<0x141>(x);  // row_half_mirror
  x += dpp_f64<0x140>(x);  // row_mirror
  return (readlane_f64(x, 15) + readlane_f64(x, 31)) + (readlane_f64(x, 47) + readlane_f64(x, 63));
}

// Block-wide sums of N values; every thread gets the totals.  `scratch` holds kWaves * N
// doubles; callers rotate scratch slots so consecutive reductions need one barrier each.
template <int N>
__device__ __forceinline__ void block_sum(double (&v)[N], double* scratch) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const double s = wave_sum(v[i]);
    if (lane == 0) scratch[wave * N + i] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) s += scratch[w * N + i];
    v[i] = s;
  }
}

// Grid barrier over the write-through payload of this phase.  Returns false when the grid
// aborted (a bounded spin ran out here or in another workgroup).
// Arrivals are spread over 8 counters, one per XCD under the round-robin dispatch (block b
// adds to ctl[32 (b % 8 + 1)], each on its own 128-B line) with a NON-returning add, and the
// pollers sum the 8 counters (8 independent loads per poll): at most 32 same-address adds in a
// row and no second hop through a top-level counter.  (The two-level form - last arriver of
// each group adds to a top counter that everybody polls - took 17.9 ms at D = 2048.)
__device__ __forceinline__ bool grid_arrive_wait(unsigned* ctl_flat, unsigned phase, int* s_flag) {
  gu32* ctl = (gu32*)ctl_flat;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's payload stores are done
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned target = gridDim.x * phase;
    __hip_atomic_fetch_add(&ctl[32u * ((blockIdx.x & 7u) + 1u)], 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (unsigned spins = 0;; ++spins) {
      unsigned sum = 0;
#pragma unroll
      for (unsigned x = 0; x < 8u; ++x)
        sum += __hip_atomic_load(&ctl[32u * (x + 1u)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (sum >= target) break;
      if (__hip_atomic_load(&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
        ok = 0;
        break;
      }
      if (spins > kSpinLimit) {
        __hip_atomic_store(&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
#ifdef VARIANT_ACQ
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // drop this CU's stale L1 lines
#endif
    *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}

struct Reflector {
  double tau, beta, scale, diag;
};

// LAPACK dlarfg on x = a[j+1 .. n): alpha = a[j+1], sigma = sum_{k >= j+2} a[k]^2; also
// broadcasts the diagonal a[j].  v[k] = 1 at k = j+1, a[k] * scale beyond, 0 before.
__device__ __forceinline__ Reflector householder(const double (&a)[kMaxCols], int j, int n,
                                                 double* scratch) {
  double r[3] = {0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < kMaxCols; ++s) {
    const int k = threadIdx.x + s * kThreads;
    const double x = a[s];
    r[0] += (k >= j + 2 && k < n) ? x * x : 0.0;
    r[1] += (k == j + 1) ? x : 0.0;
    r[2] += (k == j) ? x : 0.0;
  }
  block_sum<3>(r, scratch);
  Reflector h;
  const double sigma = r[0], alpha = r[1];
  h.diag = r[2];
  if (sigma == 0.0) {
    h.tau = 0.0;
    h.beta = alpha;
    h.scale = 0.0;
  } else {
    const double mu = sqrt(alpha * alpha + sigma);
    h.beta = alpha >= 0.0 ? -mu : mu;
    h.tau = (h.beta - alpha) / h.beta;
    h.scale = 1.0 / (alpha - h.beta);
  }
  return h;
}

__device__ __forceinline__ void make_v(const double (&a)[kMaxCols], const Reflector& h, int j,
                                       double (&v)[kMaxCols]) {
#pragma unroll
  for (int s = 0; s < kMaxCols; ++s) {
    const int k = threadIdx.x + s * kThreads;
    v[s] = k == j + 1 ? 1.0 : (k >= j + 2 ? a[s] * h.scale : 0.0);
  }
}

// One workgroup per CU; dynamic LDS = R * n doubles (the owned rows).  Slots: pslot[q * ld + i]
// = p_q[i], rslot[q * ld + k] = row q+1 as updated through step q-1.  ctl[0] arrivals,
// ctl[1] abort, ctl[32 (x + 1)] arrival counters (own 128-B lines); zeroed by the launcher.
__global__ __launch_bounds__(kThreads) void tridiag_kernel(const double* __restrict__ A, int n,
                                                           int R, int64_t ld, double* d_out,
                                                           double* e_out, double* pslot,
                                                           double* rslot, unsigned* ctl) {
  extern __shared__ double rows[];
  __shared__ double red[3][kWaves * kMaxRows];
  __shared__ double vw[2][kMaxRows];
  __shared__ int s_flag;

  const int t = threadIdx.x;
  const int row0 = blockIdx.x * R;
  const int nrows = min(R, n - row0);
  for (int idx = t; idx < nrows * n; idx += kThreads) rows[idx] = A[(int64_t)row0 * n + idx];

  double a[kMaxCols], v[kMaxCols], w[kMaxCols], vn[kMaxCols];
#pragma unroll
  for (int s = 0; s < kMaxCols; ++s) {
    const int k = t + s * kThreads;
    a[s] = k < n ? A[k] : 0.0;  // row 0
  }
  __syncthreads();

  // ---- phase 0: reflector 0 and p_0 from the original rows
  Reflector h = householder(a, 0, n, red[0]);
  make_v(a, h, 0, v);
  if (blockIdx.x == 0 && t == 0) {
    d_out[0] = h.diag;
    e_out[0] = h.beta;
  }
  {
    double acc[kMaxRows];
#pragma unroll
    for (int r = 0; r < kMaxRows; ++r) {
      acc[r] = 0.0;
      if (r < nrows) {
#pragma unroll
        for (int s = 0; s < kMaxCols; ++s) {
          const int k = t + s * kThreads;
          if (k < n) acc[r] += rows[r * n + k] * v[s];
        }
      }
    }
    block_sum<kMaxRows>(acc, red[2]);
    if (t < nrows && row0 + t >= 1) st_wt(&pslot[row0 + t], h.tau * acc[t]);
    if (1 >= row0 && 1 < row0 + nrows) {
#pragma unroll
      for (int s = 0; s < kMaxCols; ++s) {
        const int k = t + s * kThreads;
        if (k >= 1 && k < n) st_wt(&rslot[k], rows[(1 - row0) * n + k]);
      }
    }
  }
  if (!grid_arrive_wait(ctl, 1u, &s_flag)) return;

  // (Skipping whole dead column slots with wave-uniform branches in the loads and the LDS
  // pass measured slower - 19.4 vs 17.9 ms at D = 2048: the branches split the batched loads.)
  for (int j = 0; j <= n - 3; ++j) {
    // ---- w_j from the gathered p_j; row j+1 updated through step j
    double* ps = pslot + (int64_t)j * ld;
    double* rs = rslot + (int64_t)j * ld;
    double r1[2] = {0.0, 0.0};
#pragma unroll
    for (int s = 0; s < kMaxCols; ++s) {
      const int k = t + s * kThreads;
      const bool act = k >= j + 1 && k < n;
#ifdef VARIANT_ACQ
      const double p = act ? ps[k] : 0.0;  // plain (L2-cacheable) loads behind the acquire
      a[s] = act ? rs[k] : 0.0;
#else
      const double p = act ? ld_wt(ps + k) : 0.0;
      a[s] = act ? ld_wt(rs + k) : 0.0;
#endif
      w[s] = p;
      r1[0] += p * v[s];
      r1[1] += k == j + 1 ? p : 0.0;
    }
    block_sum<2>(r1, red[0]);
    const double c = 0.5 * h.tau * r1[0];
    const double wj1 = r1[1] - c;  // w_j[j+1] (v_j[j+1] = 1)
#pragma unroll
    for (int s = 0; s < kMaxCols; ++s) {
      w[s] -= c * v[s];
      a[s] -= w[s] + wj1 * v[s];  // row j+1 <- row j+1 - v_j[j+1] w_j - w_j[j+1] v_j
      const int k = t + s * kThreads;
      const int r = k - row0;
      if (r >= 0 && r < nrows) {  // the owned rows' v_j[i], w_j[i] for the rank-2 update
        vw[0][r] = v[s];
        vw[1][r] = w[s];
      }
    }

    if (j == n - 3) {
      // last step: row n-2 is final; the owner of row n-1 finishes its diagonal
      if (blockIdx.x == 0) {
#pragma unroll
        for (int s = 0; s < kMaxCols; ++s) {
          const int k = t + s * kThreads;
          if (k == n - 2) d_out[n - 2] = a[s];
          if (k == n - 1) e_out[n - 2] = a[s];
        }
      }
      __syncthreads();
      const int r = (n - 1) - row0;
      if (r >= 0 && r < nrows) {
#pragma unroll
        for (int s = 0; s < kMaxCols; ++s) {
          const int k = t + s * kThreads;
          if (k == n - 1) d_out[n - 1] = rows[r * n + k] - 2.0 * vw[0][r] * vw[1][r];
        }
      }
      break;
    }

    // ---- reflector j+1 (redundant in every workgroup)
    const Reflector hn = householder(a, j + 1, n, red[1]);  // its barrier publishes vw
    make_v(a, hn, j + 1, vn);
    if (blockIdx.x == 0 && t == 0) {
      d_out[j + 1] = hn.diag;
      e_out[j + 1] = hn.beta;
    }

    // ---- one LDS pass: apply step j to the owned rows, accumulate p_{j+1}
    double acc[kMaxRows];
#pragma unroll
    for (int r = 0; r < kMaxRows; ++r) {
      acc[r] = 0.0;
      if (r < nrows && row0 + r >= j + 1) {
        const double vi = vw[0][r], wi = vw[1][r];
#pragma unroll
        for (int s = 0; s < kMaxCols; ++s) {
          const int k = t + s * kThreads;
          if (k >= j + 1 && k < n) {
            const double x = rows[r * n + k] - (vi * w[s] + wi * v[s]);
            rows[r * n + k] = x;
            acc[r] += x * vn[s];
          }
        }
      }
    }
    // the owner of row j+2 (the grid's slowest arriver: 16 KB more to publish) issues the
    // row's stores before the p reduction so they drain behind it; each thread re-reads only
    // the LDS words it wrote itself
    double* pn = pslot + (int64_t)(j + 1) * ld;
    double* rn = rslot + (int64_t)(j + 1) * ld;
    const int ro = (j + 2) - row0;
    if (ro >= 0 && ro < nrows) {
#pragma unroll
      for (int s = 0; s < kMaxCols; ++s) {
        const int k = t + s * kThreads;
        if (k >= j + 2 && k < n) st_wt(&rn[k], rows[ro * n + k]);
      }
    }
    block_sum<kMaxRows>(acc, red[2]);
    if (t < nrows && row0 + t >= j + 2) st_wt(&pn[row0 + t], hn.tau * acc[t]);
#pragma unroll
    for (int s = 0; s < kMaxCols; ++s) v[s] = vn[s];
    h = hn;
    if (!grid_arrive_wait(ctl, (unsigned)(j + 2), &s_flag)) return;
  }
}

// # eigenvalues of the tridiagonal (d, e2 = e^2) below x (LAPACK dstebz's Sturm count).
// (A v_rcp_f64 + Newton reciprocal with two interleaved chains per lane measured 13% slower
// than this plain division at D = 2048: 2.15 vs 1.9 ms.)
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int n, double x,
                                           double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int cnt = q < 0.0;
  for (int k = 1; k < n; ++k) {
    q = d[k] - x - e2[k - 1] / q;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

constexpr int kEigMaxN = 2560;

// One wave per eigenvalue index i (ascending): 64-point multisection of [lo, hi] keeping
// count(a) <= i < count(b).
__global__ __launch_bounds__(kThreads) void tridiag_eigvals_kernel(const double* __restrict__ d_in,
                                                                   const double* __restrict__ e_in,
                                                                   int n, double* lam) {
  __shared__ double d[kEigMaxN], e2[kEigMaxN];
  __shared__ double red[3][kWaves];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double lo = DBL_MAX, hi = -DBL_MAX, emax = 0.0;
  for (int k = t; k < n; k += kThreads) {
    const double dk = d_in[k];
    const double ek = k + 1 < n ? fabs(e_in[k]) : 0.0;
    const double ep = k > 0 ? fabs(e_in[k - 1]) : 0.0;
    d[k] = dk;
    e2[k] = ek * ek;
    lo = fmin(lo, dk - ek - ep);
    hi = fmax(hi, dk + ek + ep);
    emax = fmax(emax, ek * ek);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o, 64));
    hi = fmax(hi, __shfl_xor(hi, o, 64));
    emax = fmax(emax, __shfl_xor(emax, o, 64));
  }
  if (lane == 0) {
    red[0][wave] = lo;
    red[1][wave] = hi;
    red[2][wave] = emax;
  }
  __syncthreads();
  lo = red[0][0];
  hi = red[1][0];
  emax = red[2][0];
  for (int w = 1; w < kWaves; ++w) {
    lo = fmin(lo, red[0][w]);
    hi = fmax(hi, red[1][w]);
    emax = fmax(emax, red[2][w]);
  }
  const double pivmin = DBL_MIN * fmax(1.0, emax);
  const double span = fmax(fabs(lo), fabs(hi));
  // widen so count(lo) = 0 and count(hi) = n hold despite rounding
  double a = lo - 2.0 * DBL_EPSILON * span * n - 2.0 * pivmin;
  double b = hi + 2.0 * DBL_EPSILON * span * n + 2.0 * pivmin;
  const int idx = blockIdx.x * kWaves + wave;
  if (idx >= n) return;  // no block barrier below
  for (int round = 0; round < 14; ++round) {
    const double width = b - a;
    // absolute tolerance eps * ||T|| (the accuracy any backward-stable solver delivers)
    if (width <= DBL_EPSILON * span + 2.0 * DBL_EPSILON * fmax(fabs(a), fabs(b)) + pivmin) break;
    const double x = a + width * (double)(lane + 1) / 65.0;
    const int c = sturm_count(d, e2, n, x, pivmin);
    const unsigned long long above = __ballot(c > idx);
    const int first = above ? __ffsll((long long)above) - 1 : 64;
    const double xa = __shfl(x, first > 0 ? first - 1 : 0, 64);
    const double xb = __shfl(x, first < 64 ? first : 63, 64);
    if (first > 0) a = xa;
    if (first < 64) b = xb;
  }
  if (lane == 0) lam[idx] = 0.5 * (a + b);
}

}  // namespace

int symeig_plan_v(int64_t n, int* grid, int* rows_per_block) {
  if (n < 3 || n > (int64_t)kMaxCols * kThreads || n > kEigMaxN) return 1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 2;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 2;
  int64_t R = (n + cus - 1) / cus;
  if (R > kMaxRows) return 1;
  if (R * n * (int64_t)sizeof(double) > 152 * 1024) return 1;
  *grid = (int)((n + R - 1) / R);
  *rows_per_block = (int)R;
  return 0;
}



int launch_symeig(const tea::SymEigArgs& a, hipStream_t stream) {
  int G = 0, R = 0;
  if (symeig_plan_v(a.n, &G, &R) != 0) return 1;
  const size_t lds = (size_t)R * a.n * sizeof(double);
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(&tridiag_kernel),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return 2;
  if (hipMemsetAsync(a.ctl, 0, kCtlBytes, stream) != hipSuccess) return 2;
  const double* A = a.a;
  int n = (int)a.n;
  int64_t ld = a.ld;
  double *d = a.d, *e = a.e, *ps = reinterpret_cast<double*>(a.gran), *rs = reinterpret_cast<double*>(a.gran) + (a.n - 2) * a.ld;
  unsigned* ctl = a.ctl;
  void* args[] = {&A, &n, &R, &ld, &d, &e, &ps, &rs, &ctl};
  if (hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&tridiag_kernel), dim3(G),
                                 dim3(kThreads), args, lds, stream) != hipSuccess)
    return 3;
  tridiag_eigvals_kernel<<<(n + kWaves - 1) / kWaves, kThreads, 0, stream>>>(d, e, n, a.lam);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea
