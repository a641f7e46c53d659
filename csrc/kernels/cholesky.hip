// K9d: the whole blocked FP64 Cholesky of FID's covariance in ONE persistent launch.
//
// FID compute factors S1 = L L^T (metrics/image/fid.py; reference torcheval/metrics/image/
// fid.py:192-230 takes linalg.eigvals of S1 S2 instead).  Round 5's K9c factored the 32
// diagonal 64 x 64 blocks of D = 2048 one launch each (37 us per block, a barrier per column)
// with three library launches per block in between from a Python loop: 1.75 ms
// (profiles/symeig_timing_final_r5.json).  Here the factorisation is a dataflow over 64 x 64
// tiles in one launch:
//
//   * tasks, in ticket order (a global counter; a task only ever waits on tasks with lower
//     tickets, which running workgroups hold, so the grid cannot deadlock whatever the dispatch
//     order):  for each tile column c:  D_c, then T(i, c) for i >= c + 2.
//       D_c ("pair owner") owns tiles (c, c) and (c, c-1): it subtracts every L(c,k) L(c,k)^T
//       and L(c,k) L(c-1,k)^T (k <= c-2) as those tiles appear, then - the critical chain -
//       takes inv(L(c-1,c-1)) from D_{c-1}, forms L(c,c-1) = Z inv^T, subtracts its own
//       L(c,c-1) L(c,c-1)^T and factors (c, c): ONE cross-CU hand-off per tile column.
//       T(i, c) (left-looking) accumulates A(i,c) - sum_k L(i,k) L(c,k)^T and multiplies by
//       inv(L(c,c))^T.
//   * tile products on FP64 MFMA (v_mfma_f64_16x16x4_f64): wave w owns output columns
//     16w..16w+15 (four 16 x 16 C blocks), operands staged row-major in LDS (68-double rows).
//   * the diagonal factorisation: wave 0 holds row i of the tile in lane i (64 doubles) and
//     eliminates column by column; each column is broadcast through an LDS ring slot (written
//     once, no barrier), and wave 1, trailing it through an LDS flag, applies the same
//     eliminations to the identity with column c of the inverse in lane c - so the inverse
//     costs no extra broadcast and no barrier per column (K9c: 16 x 16 threads, one barrier per
//     column, 37 us).
//   * hand-offs: every published double is ONE agent-scope (write-through) 8-byte store into a
//     buffer the launcher fills with all-one bytes; consumers poll with agent-scope loads until
//     no value is the sentinel (the data is the flag, as K9b's slots: symeig.hip).  NaN is
//     canonicalised on the way out, so no published value is the sentinel.  Spins are bounded:
//     a timed-out poll raises the abort word and the host falls back to the library.
//
// Output: the padded N x N factor (N = 64 * ceil(n / 64); identity-padded input, so the
// padding factors to the identity), upper triangle zero; status[0] = LAPACK info (first
// non-positive pivot column + 1), status[1] = abort.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tea_kernels.h"

namespace tea {
namespace {

constexpr int kTB = 64;        // tile
constexpr int kLd = 68;        // LDS row stride (doubles): conflict-free MFMA fragment reads
constexpr int kCT = 256;       // threads per workgroup (4 waves)
constexpr unsigned kChSpin = 1u << 22;

typedef __attribute__((address_space(1))) unsigned long long cg_u64;
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr unsigned long long kSent = ~0ull;

__device__ __forceinline__ void cput(double* p, double x) {
  const unsigned long long b =
      x != x ? 0x7ff8000000000000ull : static_cast<unsigned long long>(__double_as_longlong(x));
  __hip_atomic_store((cg_u64*)(reinterpret_cast<unsigned long long*>(p)), b, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long cget(const double* p) {
  return __hip_atomic_load((cg_u64*)(reinterpret_cast<unsigned long long*>(const_cast<double*>(p))),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct ChArgs {
  const double* A;  // input, lower triangle read
  int64_t lda;
  int n;
  int nt;           // tiles per side
  int64_t ldl;      // = 64 * nt
  double* L;        // padded factor, sentinel-filled
  double* Linv;     // nt x 64 x 64 inverses of the diagonal tiles, sentinel-filled
  int* ctl;         // [0] ticket counter (zeroed)
  int* status;      // [0] info, [1] abort (zeroed)
  int ntasks;
  unsigned long long* trace;  // optional: [nt][8] s_memrealtime stamps of the D_c phases
};

// phase stamps of pair owner c (thread 0): 0 start, 1 updates done, 2 inverse arrived,
// 3 L(c, c-1) published, 4 own update done, 5 factored, 6 published, 7 unused
#define CH_TRACE(c, k)                                                              \
  do {                                                                              \
    if (a.trace != nullptr && threadIdx.x == 0) a.trace[(c) * 8 + (k)] = wall_clock64(); \
  } while (0)

// Poll-load a published 64 x 64 tile (row stride ld) into LDS.  Every round issues all 16 loads
// of the thread at once (re-polling one value at a time costs one memory round trip per value
// that was still the sentinel at the first look: ~16 serial round trips per hand-off).
__device__ __forceinline__ void load_tile(const ChArgs& a, const double* g, int64_t ld, double (*s)[kLd]) {
  const int t = threadIdx.x;
  unsigned long long v[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int idx = e * kCT + t;
    v[e] = cget(g + (idx >> 6) * ld + (idx & 63));
  }
  unsigned spins = 0;
  for (;;) {
    bool miss = false;
#pragma unroll
    for (int e = 0; e < 16; ++e) miss |= v[e] == kSent;
    if (!miss) break;
    if (++spins > kChSpin) {
      a.status[1] = 1;  // abort: the host falls back (the values below are then garbage)
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int idx = e * kCT + t;
      if (v[e] == kSent) v[e] = cget(g + (idx >> 6) * ld + (idx & 63));
    }
  }
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int idx = e * kCT + t;
    s[idx >> 6][idx & 63] = __longlong_as_double(static_cast<long long>(v[e]));
  }
}

// Input tile (ti, tj) of A into the C layout of the wave's column stripe (identity padding).
__device__ __forceinline__ void load_input(const ChArgs& a, int ti, int tj, f64x4 (&acc)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = kTB * tj + 16 * w + (lane & 15);
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = kTB * ti + 16 * mb + (lane >> 4) + 4 * rr;
      acc[mb][rr] = (row < a.n && col < a.n) ? a.A[static_cast<int64_t>(row) * a.lda + col]
                                              : (row == col ? 1.0 : 0.0);
    }
}

// acc (+/-)= X Y^T over k = 0..63; X, Y row-major [64][kLd] in LDS.
template <bool NEG>
__device__ __forceinline__ void tile_mma(f64x4 (&acc)[4], const double (*X)[kLd], const double (*Y)[kLd]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < 16; ++ks) {
    const int k = 4 * ks + kq;
    double b = Y[16 * w + r][k];
    if (NEG) b = -b;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const double x = X[16 * mb + r][k];
      acc[mb] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, b, acc[mb], 0, 0, 0);
    }
    if ((ks & 3) == 3) asm volatile("" ::: "memory");  // bound the hoisted fragment reads
  }
}

__device__ __forceinline__ void acc_to_lds(const f64x4 (&acc)[4], double (*s)[kLd]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s[16 * mb + (lane >> 4) + 4 * rr][16 * w + (lane & 15)] = acc[mb][rr];
}

__device__ __forceinline__ void acc_publish(const ChArgs& a, const f64x4 (&acc)[4], int ti, int tj) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* g = a.L + static_cast<int64_t>(kTB * ti) * a.ldl + kTB * tj;
#pragma unroll
  for (int mb = 0; mb < 4; ++mb)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      cput(g + static_cast<int64_t>(16 * mb + (lane >> 4) + 4 * rr) * a.ldl + 16 * w + (lane & 15), acc[mb][rr]);
}

// plain zero stores of the (never polled) upper tile (ti, tj), tj > ti
__device__ __forceinline__ void zero_tile(const ChArgs& a, int ti, int tj) {
  double* g = a.L + static_cast<int64_t>(kTB * ti) * a.ldl + kTB * tj;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int idx = e * kCT + threadIdx.x;
    g[static_cast<int64_t>(idx >> 6) * a.ldl + (idx & 63)] = 0.0;
  }
}

__device__ __forceinline__ double bcast(double x, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), lane);
  return __hiloint2double(hi, lo);
}

struct alignas(16) PotrfLds {
  double col[kTB + 2][kTB];  // column j of the elimination (unscaled), slot j: written once (two
                             // spare rows: the windows below read up to 64 values past slot j)
  double rs[kTB], rd[kTB];
  int flag;                  // columns published by wave 0
};

__shared__ double sA[kTB][kLd];
__shared__ double sB[kTB][kLd];
__shared__ double sC[kTB][kLd];
__shared__ PotrfLds pl;

// The diagonal tile is factored by two waves with runtime column loops over a SHIFTING register
// window: slot m of a lane's window holds column j + m at step j, every FMA writes its result one
// slot down (r[m] <- r[m + 1] - u col[j + 1 + m]), so the pivot is always slot 0 and every
// register index stays a compile-time constant without unrolling the 64 columns.  The window
// narrows in four phases of 16 columns (64, 48, 32, 16 slots: 2496 FMAs per lane instead of the
// triangle's 2016).  Fully unrolled column loops (round 6's first K9d, and K9c before it) ran
// ~160 KB of straight-line code per tile and were instruction-fetch bound: ~900 cycles per
// column, 24.8 us per tile (profiles/k9d_trace_r6.json).
//
// wave 0: lane i = row i of L; each column is published to the LDS ring (unscaled) with its
// 1/sqrt(d) and 1/d, and its finished L entries go straight to Z (= sA) column j.
// r[m] <- r[m + 1] - u c[m] for m < W - 1, r[W - 1] <- 0: the window shift of one elimination
// step.  The column is read in 16-value chunks, each chunk's reads issued one chunk ahead of its
// FMAs behind a compiler memory fence (unfenced, the compiler hoists all W reads and spills).
template <int W>
__device__ __forceinline__ void shift_elim(double (&r)[kTB], const double* c, double u) {
  constexpr int kC = 16;
  constexpr int NC = (W - 1 + kC - 1) / kC;
  double v[2][kC];
#pragma unroll
  for (int q = 0; q < kC; ++q) v[0][q] = q < W - 1 ? c[q] : 0.0;
#pragma unroll
  for (int ch = 0; ch < NC; ++ch) {
    if (ch + 1 < NC) {
#pragma unroll
      for (int q = 0; q < kC; ++q) {
        const int m = (ch + 1) * kC + q;
        v[(ch + 1) & 1][q] = m < W - 1 ? c[m] : 0.0;
      }
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int q = 0; q < kC; ++q) {
      const int m = ch * kC + q;
      if (m < W - 1) r[m] = fma(-u, v[ch & 1][q], r[m + 1]);
    }
  }
  r[W - 1] = 0.0;
}

template <int W>
__device__ __forceinline__ void l_phase(double (&r)[kTB], int j0, int& fb, double (*Z)[kLd], PotrfLds& p,
                                        unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  for (int j = j0; j < j0 + 16; ++j) {
    if (cyc != nullptr && lane == 0) cyc[j] = clock64();
    double d = bcast(r[0], j);
    fb = (fb < 0 && !(d > 0.0)) ? j : fb;
    d = fb >= 0 ? 1.0 : d;  // keep every later value finite; the caller discards the factor
    const double aij = r[0];
    p.col[j][lane] = lane > j ? aij : 0.0;
    double rs = __builtin_amdgcn_rsq(d);
    rs = fma(0.5 * rs, fma(-d * rs, rs, 1.0), rs);
    rs = fma(0.5 * rs, fma(-d * rs, rs, 1.0), rs);
    const double rd = rs * rs;
    if (lane == 0) {
      p.rs[j] = rs;
      p.rd[j] = rd;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the column is in LDS before the flag
    if (lane == 0) __hip_atomic_store(&p.flag, j + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    const double u = lane > j ? aij * rd : 0.0;
    Z[lane][j] = lane > j ? aij * rs : (lane == j ? d * rs : 0.0);
    shift_elim<W>(r, &p.col[j][j + 1], u);
  }
}

// wave 1: lane c = column c of inv(L), trailing wave 0 through the flag; x[m] holds row j + m
template <int W>
__device__ __forceinline__ void x_phase(double (&x)[kTB], int j0, int* status, double (*X)[kLd], PotrfLds& p,
                                        unsigned long long* cyc) {
  const int lane = threadIdx.x & 63;
  for (int j = j0; j < j0 + 16; ++j) {
    if (cyc != nullptr && lane == 0) cyc[j] = clock64();
    unsigned spins = 0;
    while (__hip_atomic_load(&p.flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= j) {
      if (++spins > kChSpin) {
        status[1] = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const double u = x[0] * p.rd[j];
    X[j][lane] = x[0] * p.rs[j];
    shift_elim<W>(x, &p.col[j][j + 1], u);
  }
}

// Factor the symmetric tile in sA (row-major, full) in place: on return sA holds L (zero above
// the diagonal) and sC holds inv(L).  Waves 0 and 1 only (the caller barriers).
__device__ __noinline__ void potrf_tile(int* status, int c, unsigned long long* trace, int nt8) {
  double (*Z)[kLd] = sA;
  double (*X)[kLd] = sC;
  PotrfLds& p = pl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w == 0) {
    double r[kTB];
#pragma unroll
    for (int k = 0; k < kTB; k += 2) {
      const double2 v = *reinterpret_cast<const double2*>(&Z[lane][k]);
      r[k] = v.x;
      r[k + 1] = v.y;
    }
    int fb = -1;  // first non-positive (or NaN) pivot: LAPACK info - 1
    // profiling hook: shader-clock stamps of every column of tile column 1 (trace[nt*8 ...])
    unsigned long long* cyc = (trace != nullptr && c == 1) ? trace + nt8 : nullptr;
    l_phase<64>(r, 0, fb, Z, p, cyc);
    l_phase<48>(r, 16, fb, Z, p, cyc);
    l_phase<32>(r, 32, fb, Z, p, cyc);
    l_phase<16>(r, 48, fb, Z, p, cyc);
    if (cyc != nullptr && lane == 0) cyc[64] = clock64();
    if (lane == 0 && fb >= 0) atomicCAS(status, 0, kTB * c + fb + 1);
    if (trace != nullptr && lane == 0) trace[c * 8 + 7] = wall_clock64();  // wave 0's eliminations done
  } else if (w == 1) {
    double x[kTB];  // column `lane` of the inverse, window from row j
#pragma unroll
    for (int k = 0; k < kTB; ++k) x[k] = k == lane ? 1.0 : 0.0;
    unsigned long long* cyc = (trace != nullptr && c == 1) ? trace + nt8 + 65 : nullptr;
    x_phase<64>(x, 0, status, X, p, cyc);
    x_phase<48>(x, 16, status, X, p, cyc);
    x_phase<32>(x, 32, status, X, p, cyc);
    x_phase<16>(x, 48, status, X, p, cyc);
    if (cyc != nullptr && lane == 0) cyc[64] = clock64();
  }
}

__global__ __launch_bounds__(kCT, 1) void cholesky_kernel(ChArgs a) {
  __shared__ int s_task;
  const int t = threadIdx.x;
  for (;;) {
    if (t == 0) s_task = atomicAdd(a.ctl, 1);
    __syncthreads();
    int task = s_task;
    __syncthreads();
    if (task >= a.ntasks) return;
    int c = 0;
    for (;;) {  // column c has 1 + max(0, nt - c - 2) tasks
      const int cnt = 1 + (a.nt - c - 2 > 0 ? a.nt - c - 2 : 0);
      if (task < cnt) break;
      task -= cnt;
      ++c;
    }
    f64x4 acc[4];
    if (task == 0) {
      // ---- D_c: tiles (c, c) and (c, c-1)
      f64x4 accs[4];
      CH_TRACE(c, 0);
      load_input(a, c, c, acc);
      if (c >= 1) load_input(a, c, c - 1, accs);
      for (int k = 0; k + 2 <= c; ++k) {
        load_tile(a, a.L + static_cast<int64_t>(kTB * c) * a.ldl + kTB * k, a.ldl, sA);
        load_tile(a, a.L + static_cast<int64_t>(kTB * (c - 1)) * a.ldl + kTB * k, a.ldl, sB);
        __syncthreads();
        tile_mma<true>(acc, sA, sA);
        tile_mma<true>(accs, sA, sB);
        __syncthreads();
      }
      CH_TRACE(c, 1);
      if (c >= 1) {
        // the critical hand-off: inv(L(c-1, c-1)) from D_{c-1}
        load_tile(a, a.Linv + static_cast<int64_t>(c - 1) * kTB * kTB, kTB, sB);
        acc_to_lds(accs, sA);
        __syncthreads();
        CH_TRACE(c, 2);
        f64x4 r[4];
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) r[mb] = f64x4{0.0, 0.0, 0.0, 0.0};
        tile_mma<false>(r, sA, sB);  // L(c, c-1) = Z inv(L(c-1,c-1))^T
        acc_publish(a, r, c, c - 1);
        CH_TRACE(c, 3);
        __syncthreads();
        acc_to_lds(r, sA);
        __syncthreads();
        tile_mma<true>(acc, sA, sA);
        zero_tile(a, c - 1, c);
        __syncthreads();
        CH_TRACE(c, 4);
      }
      acc_to_lds(acc, sA);
      if (t == 0) pl.flag = 0;
      __syncthreads();
      potrf_tile(a.status, c, a.trace, a.nt * 8);
      __syncthreads();
      CH_TRACE(c, 5);
      // publish L(c, c) (zero above the diagonal) and its inverse, coalesced
      double* gl = a.L + static_cast<int64_t>(kTB * c) * a.ldl + kTB * c;
      double* gi = a.Linv + static_cast<int64_t>(c) * kTB * kTB;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int idx = e * kCT + t;
        cput(gi + idx, sC[idx >> 6][idx & 63]);
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int idx = e * kCT + t;
        cput(gl + static_cast<int64_t>(idx >> 6) * a.ldl + (idx & 63), sA[idx >> 6][idx & 63]);
      }
      __syncthreads();
      CH_TRACE(c, 6);
    } else {
      // ---- T(i, c), i >= c + 2
      const int i = c + 1 + task;
      load_input(a, i, c, acc);
      for (int k = 0; k < c; ++k) {
        load_tile(a, a.L + static_cast<int64_t>(kTB * i) * a.ldl + kTB * k, a.ldl, sA);
        load_tile(a, a.L + static_cast<int64_t>(kTB * c) * a.ldl + kTB * k, a.ldl, sB);
        __syncthreads();
        tile_mma<true>(acc, sA, sB);
        __syncthreads();
      }
      load_tile(a, a.Linv + static_cast<int64_t>(c) * kTB * kTB, kTB, sB);
      acc_to_lds(acc, sA);
      __syncthreads();
      f64x4 r[4];
#pragma unroll
      for (int mb = 0; mb < 4; ++mb) r[mb] = f64x4{0.0, 0.0, 0.0, 0.0};
      tile_mma<false>(r, sA, sB);
      acc_publish(a, r, i, c);
      zero_tile(a, c, i);
      __syncthreads();
    }
  }
}

}  // namespace

int cholesky_tiles(int64_t n) { return static_cast<int>((n + kTB - 1) / kTB); }

int launch_cholesky(const double* A, int64_t lda, int64_t n, double* L, double* Linv, int* ctl, int* status,
                    hipStream_t stream, unsigned long long* trace) {
  if (n < 1 || n > 16384) return 1;
  const int nt = cholesky_tiles(n);
  ChArgs a;
  a.A = A;
  a.lda = lda;
  a.n = static_cast<int>(n);
  a.nt = nt;
  a.ldl = static_cast<int64_t>(kTB) * nt;
  a.L = L;
  a.Linv = Linv;
  a.ctl = ctl;
  a.status = status;
  a.trace = trace;
  int tasks = 0;
  for (int c = 0; c < nt; ++c) tasks += 1 + (nt - c - 2 > 0 ? nt - c - 2 : 0);
  a.ntasks = tasks;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    return 2;
  const size_t lbytes = static_cast<size_t>(a.ldl) * a.ldl * sizeof(double);
  if (hipMemsetAsync(L, 0xff, lbytes, stream) != hipSuccess) return 2;
  if (hipMemsetAsync(Linv, 0xff, static_cast<size_t>(nt) * kTB * kTB * sizeof(double), stream) != hipSuccess)
    return 2;
  if (hipMemsetAsync(ctl, 0, sizeof(int), stream) != hipSuccess) return 2;
  if (hipMemsetAsync(status, 0, 2 * sizeof(int), stream) != hipSuccess) return 2;
  const int grid = tasks < cus ? tasks : cus;
  hipLaunchKernelGGL(cholesky_kernel, dim3(grid), dim3(kCT), 0, stream, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea
