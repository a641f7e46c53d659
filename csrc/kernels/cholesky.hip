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
#include <cstdlib>

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
  int exp;                    // A/B probe (TORCHEVAL_AMD_K9D_PROBE, results invalid when set):
                              // 1 skip the window updates, 2 skip the inverse's wave, 8 skip the
                              // diagonal factorisation
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

constexpr int kPB = 4;  // columns per elimination step of the diagonal-tile factorisation

struct alignas(16) PotrfLds {
  double col[kTB + 4][kTB];  // column j of L below the step's 4 x 4 pivot block (by row), slot j
                             // written once; four spare rows for the reads past the last column
  double piv[kTB / kPB][16]; // per step: L44 (l00, l10, l11, l20, l21, l22, l30, l31, l32, l33)
                             // and 1 / l_qq (q = 0..3) for the inverse's wave
  double g[kPB][kPB];        // the step's pivot block rows, gathered by their lanes
  int flag;                  // columns published by wave 0
};

__shared__ double sA[kTB][kLd];
__shared__ double sB[kTB][kLd];
__shared__ double sC[kTB][kLd];
__shared__ PotrfLds pl;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Two consecutive doubles of LDS (8-byte aligned; a broadcast read when every lane passes the same
// address), by inline asm so that a chunk's reads are all in flight together; the caller waits
// explicitly.  (Compiler-scheduled, such reads ran two in flight with a full LDS round trip per
// pair, csrc/bench/fp64_rates.hip.)
__device__ __forceinline__ u32x4 lds_2x64(unsigned addr) {
  u32x4 v;
  asm volatile("ds_read2_b64 %0, %1 offset1:1" : "=v"(v) : "v"(addr) : "memory");
  return v;
}

__device__ __forceinline__ double lo64(u32x4 v) { return __hiloint2double(static_cast<int>(v.y), static_cast<int>(v.x)); }
__device__ __forceinline__ double hi64(u32x4 v) { return __hiloint2double(static_cast<int>(v.w), static_cast<int>(v.z)); }

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>(p));
}

// N pairs of doubles from consecutive LDS (a broadcast read), all issued before one wait: the
// compiler's own schedule of such reads keeps two in flight with a full round trip per pair
// (~130 cycles each: the 16-value pivot-block gather alone cost ~1000 cycles per step)
template <int N>
__device__ __forceinline__ void lds_read_pairs(const void* p, double (&out)[2 * N]) {
  const unsigned a = lds_addr(p);
  u32x4 v[N];
#pragma unroll
  for (int t = 0; t < N; ++t) v[t] = lds_2x64(a + 16 * t);
  if constexpr (N == 5) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]));
  } else {
    static_assert(N == 8, "lds_read_pairs: 5 or 8 pairs");
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]));
  }
#pragma unroll
  for (int t = 0; t < N; ++t) {
    out[2 * t] = lo64(v[t]);
    out[2 * t + 1] = hi64(v[t]);
  }
}

// 1 / sqrt(d): the hardware estimate + two Newton steps
__device__ __forceinline__ double rsqrt_nr(double d) {
  double r = __builtin_amdgcn_rsq(d);
  r = fma(0.5 * r, fma(-d * r, r, 1.0), r);
  r = fma(0.5 * r, fma(-d * r, r, 1.0), r);
  return r;
}

// The window update of one 4-column step: r[m] <- r[m + 4] - sum_q c[q] col[j + q][j + 4 + m] for
// m < W - 4, the top four slots cleared (slot m holds column j + m before, j + 4 + m after).  The
// four columns' values are read 2 slots at a time (one ds_read2_b64 per column), each chunk
// issued three chunks ahead of its FMAs (lgkmcnt counts at most 15), one explicit wait per chunk
// (one chunk of 4 slots ahead left LDS latency exposed: 3500-4400 cycles per 60-slot step).
template <int W>
__device__ __forceinline__ void block_elim(double (&r)[kTB], const PotrfLds& p, int j, const double (&c)[kPB]) {
  constexpr int kS = 2;                        // slots per chunk
  constexpr int NC = (W - kPB + kS - 1) / kS;  // chunks
  constexpr int kR = kPB * kS / 2;             // reads per chunk (4)
  constexpr int kAhead = 3;                    // chunks in flight ahead of the one consumed
  unsigned base[kPB];
#pragma unroll
  for (int q = 0; q < kPB; ++q) base[q] = lds_addr(&p.col[j + q][j + kPB]);
  u32x4 v[kAhead + 1][kR];
  auto issue = [&](int ch, u32x4 (&dst)[kR]) {
#pragma unroll
    for (int q = 0; q < kPB; ++q)
#pragma unroll
      for (int h = 0; h < kS / 2; ++h) dst[q * (kS / 2) + h] = lds_2x64(base[q] + 8 * (ch * kS + 2 * h));
  };
#pragma unroll
  for (int ch = 0; ch < kAhead && ch < NC; ++ch) issue(ch, v[ch]);
#pragma unroll
  for (int ch = 0; ch < NC; ++ch) {
    u32x4 (&cur)[kR] = v[ch % (kAhead + 1)];
    if (ch + kAhead < NC) issue(ch + kAhead, v[(ch + kAhead) % (kAhead + 1)]);
    // reads still allowed in flight behind this chunk's (in order): min(kAhead, NC - 1 - ch) chunks
    constexpr int kFull = kAhead * kR;
    const int behind = (NC - 1 - ch < kAhead ? NC - 1 - ch : kAhead) * kR;
    if (behind == kFull) {
      asm volatile("s_waitcnt lgkmcnt(12)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
    } else if (behind == 8) {
      asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
    } else if (behind == 4) {
      asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]));
    }
#pragma unroll
    for (int sl = 0; sl < kS; ++sl) {
      const int m = ch * kS + sl;
      if (m < W - kPB) {
        double acc = r[m + kPB];
#pragma unroll
        for (int q = 0; q < kPB; ++q) {
          const u32x4 w = cur[q * (kS / 2) + (sl >> 1)];
          acc = fma(-c[q], (sl & 1) ? hi64(w) : lo64(w), acc);
        }
        asm volatile("" : "+v"(acc));  // keep the FMAs here (sunk, they hold every read live)
        r[m] = acc;
      }
    }
  }
#pragma unroll
  for (int m = W - kPB; m < W; ++m) r[m] = 0.0;
}

// The diagonal tile's factorisation, 4 columns per step (a blocked right-looking Cholesky inside
// the tile: the step's 4 x 4 pivot block factored redundantly in every lane, then a rank-4 window
// update), by two waves with runtime step loops over a SHIFTING register window (slot m holds
// column j + m, every update writes 4 slots down, so every register index is a compile-time
// constant without unrolling the columns).  The window narrows in four phases of 16 columns
// (64, 48, 32, 16 slots).  Measured per-column costs that motivated the blocking: a one-column
// step spends ~700 cycles on its pivot, broadcast and hand-off whatever its window (~830 cycles
// at 16 slots, profiles/k9d_trace_windowed_r6.json) - four columns per step pay that once.
//
// wave 0: lane i = row i of L.  Each step publishes the 4 finished columns below the pivot block
// (col ring) and the block itself (piv) for wave 1, and writes its L entries to Z (= sA).
template <int W>
__device__ __forceinline__ void l_phase(double (&r)[kTB], int j0, int& fb, double (*Z)[kLd], PotrfLds& p, int probe,
                                        unsigned long long* cyc) {
#define CH_CYC(k) do { if (cyc != nullptr && lane == 0) cyc[(js / kPB) * 8 + (k)] = clock64(); } while (0)
  const int lane = threadIdx.x & 63;
  // the 4 steps of a phase unrolled: a runtime step loop made the back edge rotate every window
  // register (r[m] <- r[m + 4] lands in a new register: ~1300 extra moves per wave and tile)
#pragma unroll
  for (int js = 0; js < 16; js += kPB) {
    const int j = j0 + js;
    CH_CYC(0);
    // gather the pivot block rows j..j+3 (slots 0..3 of lanes j..j+3)
    if (lane >= j && lane < j + kPB) {
#pragma unroll
      for (int b = 0; b < kPB; ++b) p.g[lane - j][b] = r[b];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    double gv[16];
    lds_read_pairs<8>(&p.g[0][0], gv);
    double a[kPB][kPB];
#pragma unroll
    for (int x = 0; x < kPB; ++x)
#pragma unroll
      for (int y = 0; y < kPB; ++y) a[x][y] = gv[kPB * x + y];
    CH_CYC(1);
    // 4 x 4 Cholesky (uniform: every lane the same values)
    double l[kPB][kPB], rs[kPB];
#pragma unroll
    for (int q = 0; q < kPB; ++q) {
      double d = a[q][q];
#pragma unroll
      for (int b = 0; b < q; ++b) d = fma(-l[q][b], l[q][b], d);
      fb = (fb < 0 && !(d > 0.0)) ? j + q : fb;
      d = fb >= 0 ? 1.0 : d;  // keep every later value finite; the caller discards the factor
      rs[q] = rsqrt_nr(d);
      l[q][q] = d * rs[q];
#pragma unroll
      for (int x = q + 1; x < kPB; ++x) {
        double t = a[x][q];
#pragma unroll
        for (int b = 0; b < q; ++b) t = fma(-l[x][b], l[q][b], t);
        l[x][q] = t * rs[q];
      }
    }
    CH_CYC(2);
    // this lane's coefficients l_i,j..j+3 (forward substitution with the pivot block)
    double c[kPB];
#pragma unroll
    for (int q = 0; q < kPB; ++q) {
      double t = r[q];
#pragma unroll
      for (int b = 0; b < q; ++b) t = fma(-c[b], l[q][b], t);
      c[q] = t * rs[q];
    }
    const bool below = lane >= j + kPB;
#pragma unroll
    for (int q = 0; q < kPB; ++q) {
      c[q] = below ? c[q] : 0.0;
      p.col[j + q][lane] = c[q];
      // L entries: below the block c, inside it the block's row, above it zero
      const int rb = lane - j;
      double lv = 0.0;
#pragma unroll
      for (int x = 0; x < kPB; ++x) lv = (rb == x && q <= x) ? l[x][q] : lv;
      Z[lane][j + q] = below ? c[q] : lv;
    }
    CH_CYC(3);
    if (lane == 0) {
      double* pv = p.piv[j / kPB];
      pv[0] = l[1][0];
      pv[1] = l[2][0];
      pv[2] = l[2][1];
      pv[3] = l[3][0];
      pv[4] = l[3][1];
      pv[5] = l[3][2];
#pragma unroll
      for (int q = 0; q < kPB; ++q) pv[8 + q] = rs[q];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the step is in LDS before the flag
    if (lane == 0) __hip_atomic_store(&p.flag, j + kPB, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    CH_CYC(4);
    if (!(probe & 1)) block_elim<W>(r, p, j, c);
    CH_CYC(5);
  }
#undef CH_CYC
}

// wave 1: lane c = column c of inv(L), trailing wave 0 through the flag; x[m] holds row j + m.
// Per step: the pivot rows j..j+3 by forward substitution with the block, then the rank-4 update
// of the rows below with the published columns.
template <int W>
__device__ __forceinline__ void x_phase(double (&x)[kTB], int j0, int* status, double (*X)[kLd], PotrfLds& p,
                                        int probe) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int js = 0; js < 16; js += kPB) {
    const int j = j0 + js;
    unsigned spins = 0;
    while (__hip_atomic_load(&p.flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < j + kPB) {
      if (++spins > kChSpin) {
        status[1] = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    double pv[16];
    lds_read_pairs<8>(p.piv[j / kPB], pv);
    const double l10 = pv[0], l20 = pv[1], l21 = pv[2], l30 = pv[3], l31 = pv[4], l32 = pv[5];
    double xn[kPB];
    xn[0] = x[0] * pv[8];
    xn[1] = fma(-l10, xn[0], x[1]) * pv[9];
    xn[2] = fma(-l21, xn[1], fma(-l20, xn[0], x[2])) * pv[10];
    xn[3] = fma(-l32, xn[2], fma(-l31, xn[1], fma(-l30, xn[0], x[3]))) * pv[11];
#pragma unroll
    for (int q = 0; q < kPB; ++q) X[j + q][lane] = xn[q];
    if (!(probe & 1)) block_elim<W>(x, p, j, xn);
  }
}

// Factor the symmetric tile in sA (row-major, full) in place: on return sA holds L (zero above
// the diagonal) and sC holds inv(L).  Waves 0 and 1 only (the caller barriers).
__device__ __noinline__ void potrf_tile(int* status, int c, unsigned long long* trace, int probe) {
  double (*Z)[kLd] = sA;
  double (*X)[kLd] = sC;
  PotrfLds& p = pl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (probe & 8) return;
  if (w == 0) {
    double r[kTB];
#pragma unroll
    for (int k = 0; k < kTB; k += 2) {
      const double2 v = *reinterpret_cast<const double2*>(&Z[lane][k]);
      r[k] = v.x;
      r[k + 1] = v.y;
    }
    int fb = -1;  // first non-positive (or NaN) pivot: LAPACK info - 1
    unsigned long long* cyc = (trace != nullptr && c == 1) ? trace + 32 * 8 : nullptr;  // (nt = 32 in the probe)
    l_phase<64>(r, 0, fb, Z, p, probe, cyc);
    l_phase<48>(r, 16, fb, Z, p, probe, nullptr);
    l_phase<32>(r, 32, fb, Z, p, probe, nullptr);
    l_phase<16>(r, 48, fb, Z, p, probe, nullptr);
    if (lane == 0 && fb >= 0) atomicCAS(status, 0, kTB * c + fb + 1);
    if (trace != nullptr && lane == 0) trace[c * 8 + 7] = wall_clock64();  // wave 0's eliminations done
  } else if (w == 1 && !(probe & 2)) {
    double x[kTB];  // column `lane` of the inverse, window from row j
#pragma unroll
    for (int k = 0; k < kTB; ++k) x[k] = k == lane ? 1.0 : 0.0;
    x_phase<64>(x, 0, status, X, p, probe);
    x_phase<48>(x, 16, status, X, p, probe);
    x_phase<32>(x, 32, status, X, p, probe);
    x_phase<16>(x, 48, status, X, p, probe);
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
      potrf_tile(a.status, c, a.trace, a.exp);
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
  static const int probe = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K9D_PROBE");
    return e ? std::atoi(e) : 0;
  }();
  a.exp = probe;
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
