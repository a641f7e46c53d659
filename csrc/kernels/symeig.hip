// K9b: eigenvalues of a symmetric FP64 matrix for the FID compute.
//
// FID's compute needs tr sqrt(S1 S2) = sum sqrt(lambda_i(L^T S2 L)) at D = 2048 (fid.py in the
// reference: torch.linalg.eigvals of the non-symmetric product, reference
// torcheval/metrics/image/fid.py:253-262).  Round 2's path ran rocSOLVER's eigvalsh: ~45 ms at
// D = 2048, and its rocprof breakdown (profiles/rocprof_suite_kernel_stats_r1.csv) is ~7000
// launches of ~5 us (latrd gemv / dot / update kernels, one group per column of the
// Householder reduction) plus the tridiagonal solver: the chip idles between tiny launches.
//
// MI355X design: the whole D x D FP64 matrix lives on chip for the whole reduction, in the
// vector registers of one workgroup per CU (2048 x 2048 x 8 B = 32 MiB = 256 CUs x 128 KB;
// at D = 2048 a 512-thread workgroup, each thread holding 8 rows x 4 columns), one cooperative
// launch.  Workgroup g owns R consecutive rows; the matrix never goes
// back to HBM.  Householder tridiagonalisation (unblocked, LAPACK sytd2 semantics) with ONE
// grid-wide hand-off per column:
//   phase j publishes p_j = tau_j A v_j for the owned rows (8 B each) and, from the owner of
//   row j+1, that row as updated through step j-1; after the barrier every workgroup holds
//   the full p_j and row j+1, forms w_j = p_j - (tau_j/2)(p_j . v_j) v_j, applies step j to
//   row j+1 itself (so row j+1 is never re-published), derives the next reflector v_{j+1}
//   redundantly, and then ONE register pass over its rows both applies A -= v_j w_j^T + w_j v_j^T
//   and accumulates the next p_{j+1} = tau_{j+1} A v_{j+1}.
// Hand-offs: every handed-off double has its own 8-byte slot, used by exactly one phase of the
// launch; the launcher fills the slot planes with all-one bytes (a NaN pattern no stored value
// carries: every NaN is canonicalised to the default quiet NaN on the way out), the producer
// writes each value with ONE agent-scope (write-through) store, and consumers poll their slots
// with agent-scope loads until none is the sentinel - the data IS the flag: no drain, no
// counter, no fence.  (Round 2's form carried {32-bit phase tag, 32-bit half} granules, two per
// double; the sentinel form halves the bytes the 256 consumers re-read every column:
// 16.99 -> 16.25 ms at D = 2048, profiles/symeig_handoff_ab_r3.json.)  Every spin is bounded:
// a timed-out workgroup raises an abort word that every poller checks, the grid drains, and
// the host falls back to rocSOLVER when the status word is non-zero.
//
// The tridiagonal eigenvalues then come from ``tridiag_eigvals_kernel``: one wave per
// eigenvalue index (16 or 64 lanes), multisection of the Gershgorin interval with Sturm counts
// (LAPACK dstebz's count with pivmin), ~9-13 rounds to double precision.  Eigenvalues are written
// in ascending order; the caller sums sqrt(max(lambda, 0)).

#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "tea_kernels.h"

namespace tea {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxCols = 10;   // columns per thread: n <= 2560
constexpr int kMaxRows = 10;   // rows per workgroup (registers: R x C doubles per thread)
constexpr unsigned kSpinLimit = 1u << 18;
constexpr size_t kCtlBytes = 128;  // ctl[1] = abort word
// The last kTail columns of the reduction run in ONE workgroup with the trailing block in
// registers (symeig_tail_kernel): ~1.7 us a column there (a latency-bound chain of LDS round
// trips, DPP sums, sqrt / divisions and two barriers) against ~3.7 us a column for the grid's
// cross-CU hand-off (the grid's column cost is nearly flat in j: 4.4 us at j = 0, 3.7 at the end)
constexpr int kTail = 128;

#ifdef TEA_SYMEIG_TRACE  // csrc/bench/k9b_trace.hip: per-phase timestamps of two workgroups
__device__ unsigned long long* g_symeig_trace;
__device__ unsigned long long* g_symeig_col;  // workgroup 0's s_memrealtime (100 MHz) at every column
__device__ unsigned long long* g_symeig_tailtr;  // symeig_tail_kernel phase stamps, columns 0..15
#define SYM_TT(j, i)                                                                   \
  do {                                                                                 \
    if (threadIdx.x == 0 && (j) < 16) g_symeig_tailtr[(j) * 8 + (i)] = clock64();      \
  } while (0)
#define SYM_COL(j)                                                        \
  do {                                                                    \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_symeig_col[j] = wall_clock64(); \
  } while (0)
#define SYM_TRACE(j, i)                                                                       \
  do {                                                                                       \
    if (threadIdx.x == 0 && (blockIdx.x == 0 || blockIdx.x == 100) && (j) >= 1000 &&         \
        (j) < 1016)                                                                          \
      g_symeig_trace[(blockIdx.x ? 16 * 8 : 0) + ((j) - 1000) * 8 + (i)] = clock64();        \
  } while (0)
#else
#define SYM_TRACE(j, i) \
  do {                  \
  } while (0)
#define SYM_COL(j) \
  do {             \
  } while (0)
#define SYM_TT(j, i) \
  do {               \
  } while (0)
#endif

// every handed-off word is a GLOBAL (address space 1) agent-scope access, never flat
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

// the sentinel every slot holds until its phase stores it
constexpr unsigned long long kSentBits = ~0ull;

__device__ __forceinline__ void put(unsigned long long* g, int64_t i, double x) {
  const unsigned long long b =
      x != x ? 0x7ff8000000000000ull : static_cast<unsigned long long>(__double_as_longlong(x));
  __hip_atomic_store((gu64*)(g + i), b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long get(unsigned long long* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double as_double(unsigned long long b) {
  return __longlong_as_double(static_cast<long long>(b));
}

template <int Ctrl>
__device__ __forceinline__ double dpp_f64(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), Ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), Ctrl, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Sum of each 16-lane row of a wave, in every lane of the row: DPP quad swaps, half-row and
// row mirrors (a few cycles per step instead of an LDS-latency ds_bpermute).
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp_f64<0xB1>(x);   // quad_perm [1,0,3,2]
  x += dpp_f64<0x4E>(x);   // quad_perm [2,3,0,1]
  x += dpp_f64<0x141>(x);  // row_half_mirror
  x += dpp_f64<0x140>(x);  // row_mirror
  return x;
}

// Block-wide sums of N values: the NT / 16 row sums of the block go to LDS from the row's
// lanes, one barrier, then the partials are added as a fixed-order tree.  `scratch` holds
// (NT / 16) * N doubles; callers rotate scratch slots so consecutive reductions need one barrier
// each.  (Readlane-ing the 4 row sums of every wave first took ~15% more of the column's
// cycles, profiles/k9b_phase_trace_r2.txt; DPP transposes / row broadcasts instead, round 5:
// profiles/symeig_timing_dpp_reductions_r5.json.)
template <int N>
__device__ __forceinline__ void row_partials(const double (&v)[N], double* scratch) {
  const bool tail = (threadIdx.x & 15) == 15;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const double x = row16_sum(v[i]);
    if (tail) scratch[(threadIdx.x >> 4) * N + i] = x;
  }
  __syncthreads();
}

// every thread gets every total
// the NT / 16 row partials of one value, added as a pairwise tree (depth log2 instead of a
// chain of NT / 16 dependent FP64 adds; fixed order, so still deterministic)
template <int N, int NT>
__device__ __forceinline__ double tree_partials(const double* scratch, int i) {
  constexpr int NP = NT / 16;
  double p[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) p[q] = scratch[q * N + i];
#pragma unroll
  for (int w = NP / 2; w >= 1; w /= 2) {
#pragma unroll
    for (int q = 0; q < w; ++q) p[q] += p[q + w];
  }
  return p[0];
}

template <int Ctrl, int RowMask>
__device__ __forceinline__ double dpp_f64_rows(double x) {  // 0 in the rows RowMask leaves out
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), Ctrl, RowMask, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), Ctrl, RowMask, 0xf, false);
  return __hiloint2double(hi, lo);
}

template <int N, int NT = kThreads>
__device__ __forceinline__ void block_sum(double (&v)[N], double* scratch) {
  if constexpr (N == 1) {
    // one value: the wave total by DPP (row sums, then row_bcast:15 / row_bcast:31 into lane
    // 63), so the tree below adds NT / 64 wave partials instead of NT / 16 row partials
    double x = row16_sum(v[0]);
    x += dpp_f64_rows<0x142, 0xa>(x);
    x += dpp_f64_rows<0x143, 0xc>(x);
    if ((threadIdx.x & 63) == 63) scratch[threadIdx.x >> 6] = x;
    __syncthreads();
    constexpr int NP = NT / 64;
    double q[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) q[k] = scratch[k];
#pragma unroll
    for (int w = NP / 2; w >= 1; w /= 2) {
#pragma unroll
      for (int k = 0; k < w; ++k) q[k] += q[k + w];
    }
    v[0] = q[0];
  } else {
    row_partials<N>(v, scratch);
#pragma unroll
    for (int i = 0; i < N; ++i) v[i] = tree_partials<N, NT>(scratch, i);
  }
}

// x plus the same lane of the other 16-lane row of its pair (rows 0+1, 2+3) / of the other
// 32-lane half, in every lane: gfx950's v_permlane16_swap / v_permlane32_swap with both operands
// x, so the two outputs are x and its partner's x
__device__ __forceinline__ double perm_pair_sum16(double x) {
  const unsigned lo = static_cast<unsigned>(__double2loint(x)), hi = static_cast<unsigned>(__double2hiint(x));
  const auto a = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(static_cast<int>(b[0]), static_cast<int>(a[0])) +
         __hiloint2double(static_cast<int>(b[1]), static_cast<int>(a[1]));
}
__device__ __forceinline__ double perm_pair_sum32(double x) {
  const unsigned lo = static_cast<unsigned>(__double2loint(x)), hi = static_cast<unsigned>(__double2hiint(x));
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __hiloint2double(static_cast<int>(b[0]), static_cast<int>(a[0])) +
         __hiloint2double(static_cast<int>(b[1]), static_cast<int>(a[1]));
}

// thread t < N gets total t (the per-row p values, published by thread t)
template <int N, int NT = kThreads>
__device__ __forceinline__ double block_sum_own(const double (&v)[N], double* scratch) {
  if constexpr (N == 8) {
    // eight values (the p reduction of 8 owned rows): a transposing reduction inside each
    // 16-lane row - every exchange step halves the values a lane keeps and doubles the lanes each
    // is summed over (row mirror, half-row mirror, quad reverse, quad swap: 8 DPP exchanges
    // instead of 8 x 4, 12.17 -> 11.86 ms at D = 2048) - then the 4 rows of the wave by permlane
    // swaps: NT / 64 wave partials per value instead of NT / 16 row partials (-> 10.93 ms)
    const int p = threadIdx.x & 15;
    const bool b3 = (p & 8) != 0, b2 = (p & 4) != 0, b1 = (p & 2) != 0;
    double u1[4], u2[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const double send = b3 ? v[k] : v[k + 4], keep = b3 ? v[k + 4] : v[k];
      u1[k] = keep + dpp_f64<0x140>(send);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const double send = b2 ? u1[k] : u1[k + 2], keep = b2 ? u1[k + 2] : u1[k];
      u2[k] = keep + dpp_f64<0x141>(send);
    }
    const double send3 = b1 ? u2[0] : u2[1], keep3 = b1 ? u2[1] : u2[0];
    double u = keep3 + dpp_f64<0x1B>(send3);
    u += dpp_f64<0xB1>(u);
    u = perm_pair_sum16(u);
    u = perm_pair_sum32(u);
    if ((threadIdx.x & 63) < 16 && !(p & 1))
      scratch[(threadIdx.x >> 6) * 8 + (b3 ? 4 : 0) + (b2 ? 2 : 0) + (b1 ? 1 : 0)] = u;
    __syncthreads();
    if (threadIdx.x >= 8) return 0.0;
    constexpr int NP = NT / 64;
    double q[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) q[k] = scratch[k * 8 + threadIdx.x];
#pragma unroll
    for (int w = NP / 2; w >= 1; w /= 2) {
#pragma unroll
      for (int k = 0; k < w; ++k) q[k] += q[k + w];
    }
    return q[0];
  } else {
    row_partials<N>(v, scratch);
    return threadIdx.x < N ? tree_partials<N, NT>(scratch, threadIdx.x) : 0.0;
  }
}

struct Reflector {
  double tau, beta, scale, diag;
};

// LAPACK dlarfg on x = a[j+1 .. n): alpha = a[j+1], sigma = sum_{k >= j+2} a[k]^2; also
// broadcasts the diagonal a[j].  v[k] = 1 at k = j+1, a[k] * scale beyond, 0 before.
template <int C, int NT = kThreads>
__device__ __forceinline__ Reflector householder(const double (&a)[C], int j, int n,
                                                 double* scratch, double* bcast) {
  // sigma by the block reduction; alpha = a[j+1] and the diagonal a[j] are single elements,
  // so their owner threads just store them next to the partials (the reduction's barrier
  // publishes them)
  double r[1] = {0.0};
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int k = threadIdx.x + s * NT;
    const double x = a[s];
    r[0] += (k >= j + 2 && k < n) ? x * x : 0.0;
    if (k == j + 1) bcast[0] = x;
    if (k == j) bcast[1] = x;
  }
  block_sum<1, NT>(r, scratch);
  Reflector h;
  const double sigma = r[0], alpha = bcast[0];
  h.diag = bcast[1];
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

template <int C, int NT = kThreads>
__device__ __forceinline__ void make_v(const double (&a)[C], const Reflector& h, int j,
                                       double (&v)[C]) {
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int k = threadIdx.x + s * NT;
    v[s] = k == j + 1 ? 1.0 : (k >= j + 2 ? a[s] * h.scale : 0.0);
  }
}

// element s of owned row r for a run-time r (the publishing owner only): a select chain over the
// register-resident rows
template <int C, int RM>
__device__ __forceinline__ double row_elem(const double (&rw)[RM][C], int r, int s_) {
  double x = 0.0;
#pragma unroll
  for (int q = 0; q < RM; ++q) {
#pragma unroll
    for (int s = 0; s < C; ++s) x = (q == r && s == s_) ? rw[q][s] : x;
  }
  return x;
}

// One workgroup per CU; each thread holds its columns (t + 256 s) of the workgroup's R owned
// rows in registers for the whole reduction (round 2 kept them in LDS: the per-column pass was
// LDS-bandwidth bound, ~16 B of LDS traffic per element per column).  Slot planes of
// [n - 2, ld] each at slots + {0, 1} * plane: p_q, then row q+1 (as updated through step q-1);
// all sentinel-filled by the launcher.  ctl[1] = abort word, zeroed by the launcher.
// NT threads per workgroup (256, or 512 for the two-waves-per-SIMD A/B arm: half the columns
// per thread, twice the row partials per reduction)
template <int C, int RM, int NT = kThreads>
__global__ __launch_bounds__(NT) void tridiag_kernel(const double* __restrict__ A, int n,
                                                     int R, int64_t ld, double* d_out,
                                                     double* e_out, unsigned long long* slots,
                                                     unsigned* ctl, double* tail, int jt) {
  __shared__ double red[3][(NT / 16) * RM];
  __shared__ double bc[2][4];  // single-element broadcasts riding on the reductions' barriers
  __shared__ double vw[2][RM];
  __shared__ int s_abort;  // a poll timed out / saw the abort word (read after R1's barrier)
  const int64_t plane = (int64_t)(n - 2) * ld;
  unsigned long long* const gp0 = slots;          // p plane
  unsigned long long* const gr0 = slots + plane;  // row plane

  const int t = threadIdx.x;
  const int row0 = blockIdx.x * R;
  const int nrows = min(R, n - row0);
  double rw[RM][C];  // owned row r, column t + s * NT
#pragma unroll
  for (int r = 0; r < RM; ++r)
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = t + s * NT;
      rw[r][s] = (r < nrows && k < n) ? A[(int64_t)(row0 + r) * n + k] : 0.0;
    }

  double a[C], v[C], w[C], vn[C];
#pragma unroll
  for (int s = 0; s < C; ++s) {
    const int k = t + s * NT;
    a[s] = k < n ? A[k] : 0.0;  // row 0
  }
  if (t == 0) s_abort = 0;
  __syncthreads();

  // ---- phase 0: reflector 0 and p_0 from the original rows
  Reflector h = householder<C, NT>(a, 0, n, red[0], bc[0]);
  make_v<C, NT>(a, h, 0, v);
  if (blockIdx.x == 0 && t == 0) {
    d_out[0] = h.diag;
    e_out[0] = h.beta;
  }
  {
    double acc[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      acc[r] = 0.0;
      if (r < nrows) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = t + s * NT;
          if (k < n) acc[r] += rw[r][s] * v[s];
        }
      }
    }
    const double pt = block_sum_own<RM, NT>(acc, red[2]);
    if (t < nrows && row0 + t >= 1) put(gp0, row0 + t, h.tau * pt);
    if (1 >= row0 && 1 < row0 + nrows) {
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = t + s * NT;
        if (k >= 1 && k < n) put(gr0, k, row_elem<C, RM>(rw, 1 - row0, s));
      }
    }
  }

  // (Skipping whole dead column slots with wave-uniform branches in the loads and the LDS
  // pass measured slower - 19.4 vs 17.9 ms at D = 2048: the branches split the batched loads.)
  for (int j = 0; j <= n - 3; ++j) {
    if (j == jt) break;  // the trailing block goes to symeig_tail_kernel (below the loop)
    SYM_COL(j);
    // ---- w_j from the gathered p_j; row j+1 updated through step j.  Each thread polls the
    // slots of ITS columns until none holds the sentinel (bounded; any abort ends the
    // block at the reduction barrier below)
    unsigned long long* const gp = gp0 + (int64_t)j * ld;
    unsigned long long* const gr = gr0 + (int64_t)j * ld;
    bool aborted = false;
    for (unsigned spins = 0;; ++spins) {
      // the abort word is loaded with the slots, in the same round trip (loaded after a failed
      // poll it doubled every poll period: one more ~1 us round trip before the next poll)
      const unsigned abort_word = __hip_atomic_load((gu32*)&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // every slot load issued unconditionally (dead columns read a live slot, masked after): a
      // per-lane `if (live) load` can compile to a branch and a wait per column
      unsigned long long xs[C], ys[C];
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = t + s * NT;
        const int kc = k < j + 1 ? j + 1 : (k < n ? k : n - 1);
        xs[s] = get(gp + kc);
        ys[s] = get(gr + kc);
      }
      bool ok = true;
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = t + s * NT;
        const bool live = k >= j + 1 && k < n;
        ok = ok && (!live || (xs[s] != kSentBits && ys[s] != kSentBits));
        w[s] = live ? as_double(xs[s]) : 0.0;
        a[s] = live ? as_double(ys[s]) : 0.0;
      }
      if (ok) break;
      if (abort_word != 0u) {
        aborted = true;
        break;
      }
      if (spins > kSpinLimit) {
        __hip_atomic_store((gu32*)&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        aborted = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    // no barrier of its own: the abort vote rides R1's reduction barrier (every LDS slot it
    // writes was last read before the previous column's reflector barrier)
    if (aborted) s_abort = 1;
    SYM_TRACE(j, 0);
    double r1[1] = {0.0};
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = t + s * NT;
      r1[0] += w[s] * v[s];
      if (k == j + 1) bc[0][2] = w[s];  // p_j[j+1], published by the reduction's barrier
    }
    block_sum<1, NT>(r1, red[0]);
    if (s_abort) return;  // block-uniform
    SYM_TRACE(j, 1);
    const double c = 0.5 * h.tau * r1[0];
    const double wj1 = bc[0][2] - c;  // w_j[j+1] (v_j[j+1] = 1)
#pragma unroll
    for (int s = 0; s < C; ++s) {
      w[s] -= c * v[s];
      a[s] -= w[s] + wj1 * v[s];  // row j+1 <- row j+1 - v_j[j+1] w_j - w_j[j+1] v_j
      const int k = t + s * NT;
      const int r = k - row0;
      if (r >= 0 && r < nrows) {  // the owned rows' v_j[i], w_j[i] for the rank-2 update
        vw[0][r] = v[s];
        vw[1][r] = w[s];
      }
    }

    SYM_TRACE(j, 6);
    if (j == n - 3) {
      // last step: row n-2 is final; the owner of row n-1 finishes its diagonal
      if (blockIdx.x == 0) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = t + s * NT;
          if (k == n - 2) d_out[n - 2] = a[s];
          if (k == n - 1) e_out[n - 2] = a[s];
        }
      }
      __syncthreads();
      const int r = (n - 1) - row0;
      if (r >= 0 && r < nrows) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = t + s * NT;
          if (k == n - 1) d_out[n - 1] = row_elem<C, RM>(rw, r, s) - 2.0 * vw[0][r] * vw[1][r];
        }
      }
      break;
    }

    // ---- reflector j+1 (redundant in every workgroup)
    const Reflector hn = householder<C, NT>(a, j + 1, n, red[1], bc[1]);  // its barrier publishes vw
    make_v<C, NT>(a, hn, j + 1, vn);
    SYM_TRACE(j, 2);
    if (blockIdx.x == 0 && t == 0) {
      d_out[j + 1] = hn.diag;
      e_out[j + 1] = hn.beta;
    }

    // ---- one register pass: apply step j to the owned rows, accumulate p_{j+1}.  No column
    // test: below column j+1 (and past n) w_j, v_j and v_{j+1} are zero, so those entries are
    // left as they are and add nothing.  (Deferring the update past the p hand-off, with p
    // corrected for it as LAPACK latrd does, measured no faster: 14.74 vs 14.69 ms at D = 2048.)
    double acc[RM];
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      acc[r] = 0.0;
      if (r < nrows && row0 + r >= j + 1) {  // block-uniform
        // two FMAs per element for the rank-2 update (the pass is near the FP64 FMA rate: 3
        // instead of 4 VALU ops per element)
        const double nvi = -vw[0][r], nwi = -vw[1][r];
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const double x = fma(nvi, w[s], fma(nwi, v[s], rw[r][s]));
          rw[r][s] = x;
          acc[r] = fma(x, vn[s], acc[r]);
        }
      }
    }
    // the owner of row j+2 publishes the row before the p reduction
    SYM_TRACE(j, 3);
    const int ro = (j + 2) - row0;
    if (ro >= 0 && ro < nrows) {
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = t + s * NT;
        if (k >= j + 2 && k < n) put(gr0 + (int64_t)(j + 1) * ld, k, row_elem<C, RM>(rw, ro, s));
      }
    }
    SYM_TRACE(j, 7);
    const double pt = block_sum_own<RM, NT>(acc, red[2]);
    SYM_TRACE(j, 4);
    if (t < nrows && row0 + t >= j + 2) put(gp0 + (int64_t)(j + 1) * ld, row0 + t, hn.tau * pt);
#pragma unroll
    for (int s = 0; s < C; ++s) v[s] = vn[s];
    h = hn;
    SYM_TRACE(j, 5);
  }
  if (jt < n) {
    // stopped at column jt: the owned rows' columns >= jt (updated through step jt - 1) are the
    // tail kernel's trailing block
#pragma unroll
    for (int r = 0; r < RM; ++r) {
      const int row = row0 + r;
      if (r < nrows && row >= jt) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = t + s * NT;
          if (k >= jt && k < n) tail[(int64_t)(row - jt) * kTail + (k - jt)] = rw[r][s];
        }
      }
    }
  }
}

// ---------------------------------------------------------------- K9b v2: rows per WAVE
// The same one-launch Householder reduction with a different ownership: each WAVE holds kRW
// whole rows (lane l: columns l + 64 s, s < C), so every reduction of a column step is a
// wave reduction (DPP inside 16-lane rows + 4 readlanes) instead of a block reduction with an
// LDS round trip and a barrier.  The per-column phase trace of tridiag_kernel
// (csrc/bench/k9b_trace.hip, round 5) spent ~8.9k of ~15.7k cycles per column in its three
// block reductions, the reflector and the pass; the hand-off wait was the other ~6.8k.  Per
// column here: the workgroup stages the handed-off p_j and row j+1 in LDS (one barrier,
// double-buffered by column parity), then each wave redundantly forms w_j, updates row j+1,
// derives reflector j+1 and applies step j to its rows while accumulating p_{j+1} - no further
// barrier.  Hand-off slots, sentinel protocol, abort word and outputs are tridiag_kernel's.
// Measured (round 5, profiles/symeig_wave_ab_r5.json): exact (the K9b tests pass with it), but
// 18.5 ms at D = 2048 against tridiag_kernel's 14.7 ms - every wave redoes the column-length
// work (R1, the row j+1 update, the reflector: 32 elements per lane instead of 8) and at one
// wave per SIMD nothing hides the dependent DPP / readlane chains - so it is opt-in.
constexpr int kRW = 2;                // rows per wave
constexpr int kWRows = kRW * kWaves;  // rows per workgroup

__device__ __forceinline__ double readlane_d(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

// the wave's total in every lane, fixed order (deterministic)
__device__ __forceinline__ double wave_sum_d(double x) {
  x = row16_sum(x);
  return (readlane_d(x, 15) + readlane_d(x, 31)) + (readlane_d(x, 47) + readlane_d(x, 63));
}

// LAPACK dlarfg on x = a[jj+1 .. n) with the diagonal a[jj]; `alpha`, `diag` broadcast by the
// caller; returns tau / beta / scale (v[jj+1] = 1, v[k] = a[k] * scale beyond)
__device__ __forceinline__ Reflector reflector_of(double alpha, double sigma, double diag) {
  Reflector h;
  h.diag = diag;
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

template <int C>
__global__ __launch_bounds__(kThreads, 1) void tridiag_wave_kernel(const double* __restrict__ A, int n, int64_t ld,
                                                                    double* d_out, double* e_out,
                                                                    unsigned long long* slots, unsigned* ctl) {
  constexpr int kCols = C * 64;
  constexpr int kQ = kCols / kThreads;  // staged slots per thread per plane
  __shared__ double sp[2][kCols];       // p_j, by column parity
  __shared__ double sr[2][kCols];       // row j+1 (updated through step j-1)
  const int64_t plane = (int64_t)(n - 2) * ld;
  unsigned long long* const gp0 = slots;
  unsigned long long* const gr0 = slots + plane;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int row0 = blockIdx.x * kWRows + wv * kRW;  // this wave's first row
  // registers: the wave's rows, v_j and a (row j+1, turned into v_{j+1} in place); w_j is
  // re-formed from the staged p_j where it is needed (register pressure: 4 x C doubles)
  double rw[kRW][C];
#pragma unroll
  for (int r = 0; r < kRW; ++r)
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = lane + 64 * s, row = row0 + r;
      rw[r][s] = (row < n && k < n) ? A[(int64_t)row * n + k] : 0.0;
    }
  double v[C], a[C];

  // ---- phase 0: reflector 0 from row 0, p_0 of the wave's rows, row 1 published as is
  Reflector h;
  {
    double s2 = 0.0, alpha = 0.0, diag = 0.0;
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = lane + 64 * s;
      a[s] = k < n ? A[k] : 0.0;
      s2 += k >= 2 ? a[s] * a[s] : 0.0;
      alpha = k == 1 ? a[s] : alpha;
      diag = k == 0 ? a[s] : diag;
    }
    h = reflector_of(readlane_d(alpha, 1), wave_sum_d(s2), readlane_d(diag, 0));
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = lane + 64 * s;
      v[s] = k == 1 ? 1.0 : (k >= 2 ? a[s] * h.scale : 0.0);
    }
    if (blockIdx.x == 0 && t == 0) {
      d_out[0] = h.diag;
      e_out[0] = h.beta;
    }
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int s = 0; s < C; ++s) acc += rw[r][s] * v[s];
      acc = wave_sum_d(acc);
      const int row = row0 + r;
      if (lane == 0 && row < n && row >= 1) put(gp0, row, h.tau * acc);
    }
    if (row0 <= 1 && 1 < row0 + kRW) {
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = lane + 64 * s;
        if (k >= 1 && k < n) put(gr0, k, row0 == 1 ? rw[0][s] : rw[1][s]);
      }
    }
  }

  for (int j = 0; j <= n - 3; ++j) {
    // ---- stage p_j and row j+1 in LDS (dead / padded columns as zeros); bounded spin
    unsigned long long* const gp = gp0 + (int64_t)j * ld;
    unsigned long long* const gr = gr0 + (int64_t)j * ld;
    double* const P = sp[j & 1];
    double* const R = sr[j & 1];
    bool aborted = false;
    for (unsigned spins = 0;; ++spins) {
      const unsigned abort_word = __hip_atomic_load((gu32*)&ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bool ok = true;
#pragma unroll
      for (int q = 0; q < kQ; ++q) {
        const int k = t + kThreads * q;
        if (k >= j + 1 && k < n) {
          const unsigned long long x0 = get(gp + k), y0 = get(gr + k);
          ok = ok && x0 != kSentBits && y0 != kSentBits;
          P[k] = as_double(x0);
          R[k] = as_double(y0);
        } else {
          P[k] = 0.0;
          R[k] = 0.0;
        }
      }
      if (ok) break;
      if (abort_word != 0u) {
        aborted = true;
        break;
      }
      if (spins > kSpinLimit) {
        __hip_atomic_store((gu32*)&ctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        aborted = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (__syncthreads_or(aborted)) return;

    // ---- w_j = p_j - c v_j, row j+1 <- row j+1 - v_j[j+1] w_j - w_j[j+1] v_j (every wave)
    double r1 = 0.0;
#pragma unroll
    for (int s = 0; s < C; ++s) r1 += P[lane + 64 * s] * v[s];
    r1 = wave_sum_d(r1);
    const double c = 0.5 * h.tau * r1;
    const double wj1 = P[j + 1] - c;  // v_j[j+1] = 1
    double vi0 = 0.0, vi1 = 0.0, a1 = 0.0, a2 = 0.0, s2 = 0.0;
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = lane + 64 * s;
      const double ws = P[k] - c * v[s];
      a[s] = R[k] - (ws + wj1 * v[s]);
      vi0 = k == row0 ? v[s] : vi0;
      vi1 = k == row0 + 1 ? v[s] : vi1;
      a1 = k == j + 1 ? a[s] : a1;
      a2 = k == j + 2 ? a[s] : a2;
      s2 += k >= j + 3 ? a[s] * a[s] : 0.0;
    }
    // the wave's rows' v_j[i] (lane i & 63 holds them), w_j[i] from the staged p_j
    double vi[kRW], wi[kRW];
    vi[0] = row0 < n ? readlane_d(vi0, row0 & 63) : 0.0;
    vi[1] = row0 + 1 < n ? readlane_d(vi1, (row0 + 1) & 63) : 0.0;
    wi[0] = row0 < n ? P[row0] - c * vi[0] : 0.0;
    wi[1] = row0 + 1 < n ? P[row0 + 1] - c * vi[1] : 0.0;
    a1 = readlane_d(a1, (j + 1) & 63);

    if (j == n - 3) {
      // last step: row n-2 is final; the owner of row n-1 finishes its diagonal
      if (blockIdx.x == 0 && wv == 0) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = lane + 64 * s;
          if (k == n - 2) d_out[n - 2] = a[s];
          if (k == n - 1) e_out[n - 2] = a[s];
        }
      }
      const int r = (n - 1) - row0;
      if (r >= 0 && r < kRW) {
#pragma unroll
        for (int s = 0; s < C; ++s) {
          const int k = lane + 64 * s;
          if (k == n - 1) d_out[n - 1] = (r == 0 ? rw[0][s] : rw[1][s]) - 2.0 * vi[r] * wi[r];
        }
      }
      break;
    }

    // ---- reflector j+1 (redundant in every wave); a becomes v_{j+1}
    a2 = readlane_d(a2, (j + 2) & 63);
    const Reflector hn = reflector_of(a2, wave_sum_d(s2), a1);
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const int k = lane + 64 * s;
      a[s] = k == j + 2 ? 1.0 : (k >= j + 3 ? a[s] * hn.scale : 0.0);
    }
    if (blockIdx.x == 0 && t == 0) {
      d_out[j + 1] = hn.diag;
      e_out[j + 1] = hn.beta;
    }

    // ---- one register pass: step j on the wave's rows, p_{j+1} accumulated
    double acc[kRW] = {0.0, 0.0};
    const bool live0 = row0 < n && row0 >= j + 1, live1 = row0 + 1 < n && row0 + 1 >= j + 1;  // wave-uniform
#pragma unroll
    for (int s = 0; s < C; ++s) {
      const double ws = P[lane + 64 * s] - c * v[s];
      if (live0) {
        const double x = rw[0][s] - (vi[0] * ws + wi[0] * v[s]);
        rw[0][s] = x;
        acc[0] += x * a[s];
      }
      if (live1) {
        const double x = rw[1][s] - (vi[1] * ws + wi[1] * v[s]);
        rw[1][s] = x;
        acc[1] += x * a[s];
      }
    }
    // the owner of row j+2 publishes the row before the p reduction
    const int ro = (j + 2) - row0;
    if (ro >= 0 && ro < kRW) {
#pragma unroll
      for (int s = 0; s < C; ++s) {
        const int k = lane + 64 * s;
        if (k >= j + 2 && k < n) put(gr0 + (int64_t)(j + 1) * ld, k, ro == 0 ? rw[0][s] : rw[1][s]);
      }
    }
#pragma unroll
    for (int r = 0; r < kRW; ++r) {
      const double pt = wave_sum_d(acc[r]);
      const int row = row0 + r;
      if (lane == 0 && row < n && row >= j + 2) put(gp0 + (int64_t)(j + 1) * ld, row, hn.tau * pt);
    }
#pragma unroll
    for (int s = 0; s < C; ++s) v[s] = a[s];
    h = hn;
  }
}

// The reduction's last kTail columns on one workgroup (LAPACK dsytd2 on the trailing block),
// the block held in registers: TR x 8 tiles, 16 tile columns, kTail / TR tile rows, one thread a
// tile (thread t: tile row t / 16, tile column t % 16; a 16-lane DPP row = one tile row).  Per
// column: the owners of column j publish it (barrier), every wave forms the reflector
// redundantly from it (DPP sums), the tile products p = M v reduce over the 16 lanes of a tile
// row (DPP), tau p goes through LDS (barrier), p . v reduces over a tile row's column tiles,
// then the rank-2 update M -= v w^T + w v^T in registers.
// a lane's double in every lane (two readlanes)
__device__ __forceinline__ double lane_f64(double x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l), hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int TR>
__global__ __launch_bounds__(16 * kTail / TR) void symeig_tail_kernel(const double* __restrict__ tail, int n,
                                                                      double* d_out, double* e_out) {
  constexpr int NT = 16 * kTail / TR;
  __shared__ double col[kTail];
  __shared__ double tp[kTail];
  const int t = threadIdx.x, rb = t >> 4, cb = t & 15, jt = n - kTail;
  double m[TR][8];
#pragma unroll
  for (int a = 0; a < TR; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) m[a][b] = tail[(rb * TR + a) * kTail + cb * 8 + b];
  if (cb == 0) {
#pragma unroll
    for (int a = 0; a < TR; ++a) col[rb * TR + a] = m[a][0];
  }
  __syncthreads();
  for (int jb = 0; jb < kTail / 8; ++jb) {
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
      const int j = jb * 8 + jj;
      if (j > kTail - 3) break;
      SYM_TT(j, 0);
      // reflector of column j (rows > j), redundantly in every wave
      const int l = t & 63;
      const double x0 = col[l], x1 = col[l + 64];
      // every column value this thread needs, loaded unconditionally up front (loads under the
      // v selects below compiled to one branch and one LDS round trip each)
      double cr[TR], cc[8];
#pragma unroll
      for (int a = 0; a < TR; ++a) cr[a] = col[rb * TR + a];
#pragma unroll
      for (int b = 0; b < 8; ++b) cc[b] = col[cb * 8 + b];
      const double cj = col[j];
      double sg = row16_sum((l >= j + 2 ? x0 * x0 : 0.0) + (l + 64 >= j + 2 ? x1 * x1 : 0.0));
      sg = (lane_f64(sg, 0) + lane_f64(sg, 16)) + (lane_f64(sg, 32) + lane_f64(sg, 48));
      const double alpha = col[j + 1];
      SYM_TT(j, 1);
      double tau, beta, scale;
      if (sg == 0.0) {
        tau = 0.0;
        beta = alpha;
        scale = 0.0;
      } else {
        const double mu = sqrt(alpha * alpha + sg);
        beta = alpha >= 0.0 ? -mu : mu;
        tau = (beta - alpha) / beta;
        scale = 1.0 / (alpha - beta);
      }
      if (t == 0) {
        d_out[jt + j] = cj;
        e_out[jt + j] = beta;
      }
      SYM_TT(j, 2);
      double vr[TR], vc[8];
#pragma unroll
      for (int a = 0; a < TR; ++a) {
        const int i = rb * TR + a;
        vr[a] = i == j + 1 ? 1.0 : (i > j + 1 ? cr[a] * scale : 0.0);
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const int k = cb * 8 + b;
        vc[b] = k == j + 1 ? 1.0 : (k > j + 1 ? cc[b] * scale : 0.0);
      }
      // p = tau M v: tile products, reduced over the tile row's 16 lanes
      double p[TR];
#pragma unroll
      for (int a = 0; a < TR; ++a) {
        double acc = 0.0;
#pragma unroll
        for (int b = 0; b < 8; ++b) acc = fma(m[a][b], vc[b], acc);
        p[a] = acc;
      }
#pragma unroll
      for (int a = 0; a < TR; ++a) p[a] = tau * row16_sum(p[a]);
      SYM_TT(j, 3);
      if (cb == 0) {
#pragma unroll
        for (int a = 0; a < TR; ++a) tp[rb * TR + a] = p[a];
      }
      __syncthreads();
      SYM_TT(j, 4);
      // p . v over the tile row's 16 column tiles (every index once)
      double tc[8], pv = 0.0;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        tc[b] = tp[cb * 8 + b];
        pv = fma(tc[b], vc[b], pv);
      }
      const double K = 0.5 * tau * row16_sum(pv);
      double wr[TR], wc[8];
#pragma unroll
      for (int a = 0; a < TR; ++a) wr[a] = p[a] - K * vr[a];
#pragma unroll
      for (int b = 0; b < 8; ++b) wc[b] = tc[b] - K * vc[b];
#pragma unroll
      for (int a = 0; a < TR; ++a)
#pragma unroll
        for (int b = 0; b < 8; ++b) m[a][b] = fma(-vr[a], wc[b], fma(-wr[a], vc[b], m[a][b]));
      SYM_TT(j, 5);
      // the next column, as updated through this step
      const int jn = j + 1;
      if (cb == (jn >> 3)) {
#pragma unroll
        for (int a = 0; a < TR; ++a) {
          double x = 0.0;
#pragma unroll
          for (int b = 0; b < 8; ++b) x = b == (jn & 7) ? m[a][b] : x;
          col[rb * TR + a] = x;
        }
      }
      __syncthreads();
    }
  }
  if (t == NT - 1) {  // the last tile: rows kTail - TR .., columns kTail - 8 ..
    d_out[n - 2] = m[TR - 2][6];
    e_out[n - 2] = m[TR - 1][6];
    d_out[n - 1] = m[TR - 1][7];
  }
}

// # eigenvalues of the tridiagonal (d, e2 = e^2) below x (LAPACK dstebz's Sturm count).
// (Round 3: the bare v_rcp_f64 was faster but cost 6e-9 of accuracy, and rcp + Newton with two
// interleaved chains per lane measured 13% slower; round 5: one chain, rcp + one Newton step,
// D = 2048 eigenvalues 9.85 -> 9.40 ms at unchanged accuracy, profiles/symeig_timing_sturm_rcp_newton_r5.json.)
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int n, double x,
                                           double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int cnt = q < 0.0;
  for (int k = 1; k < n; ++k) {
    // e2 / q as e2 * (v_rcp_f64 + one Newton step): 4 dependent ops on the recurrence's critical
    // path instead of the IEEE division's ~9.  q is finite and |q| >= pivmin >= DBL_MIN (normal),
    // and e2 / |q| <= 1 / DBL_MIN, so no overflow / denormal special case arises (LAPACK's pivmin
    // argument); the refined reciprocal is within an ulp or two of the quotient's
    double r = __builtin_amdgcn_rcp(q);
    r = fma(r, fma(-q, r, 1.0), r);
    q = d[k] - x - e2[k - 1] * r;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
  }
  return cnt;
}

// The same count from the three-term recurrence of the leading minors,
// p_k = (d_k - x) p_{k-1} - e_{k-1}^2 p_{k-2} (count = sign changes of p_0 = 1, p_1, .., p_n): ONE
// FMA on the recurrence's critical path (e^2 p_{k-2} is ready a step early; the sign change is
// integer work on the sign words, off the path), against the ratio form's reciprocal, three FMAs
// and the pivot guard (~94 cycles a step at one wave per SIMD).  Needs the tridiagonal scaled to
// O(1) with every e^2 at least 2^-600 (tridiag_setup: zeros and tinier values are raised to it, a
// perturbation of 2^-300 in e), so |p| grows at most 8x a step and two consecutive minors are
// never both zero; the pair (p_{k-1}, p_{k-2}) is renormalised by a power of two every 4 steps.
// An exact zero minor comes out +0 and counts as positive: with e^2 > 0 the next minor,
// -e^2 p_{k-2}, has the sign opposite to p_{k-2}, so the pair contributes the one sign change the
// ratio form's -pivmin convention gives.  Each step is exact for d_k, e_k^2 perturbed by an ulp
// or two (backward stable, as the ratio form).
__device__ __forceinline__ int sign_flip(double p, double q) {
  return static_cast<int>((static_cast<unsigned>(__double2hiint(p)) ^ static_cast<unsigned>(__double2hiint(q))) >> 31);
}
__device__ __forceinline__ int sturm_count_prod(const double* d, const double* e2, int n, double x) {
  double p2 = 1.0;
  double p1 = d[0] - x;
  int cnt = sign_flip(p1, p2);
  int k = 1;
  for (; k + 4 <= n; k += 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double p = fma(d[k + u] - x, p1, -(e2[k + u - 1] * p2));
      cnt += sign_flip(p, p1);
      p2 = p1;
      p1 = p;
    }
    const int ex = static_cast<int>((__double_as_longlong(fmax(fabs(p1), fabs(p2))) >> 52) & 0x7ff) - 1023;
    p1 = ldexp(p1, -ex);
    p2 = ldexp(p2, -ex);
  }
  for (; k < n; ++k) {
    const double p = fma(d[k] - x, p1, -(e2[k - 1] * p2));
    cnt += sign_flip(p, p1);
    p2 = p1;
    p1 = p;
  }
  return cnt;
}

// TORCHEVAL_AMD_SYMEIG_STURM: the count both eigenvalue kernels use (they must agree: the
// multisection starts from the grid's cells).  1 = product form (default), 0 = ratio form.
#ifndef TEA_STURM_PROD
#define TEA_STURM_PROD 1
#endif
__device__ __forceinline__ int sturm_count_any(const double* d, const double* e2, int n, double x, double pivmin) {
#if TEA_STURM_PROD
  (void)pivmin;
  return sturm_count_prod(d, e2, n, x);
#else
  return sturm_count(d, e2, n, x, pivmin);
#endif
}

constexpr int kEigMaxN = 2560;

// Sturm-count grid: kGrid points evenly spaced inside the Gershgorin interval, one count per
// lane in one launch (1024 waves, about the time of one multisection round).  Every eigenvalue
// then starts from the grid cell that holds it (a binary search of the counts) instead of the
// whole interval: log16(65536) = 4 of the ~13 sixteen-point rounds, for one round's time.
constexpr int kGrid = 65536;

struct Bounds {
  double a, b, pivmin, span;
  double inv_scale;  // the arrays (and a, b, pivmin, span) are in units of 1 / inv_scale
};

// d, e^2 into LDS and the widened Gershgorin interval (block-cooperative; every kernel that
// calls it computes bitwise the same bounds, so grid points match across launches)
// min / max that propagate NaN (fmin / fmax drop it): a NaN anywhere in the tridiagonal makes
// the interval NaN, so every eigenvalue comes out NaN (torch's eigvalsh of a NaN matrix does
// not return finite numbers either) instead of a bisection over garbage counts
__device__ __forceinline__ double nan_min(double a, double b) { return (a != a || b != b) ? a + b : fmin(a, b); }
__device__ __forceinline__ double nan_max(double a, double b) { return (a != a || b != b) ? a + b : fmax(a, b); }

__device__ Bounds tridiag_setup(const double* __restrict__ d_in, const double* __restrict__ e_in, int n,
                                double* d, double* e2, double (*red)[kWaves]) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  double lo = DBL_MAX, hi = -DBL_MAX, emax = 0.0;
  for (int k = t; k < n; k += kThreads) {
    const double dk = d_in[k];
    const double ek = k + 1 < n ? fabs(e_in[k]) : 0.0;
    const double ep = k > 0 ? fabs(e_in[k - 1]) : 0.0;
    d[k] = dk;
    e2[k] = ek * ek;
    lo = nan_min(lo, dk - ek - ep);
    hi = nan_max(hi, dk + ek + ep);
    emax = fmax(emax, ek * ek);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = nan_min(lo, __shfl_xor(lo, o, 64));
    hi = nan_max(hi, __shfl_xor(hi, o, 64));
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
    lo = nan_min(lo, red[0][w]);
    hi = nan_max(hi, red[1][w]);
    emax = fmax(emax, red[2][w]);
  }
  Bounds r;
  r.inv_scale = 1.0;
#if TEA_STURM_PROD
  {
    // scale by a power of two (exact) so the Gershgorin span is in [1, 2): the product-form
    // count's growth bound; every e^2 raised to at least 2^-600 (zeros included: the count is
    // then exact for a matrix within 2^-300 of this one, far below rounding)
    const double sp = fmax(fabs(lo), fabs(hi));
    if (sp == 0.0) {  // the zero matrix: only the e^2 floor (every minor would be an exact zero)
      for (int k = t; k < n; k += kThreads) e2[k] = 0x1p-600;
      emax = 0x1p-600;
    } else if (sp <= DBL_MAX) {
      const int ex = static_cast<int>((__double_as_longlong(sp) >> 52) & 0x7ff) - 1023;
      if (ex > -1000) {
        const double sc = ldexp(1.0, -ex), sc2 = sc * sc;
        for (int k = t; k < n; k += kThreads) {
          d[k] *= sc;
          const double x = e2[k] * sc2;
          e2[k] = x < 0x1p-600 ? 0x1p-600 : x;
        }
        lo *= sc;
        hi *= sc;
        emax *= sc2;
        r.inv_scale = ldexp(1.0, ex);
      }
    }
    __syncthreads();
  }
#endif
  r.pivmin = DBL_MIN * fmax(1.0, emax);
  r.span = fmax(fabs(lo), fabs(hi));
  // widen so count(a) = 0 and count(b) = n hold despite rounding
  r.a = lo - 2.0 * DBL_EPSILON * r.span * n - 2.0 * r.pivmin;
  r.b = hi + 2.0 * DBL_EPSILON * r.span * n + 2.0 * r.pivmin;
  return r;
}

__device__ __forceinline__ double grid_x(const Bounds& q, int g) {
  return q.a + (q.b - q.a) * (double)(g + 1) / (double)(kGrid + 1);
}

__global__ __launch_bounds__(kThreads) void sturm_grid_kernel(const double* __restrict__ d_in,
                                                              const double* __restrict__ e_in, int n,
                                                              int* counts) {
  __shared__ double d[kEigMaxN], e2[kEigMaxN];
  __shared__ double red[3][kWaves];
  const Bounds q = tridiag_setup(d_in, e_in, n, d, e2, red);
  const int g = blockIdx.x * kThreads + threadIdx.x;
  if (g < kGrid) counts[g] = sturm_count_any(d, e2, n, grid_x(q, g), q.pivmin);
}

// L lanes per eigenvalue index i (ascending): L-point multisection of the eigenvalue's grid cell
// keeping count(a) <= i < count(b).
template <int L>
__global__ __launch_bounds__(kThreads) void tridiag_eigvals_kernel(const double* __restrict__ d_in,
                                                                   const double* __restrict__ e_in,
                                                                   int n, const int* __restrict__ counts,
                                                                   double* lam) {
  __shared__ double d[kEigMaxN], e2[kEigMaxN];
  __shared__ double red[3][kWaves];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const Bounds q = tridiag_setup(d_in, e_in, n, d, e2, red);
  const double pivmin = q.pivmin, span = q.span;
  // L lanes per eigenvalue, 64 / L eigenvalues per wave (fewer lanes: more rounds but less
  // Sturm work in all; the launcher picks L, see launch_symeig).
  constexpr int kPer = 64 / L;
  const int grp = lane / L, sub = lane % L;
  const int idx = (blockIdx.x * kWaves + wave) * kPer + grp;
  if ((blockIdx.x * kWaves + wave) * kPer >= n) return;  // whole wave idle; no barrier below
  bool done = idx >= n;
  // the grid cell: g* = first grid index whose count exceeds idx (count at the top end = n)
  int glo = 0, ghi = kGrid;
  while (glo < ghi) {
    const int mid = (glo + ghi) >> 1;
    if (counts[mid] > idx) ghi = mid;
    else glo = mid + 1;
  }
  double a = glo == 0 ? q.a : grid_x(q, glo - 1);
  double b = glo == kGrid ? q.b : grid_x(q, glo);
  for (int round = 0; round < 20; ++round) {
    const double width = b - a;
    // absolute tolerance eps * ||T|| (the accuracy any backward-stable solver delivers)
    done = done || width <= DBL_EPSILON * span + 2.0 * DBL_EPSILON * fmax(fabs(a), fabs(b)) + pivmin;
    if (__all(done)) break;
    const double x = a + width * (double)(sub + 1) / (double)(L + 1);
    const int c = sturm_count_any(d, e2, n, x, pivmin);
    const unsigned long long above = __ballot(c > idx);
    const unsigned long long gm = L == 64 ? above : (above >> (L * grp)) & ((1ull << (L % 64)) - 1ull);
    const int first = gm ? __ffsll((long long)gm) - 1 : L;
    const double xa = __shfl(x, L * grp + (first > 0 ? first - 1 : 0), 64);
    const double xb = __shfl(x, L * grp + (first < L ? first : L - 1), 64);
    if (!done) {
      if (first > 0) a = xa;
      if (first < L) b = xb;
    }
  }
  if (sub == 0 && idx < n) lam[idx] = 0.5 * (a + b) * q.inv_scale;
}

}  // namespace

int symeig_plan(int64_t n, int* grid, int* rows_per_block) {
  if (n < 3 || n > (int64_t)kMaxCols * kThreads || n > kEigMaxN) return 1;
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 2;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 2;
  int64_t R = (n + cus - 1) / cus;
  if (R > kMaxRows) return 1;
  *grid = (int)((n + R - 1) / R);
  *rows_per_block = (int)R;
  return 0;
}

int64_t symeig_slot_stride(int64_t n) { return (n + 15) / 16 * 16; }

int64_t symeig_grid_bytes() { return (int64_t)kGrid * sizeof(int); }

int64_t symeig_tail_bytes() { return (int64_t)kTail * kTail * sizeof(double); }

int64_t symeig_slot_bytes(int64_t n) { return 2 * (n - 2) * symeig_slot_stride(n) * (int64_t)sizeof(unsigned long long); }

int launch_symeig(const SymEigArgs& a, hipStream_t stream) {
  int G = 0, R = 0;
  if (symeig_plan(a.n, &G, &R) != 0) return 1;
  // K9b v2 (rows per wave) only on TORCHEVAL_AMD_SYMEIG_WAVE=1, and only when the grid of
  // n / 8 workgroups fits the device's CUs and the row fits 32 columns per lane (n <= 2048):
  // measured slower than tridiag_kernel (18.5 vs 14.7 ms at D = 2048,
  // profiles/symeig_wave_ab_r5.json), kept as the A/B arm
  static const bool wave_mode = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_WAVE");
    return e && e[0] == '1';
  }();
  const void* wkern = nullptr;
  int GW = 0;
  if (wave_mode && a.n <= 2048) {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
        (a.n + kWRows - 1) / kWRows <= cus) {
      GW = (int)((a.n + kWRows - 1) / kWRows);
      wkern = a.n <= 512    ? reinterpret_cast<const void*>(&tridiag_wave_kernel<8>)
              : a.n <= 1024 ? reinterpret_cast<const void*>(&tridiag_wave_kernel<16>)
              : a.n <= 1536 ? reinterpret_cast<const void*>(&tridiag_wave_kernel<24>)
                            : reinterpret_cast<const void*>(&tridiag_wave_kernel<32>);
    }
  }
  // the smallest instance holding ceil(n / 256) columns and R rows per thread: every register
  // slot is live (the pass has no per-element column test), e.g. 8 x 8 for the FID's D = 2048
  const int need = (int)max((a.n + kThreads - 1) / kThreads, (int64_t)R);
  const void* kern = need <= 2   ? reinterpret_cast<const void*>(&tridiag_kernel<2, 2>)
                     : need <= 4 ? reinterpret_cast<const void*>(&tridiag_kernel<4, 4>)
                     : need <= 6 ? reinterpret_cast<const void*>(&tridiag_kernel<6, 6>)
                     : need <= 8 ? reinterpret_cast<const void*>(&tridiag_kernel<8, 8>)
                     : need <= 9 ? reinterpret_cast<const void*>(&tridiag_kernel<9, 9>)
                                 : reinterpret_cast<const void*>(&tridiag_kernel<kMaxCols, kMaxRows>);
  // 512-thread workgroups over the same rows (two waves per SIMD, half the columns per thread)
  // where the 256-thread instance is the 8 x 8 one (1536 < n <= 2048, the FID's D = 2048): that
  // instance holds 256 VGPRs + AGPRs at one wave per SIMD, and every dependent FP64 chain of the
  // pass and the reductions stalls; 512 threads: 12.9 vs 14.7 ms at D = 2048, but 2-5% slower at
  // D = 512 / 1000, where the 256-thread instances are small (profiles/symeig_nt_ab_r5.json).
  // TORCHEVAL_AMD_SYMEIG_NT=256 / 512 / 1024 forces a size (A/B; 1024 measured slower everywhere)
  static const int nt_env = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_NT");
    return e ? std::atoi(e) : 0;
  }();
  int nt = kThreads;
  if (nt_env == 512 || (nt_env == 0 && need > 6 && need <= 8)) {
    const int64_t c = (a.n + 511) / 512;
    const void* k512 = (c <= 1 && R <= 2)    ? reinterpret_cast<const void*>(&tridiag_kernel<1, 2, 512>)
                       : (c <= 2 && R <= 4)  ? reinterpret_cast<const void*>(&tridiag_kernel<2, 4, 512>)
                       : (c <= 3 && R <= 6)  ? reinterpret_cast<const void*>(&tridiag_kernel<3, 6, 512>)
                       : (c <= 4 && R <= 8)  ? reinterpret_cast<const void*>(&tridiag_kernel<4, 8, 512>)
                                             : nullptr;  // (5 x 10 spills: n > 2048 stays at 256)
    if (k512) {
      kern = k512;
      nt = 512;
    }
  } else if (nt_env == 1024) {
    const int64_t c = (a.n + 1023) / 1024;
    const void* k1k = (c <= 1 && R <= 2)    ? reinterpret_cast<const void*>(&tridiag_kernel<1, 2, 1024>)
                      : (c <= 1 && R <= 4)  ? reinterpret_cast<const void*>(&tridiag_kernel<1, 4, 1024>)
                      : (c <= 2 && R <= 8)  ? reinterpret_cast<const void*>(&tridiag_kernel<2, 8, 1024>)
                                            : nullptr;  // (3 x 10 spills: n > 2048 stays at 256)
    if (k1k) {
      kern = k1k;
      nt = 1024;
    }
  }
  if (hipMemsetAsync(a.ctl, 0, kCtlBytes, stream) != hipSuccess) return 2;
  if (hipMemsetAsync(a.slots, 0xff, (size_t)symeig_slot_bytes(a.n), stream) != hipSuccess) return 2;
  const double* A = a.a;
  int n = (int)a.n;
  int64_t ld = a.ld;
  double *d = a.d, *e = a.e;
  unsigned long long* slots = a.slots;
  unsigned* ctl = a.ctl;
  // the last kTail columns in one workgroup (TORCHEVAL_AMD_SYMEIG_TAIL=0: the grid does all, A/B)
  static const bool tail_on = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_TAIL");
    return !(e && e[0] == '0');
  }();
  double* tail = a.tail;
  int jt = (tail_on && tail != nullptr && !wkern && n >= 2 * kTail) ? n - kTail : n;
  void* args[] = {&A, &n, &R, &ld, &d, &e, &slots, &ctl, &tail, &jt};
  void* wargs[] = {&A, &n, &ld, &d, &e, &slots, &ctl};
  // TORCHEVAL_AMD_SYMEIG_COOP=0: a plain launch of the same grid (A/B of the cooperative
  // launch's process-exit behaviour under rocprofv3; G <= #CUs workgroups are co-resident in
  // practice and the bounded hand-off spins abort to the library fallback if they are not)
  static const bool coop = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_COOP");
    return !(e && e[0] == '0');
  }();
  const void* lk = wkern ? wkern : kern;
  void** la = wkern ? wargs : args;
  const int lg = wkern ? GW : G;
  const int lt = wkern ? kThreads : nt;
  const hipError_t lrc = coop ? hipLaunchCooperativeKernel(lk, dim3(lg), dim3(lt), la, 0, stream)
                              : hipLaunchKernel(lk, dim3(lg), dim3(lt), la, 0, stream);
  if (lrc != hipSuccess) return 3;
  // tile height: TORCHEVAL_AMD_SYMEIG_TAIL_TR=8 (256 threads, the default) / 4 (512) / 2 (1024):
  // 210 / 217 / 280 us at D = 2048 (profiles/k9b_tail_r6.json)
  static const int tail_tr = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_TAIL_TR");
    const int v = e ? std::atoi(e) : 8;
    return (v == 2 || v == 4) ? v : 8;
  }();
  if (jt < n) {
    if (tail_tr == 8)
      symeig_tail_kernel<8><<<1, 16 * kTail / 8, 0, stream>>>(tail, n, d, e);
    else if (tail_tr == 2)
      symeig_tail_kernel<2><<<1, 16 * kTail / 2, 0, stream>>>(tail, n, d, e);
    else
      symeig_tail_kernel<4><<<1, 16 * kTail / 4, 0, stream>>>(tail, n, d, e);
  }
  sturm_grid_kernel<<<kGrid / kThreads, kThreads, 0, stream>>>(d, e, n, a.grid);
  // lanes per eigenvalue: 64 (with the product-form Sturm count 64 / 32 / 16 lanes take 394-397 /
  // 402-405 / 423-426 us at D = 2048, profiles/k9b_sturm_r6.json; the ratio form's 32 lanes had
  // edged out 16 and 64 there); TORCHEVAL_AMD_SYMEIG_L=16 / 32 / 64 forces (A/B)
  static const int l_env = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_SYMEIG_L");
    return e ? std::atoi(e) : 0;
  }();
  const int L = (l_env == 16 || l_env == 32 || l_env == 64) ? l_env : 64;
  if (L == 16)
    tridiag_eigvals_kernel<16><<<(n + kWaves * 4 - 1) / (kWaves * 4), kThreads, 0, stream>>>(d, e, n, a.grid, a.lam);
  else if (L == 32)
    tridiag_eigvals_kernel<32><<<(n + kWaves * 2 - 1) / (kWaves * 2), kThreads, 0, stream>>>(d, e, n, a.grid, a.lam);
  else
    tridiag_eigvals_kernel<64><<<(n + kWaves - 1) / kWaves, kThreads, 0, stream>>>(d, e, n, a.grid, a.lam);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea

// ------------------------------------------------------------------------------------------
// K9c: diagonal-block Cholesky + triangular inverse for the blocked FP64 Cholesky of FID's
// covariance (metrics/image/fid.py).  rocSOLVER's potrf at D = 2048 spent ~2.7 ms in 17
// potf2 launches (~160 us each) and ~1.7 ms in its forward-substitution trsm
// (profiles/rocprof_k9b_symeig_r2.csv); here one workgroup factors a b x b (b <= 64) diagonal
// block in registers (potf2, LAPACK semantics: a non-positive pivot records info = column + 1 and
// stops) and inverts the factor alongside, so the panel below becomes one GEMM with the inverse
// and the trailing update one GEMM (rocBLAS/hipBLASLt FP64 MFMA) - no trsm, no small-kernel
// chains.
namespace tea {
namespace {

constexpr int kPotrfB = 64;
// 16 x 16 threads, 4 x 4 entries each (4 waves): ~35 us per 64 x 64 block.  Measured
// alternatives: 32 x 32 threads with 2 x 2 entries 38 us (the 16-wave barrier costs more than
// the FMAs it spreads), one wave with 8 x 8 entries 79 us (VALU-bound, spills to AGPRs)
constexpr int kPG = 16;
constexpr int kPE = kPotrfB / kPG;

// Register-resident: thread (ti, tj) of a kPG x kPG grid holds L[ti + kPG x][tj + kPG y] and
// the same entries of X (x, y < kPE) in registers for the whole factorisation, and the column
// loop is unrolled so the pivot's register slot (j / kPG) is a compile-time index.  Per column
// ONE barrier: the threads holding column j of L / row j of X put their kPE values into an LDS
// snapshot (double-buffered, so the next column's writes never race this column's reads),
// every thread reads the snapshot entries its rows and columns need, and updates its entries
// in registers (right-looking potf2 on the lower triangle, the same elimination applied to the
// identity).  Round 2's form kept L and X in LDS and re-read / re-wrote them every column: ~80
// LDS operations per thread per column, 76 us per 64 x 64 block.
__global__ __launch_bounds__(kPG * kPG) void potrf_block_kernel(double* A, int64_t lda, int k0, int b,
                                                          double* Linv, int* info) {
  __shared__ double s_col[2][kPotrfB];  // column j of L (unscaled), per step parity
  __shared__ double s_xr[2][kPotrfB];   // row j of X (unscaled)
  const int t = threadIdx.x;
  const int ti = t / kPG, tj = t % kPG;
  double* blk = A + (int64_t)k0 * lda + k0;
  double L[kPE][kPE], X[kPE][kPE];
#pragma unroll
  for (int x = 0; x < kPE; ++x)
#pragma unroll
    for (int y = 0; y < kPE; ++y) {
      const int i = ti + kPG * x, k = tj + kPG * y;
      L[x][y] = (i < b && k <= i) ? blk[(int64_t)i * lda + k] : 0.0;
      X[x][y] = (i == k && i < b) ? 1.0 : 0.0;
    }
  // fully unrolled (no early exit: a break kept the loop rolled, and the pivot slot then went
  // through dynamic register indexing - 164 us per block)
  bool bad = false;
#pragma clang loop unroll(full)
  for (int j = 0; j < kPotrfB; ++j) {
    if (j < b && !bad) {  // block-uniform
      const int q = j / kPG, c = j % kPG, buf = j & 1;
      if (tj == c) {
#pragma unroll
        for (int x = 0; x < kPE; ++x) s_col[buf][ti + kPG * x] = L[x][q];
      }
      if (ti == c) {
#pragma unroll
        for (int y = 0; y < kPE; ++y) s_xr[buf][tj + kPG * y] = X[q][y];
      }
      __syncthreads();
      const double d = s_col[buf][j];
      if (!(d > 0.0)) {  // not positive definite (or NaN): LAPACK info, then stop
        if (t == 0 && *info == 0) *info = k0 + j + 1;
        bad = true;
      } else {
        // 1/sqrt(d) from the hardware estimate + two Newton steps (a handful of FMAs on the
        // per-column critical path instead of the IEEE sqrt and division sequences)
        double rs = __builtin_amdgcn_rsq(d);
        rs = fma(0.5 * rs, fma(-d * rs, rs, 1.0), rs);
        rs = fma(0.5 * rs, fma(-d * rs, rs, 1.0), rs);
        const double sq = d * rs, rd = rs * rs;
        // masked coefficients instead of per-element selects: rows i <= j and columns k <= j
        // take zero.  Entries above the diagonal (k > i) take updates too: they are never read
        // (a column snapshot's rows above its pivot are masked here) and are zeroed on output.
        // X needs no column mask: row j of X is zero past column j.
        double ci[kPE], ck[kPE], xr[kPE];
#pragma unroll
        for (int x = 0; x < kPE; ++x) ci[x] = ti + kPG * x > j ? s_col[buf][ti + kPG * x] * rd : 0.0;
#pragma unroll
        for (int y = 0; y < kPE; ++y) {
          ck[y] = tj + kPG * y > j ? s_col[buf][tj + kPG * y] : 0.0;
          xr[y] = s_xr[buf][tj + kPG * y];
        }
#pragma unroll
        for (int x = 0; x < kPE; ++x) {
#pragma unroll
          for (int y = 0; y < kPE; ++y) {
            L[x][y] = fma(-ci[x], ck[y], L[x][y]);
            X[x][y] = fma(-ci[x], xr[y], X[x][y]);
          }
        }
        // finish column j of L and row j of X (the snapshot the other threads read is unscaled)
        if (tj == c) {
#pragma unroll
          for (int x = 0; x < kPE; ++x) {
            const int i = ti + kPG * x;
            L[x][q] = i > j ? L[x][q] * rs : (i == j ? sq : L[x][q]);
          }
        }
        if (ti == c) {
#pragma unroll
          for (int y = 0; y < kPE; ++y) X[q][y] = tj + kPG * y <= j ? X[q][y] * rs : X[q][y];
        }
      }
    }
  }
#pragma unroll
  for (int x = 0; x < kPE; ++x)
#pragma unroll
    for (int y = 0; y < kPE; ++y) {
      const int i = ti + kPG * x, k = tj + kPG * y;
      if (i < b && k < b) {
        blk[(int64_t)i * lda + k] = k <= i ? L[x][y] : 0.0;
        Linv[(int64_t)i * b + k] = bad ? 0.0 : X[x][y];
      }
    }
}

}  // namespace

int potrf_block_size() { return kPotrfB; }

int launch_potrf_block(double* A, int64_t lda, int k0, int b, double* Linv, int* info,
                       hipStream_t stream) {
  if (b < 1 || b > kPotrfB) return 1;
  potrf_block_kernel<<<1, kPG * kPG, 0, stream>>>(A, lda, k0, b, Linv, info);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

}  // namespace tea
