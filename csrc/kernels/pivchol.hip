// K9p: pivoted (rank-revealing) FP64 Cholesky for rank-deficient FID covariances.
//
// Reference: torcheval/metrics/image/fid.py:192-230 takes tr sqrt(S1 S2) of any rank through
// torch.linalg.eigvals of the product.  Round 5 factored a singular S1 (fewer samples than
// features, so no Cholesky factor) through rocSOLVER's eigh with eigenvectors: 88-100 ms at
// D = 2048.  Here S1 = W^T W with W [r, D] from greedy diagonal pivoting (LAPACK dpstrf
// semantics: pivot on the largest remaining Schur-complement diagonal, stop once it is <= tol =
// D eps max diag S1), and W S2 W^T (r x r) carries the non-zero spectrum of S1 S2 for K9b.  W's
// rows stay in the original feature order (row j of W = column j of the factor, P L), so no
// permutation is ever applied.
//
// MI355X design: the trailing matrix never leaves the chip.  One cooperative launch, one
// 256-thread workgroup per CU; workgroup g keeps R = ceil(D / G) <= 8 whole rows of the matrix in
// LDS (8 x 2048 x 8 B = 128 KB at D = 2048 on 256 CUs) and wave 0 of each workgroup runs the
// pivot rounds for its rows.  A round takes up to 4 columns with TWO cross-CU exchanges:
//  * A: every workgroup publishes its 4 best (Schur diagonal, feature) candidates, one packed
//    word each (the diagonal's bits with the feature in its low mantissa bits: ranking only);
//    each wave 0 reads all 4 G words (16 per lane, re-polled together) and picks the round's 4
//    best with DPP row reductions and gfx950's permlane16 / permlane32 swaps - every workgroup
//    the same, ties to the lower feature;
//  * B: each chosen candidate's owner publishes its row of the 4 x 4 block A'(p_a, p_b) (its own
//    LDS row), its panel values and its exact diagonal; every workgroup factors the block with
//    relaxed pivoting (candidate a is taken while its Schur diagonal after the earlier ones is
//    >= 1/4 of the round's first, i.e. within a factor 4 of the greedy choice; the first is the
//    exact greedy pivot) and forms its rows' values l_i,a from its LDS rows (A'(i, p_a) =
//    A'(p_a, i)), publishing them as rows of W;
//  * after 16 columns all 4 waves apply the panel's rank-16 update to the LDS rows, reading the
//    panel's W rows with plain loads behind one acquire (L2-served, 256 KB per XCD).
// (One pivot per exchange took 6.3 ms at D = 2048, rank 999; the 4-pivot rounds 4.4 ms,
// profiles/fid_singular_k9p_r6.json.)  Hand-offs are sentinel words (round 3's K9b form: the
// slots and W are filled with all-one bytes, a NaN pattern no stored value carries, and every
// value is written once with an agent-scope store; consumers poll until none is the sentinel).
// Every spin is bounded and raises an abort word; the host then falls back to eigh.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdint>

#include "tea_kernels.h"

namespace tea {
namespace {

constexpr int kPT = 256;  // threads per workgroup
constexpr int kNB = 16;   // panel width
constexpr int kRMax = 8;  // rows per workgroup
constexpr int kNMax = 2048;
constexpr unsigned kSpin = 1u << 20;
constexpr unsigned long long kSent = ~0ull;

typedef __attribute__((address_space(1))) unsigned pg_u32;
typedef __attribute__((address_space(1))) unsigned long long pg_u64;

struct PcArgs {
  const double* a;  // input, row-major
  int64_t lda;
  int n;
  int N;  // row stride of the LDS rows and of W (n padded to 64)
  int R;  // rows per workgroup
  unsigned long long* slots;  // [G] max diagonals, then [n][G][kSlotW] candidates (sentinel-filled)
  unsigned long long* w;      // [N, N] doubles: row j = factor column j (sentinel-filled)
  int* piv;                   // [n] pivot features
  int* info;                  // {rank, status: 1 NaN in the matrix, 2 aborted}
  unsigned* ctl;              // {abort}
  unsigned long long* trace;  // optional stamps (launch_pivchol)
};

__device__ __forceinline__ unsigned long long bits_of(double x) {
  return x != x ? 0x7ff8000000000000ull : static_cast<unsigned long long>(__double_as_longlong(x));
}
__device__ __forceinline__ double dbl(unsigned long long b) { return __longlong_as_double(static_cast<long long>(b)); }
__device__ __forceinline__ void put(unsigned long long* g, unsigned long long b) {
  __hip_atomic_store((pg_u64*)g, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long get(const unsigned long long* g) {
  return __hip_atomic_load((pg_u64*)const_cast<unsigned long long*>(g), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// re-read *g until it is not the sentinel; false on abort / timeout (which raises the abort word)
__device__ __forceinline__ bool wait_word(const unsigned long long* g, unsigned long long& v, unsigned* abort_w) {
  for (unsigned it = 0; v == kSent; ++it) {
    if ((it & 31) == 31 &&
        __hip_atomic_load((pg_u32*)abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
      return false;
    if (it > kSpin) {
      __hip_atomic_store((pg_u32*)abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
    v = get(g);
  }
  return true;
}

// (v, i) beats (bv, bi): larger v, ties to the lower feature (a total order: deterministic)
__device__ __forceinline__ bool better(double v, int i, double bv, int bi) { return v > bv || (v == bv && i < bi); }

template <int Ctrl>
__device__ __forceinline__ void dpp_cand(double& v, int& i) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), Ctrl, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), Ctrl, 0xf, 0xf, false);
  const int pi = __builtin_amdgcn_update_dpp(0, i, Ctrl, 0xf, 0xf, false);
  const double pv = __hiloint2double(hi, lo);
  if (better(pv, pi, v, i)) {
    v = pv;
    i = pi;
  }
}

// the two outputs of a permlane swap with both operands x are x and its partner's x
template <bool K32>
__device__ __forceinline__ void swap_cand(double& v, int& i) {
  const unsigned lo = static_cast<unsigned>(__double2loint(v)), hi = static_cast<unsigned>(__double2hiint(v));
  const unsigned ui = static_cast<unsigned>(i);
  const auto a = K32 ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false) : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto b = K32 ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false) : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const auto c = K32 ? __builtin_amdgcn_permlane32_swap(ui, ui, false, false) : __builtin_amdgcn_permlane16_swap(ui, ui, false, false);
  const double v0 = __hiloint2double(static_cast<int>(b[0]), static_cast<int>(a[0]));
  const double v1 = __hiloint2double(static_cast<int>(b[1]), static_cast<int>(a[1]));
  const int i0 = static_cast<int>(c[0]), i1 = static_cast<int>(c[1]);
  if (better(v1, i1, v0, i0)) {
    v = v1;
    i = i1;
  } else {
    v = v0;
    i = i0;
  }
}

// every lane gets the wave's best (v, i)
__device__ __forceinline__ void wave_argmax(double& v, int& i) {
  dpp_cand<0xB1>(v, i);   // quad_perm [1,0,3,2]
  dpp_cand<0x4E>(v, i);   // quad_perm [2,3,0,1]
  dpp_cand<0x141>(v, i);  // row_half_mirror
  dpp_cand<0x140>(v, i);  // row_mirror
  swap_cand<false>(v, i);
  swap_cand<true>(v, i);
}

constexpr int kBP = 4;         // pivots chosen per round (block)
constexpr int kAW = kBP;       // A-slot words per workgroup and round: 4 packed (Schur diagonal, feature)
constexpr int kBW = kBP + kNB + 1;  // B-slot words per chosen pivot: its block row, panel values, exact diagonal
// a round's later pivot is taken while its Schur diagonal (after the earlier ones of the round) is
// at least kEta x the round's first: within that factor of the greedy choice (relaxed pivoting)
constexpr double kEta = 0.25;

__device__ __forceinline__ unsigned long long* slot_a(const PcArgs& a, int s, int g) {
  return a.slots + gridDim.x + (static_cast<int64_t>(s) * gridDim.x + g) * kAW;
}
__device__ __forceinline__ unsigned long long* slot_b(const PcArgs& a, int s, int w) {
  return a.slots + gridDim.x + static_cast<int64_t>(a.n) * gridDim.x * kAW + (static_cast<int64_t>(s) * kBP + w) * kBW;
}

// a candidate as ONE word: the Schur diagonal's bits with its low 11 mantissa bits replaced by
// 2047 - feature (n <= 2048), so the words order by value and then by lower feature - for ranking
// only (the exact diagonal of a chosen pivot comes with its block row); "none" = -inf, field 0
__device__ __forceinline__ unsigned long long pack_cand(double v, int i) {
  if (i == INT_MAX) return bits_of(-HUGE_VAL) & ~0x7ffull;
  // (a zero diagonal packs as a negative subnormal, so it never passes the tolerance test)
  return (bits_of(v > 0.0 ? v : (v == 0.0 ? -0.0 : v)) & ~0x7ffull) | static_cast<unsigned long long>(2047 - i);
}
__device__ __forceinline__ void unpack_cand(unsigned long long b, double& v, int& i) {
  v = dbl(b);
  i = (b & ~0x7ffull) == (bits_of(-HUGE_VAL) & ~0x7ffull) ? INT_MAX : 2047 - static_cast<int>(b & 0x7ffull);
}

#define PC_STAMP(idx)                                                                         \
  do {                                                                                        \
    if (a.trace != nullptr && blockIdx.x == 0 && lane == 0) a.trace[(idx)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// wave 0: publish this workgroup's 4 best (Schur diagonal, feature) candidates of round s.  With
// `drain`, the wave's write-through W stores drain first: a workgroup that has seen these
// candidates may read the finished panel's W rows with plain loads after one acquire.
__device__ __forceinline__ void publish_top(const PcArgs& a, int s, double d, bool live, int fi, bool drain) {
  const int lane = threadIdx.x & 63;
  bool taken = false;
  double cv[kBP];
  int ci[kBP];
#pragma unroll
  for (int t = 0; t < kBP; ++t) {
    double v = (live && !taken && d == d) ? d : -HUGE_VAL;  // (a NaN diagonal never wins: info reports it)
    int i = (live && !taken && d == d) ? fi : INT_MAX;
    wave_argmax(v, i);
    cv[t] = v;
    ci[t] = i;
    taken = taken || (i != INT_MAX && i == fi);
  }
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane < kBP) {
    double v = cv[0];
    int i = ci[0];
#pragma unroll
    for (int t = 1; t < kBP; ++t) {
      v = lane == t ? cv[t] : v;
      i = lane == t ? ci[t] : i;
    }
    put(slot_a(a, s, blockIdx.x) + lane, pack_cand(v, i));
  }
}

// wave 0: every workgroup's 4 candidates of round s (16 per lane, loads issued together) -> the
// round's 4 best, in order, in every lane
__device__ __forceinline__ bool poll_top(const PcArgs& a, int s, double (&cv)[kBP], int (&cp)[kBP], unsigned* abort_w) {
  const int lane = threadIdx.x & 63, G = gridDim.x;
  unsigned long long cb[4][kBP];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gg = lane + 64 * u;
#pragma unroll
    for (int t = 0; t < kBP; ++t) cb[u][t] = gg < G ? get(slot_a(a, s, gg) + t) : pack_cand(0.0, INT_MAX);
  }
  // re-read every still-sentinel word together, one round trip per pass (a word-at-a-time wait
  // paid a round trip per late word)
  bool ok = true;
  for (unsigned it = 0;; ++it) {
    bool pend = false;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int t = 0; t < kBP; ++t) pend = pend || cb[u][t] == kSent;
    if (!__any(pend)) break;
    if ((it & 31) == 31 &&
        __hip_atomic_load((pg_u32*)abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      ok = false;
      break;
    }
    if (it > kSpin) {
      __hip_atomic_store((pg_u32*)abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gg = lane + 64 * u;
#pragma unroll
      for (int t = 0; t < kBP; ++t)
        if (gg < G && cb[u][t] == kSent) cb[u][t] = get(slot_a(a, s, gg) + t);
    }
  }
  unsigned taken = 0;
#pragma unroll
  for (int t = 0; t < kBP; ++t) {
    double v = -HUGE_VAL;
    int i = INT_MAX;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < kBP; ++q) {
        double x;
        int xi;
        unpack_cand(cb[u][q], x, xi);
        if (!((taken >> (u * kBP + q)) & 1u) && better(x, xi, v, i)) {
          v = x;
          i = xi;
        }
      }
    wave_argmax(v, i);
    cv[t] = v;
    cp[t] = i;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int q = 0; q < kBP; ++q) {
        double x;
        int xi;
        unpack_cand(cb[u][q], x, xi);
        if (i != INT_MAX && xi == i) taken |= 1u << (u * kBP + q);
      }
  }
  return !__any(!ok);
}

__global__ __launch_bounds__(kPT) void pivchol_kernel(PcArgs a) {
  __shared__ double rows[kRMax * kNMax];
  __shared__ double sL[kRMax][kNB];
  __shared__ double sBv[kBP * kBW];  // wave 0: the round's block rows and panel values (B slots)
  __shared__ int s_state;  // 0 go on, 1 done, 2 aborted
  const int tid = threadIdx.x, lane = tid & 63;
  const int n = a.n, N = a.N, R = a.R, G = gridDim.x, g = blockIdx.x;
  const int f0 = g * R;
  unsigned* const abort_w = a.ctl;

  bool nanf = false;
  for (int r = 0; r < R; ++r) {
    const int i = f0 + r;
    for (int m = tid; m < N; m += kPT) {
      const double x = (i < n && m < n) ? a.a[static_cast<int64_t>(i) * a.lda + m] : 0.0;
      nanf |= x != x;
      rows[r * N + m] = x;
    }
  }
  if (tid == 0) s_state = 0;
  if (__syncthreads_or(nanf) != 0 && tid == 0) atomicOr(&a.info[1], 1);

  // wave 0 state: lane r < R holds feature f0 + r
  const int fi = f0 + lane;
  bool live = false;
  double d = -HUGE_VAL;
  double Lr[kNB];
#pragma unroll
  for (int q = 0; q < kNB; ++q) Lr[q] = 0.0;
  double tol = 0.0;
  int rank = 0;
  int j = 0, s = 0;  // next factor column, round
  double cv[kBP];    // wave 0: the current round's candidates (Schur diagonal, feature), best first
  int cp[kBP];
  if (tid < 64) {
    if (lane < R && fi < n) {
      d = rows[lane * N + fi];
      live = true;
    }
    // tolerance n eps max diag: every workgroup's maximum, exchanged once
    double m = (live && d > 0.0) ? d : 0.0;
    int dummy = 0;
    wave_argmax(m, dummy);
    if (lane == 0) put(a.slots + g, bits_of(m));
    double mx = 0.0;
    bool ok = true;
    for (int u = lane; u < G; u += 64) {
      unsigned long long b = get(a.slots + u);
      ok = ok && wait_word(a.slots + u, b, abort_w);
      const double x = dbl(b);
      mx = x > mx ? x : mx;
    }
    wave_argmax(mx, dummy);
    tol = static_cast<double>(n) * DBL_EPSILON * mx;
    if (__any(!ok) && lane == 0) s_state = 2;
    publish_top(a, 0, d, live, fi, false);
    if (!poll_top(a, 0, cv, cp, abort_w) && lane == 0) s_state = 2;
  }
  __syncthreads();

  for (int P = 0; s_state == 0; ++P) {
    const int j0 = P * kNB;
    if (tid < 64) {
      int state = 0;
      int k = 0;  // columns of this panel done (uniform: Lr[k] is register-indexed)
      while (k < kNB) {
        if (j >= n) {
          state = 1;
          break;
        }
        if (!(cv[0] > tol)) {  // every remaining Schur diagonal <= tol (or none left): rank j
          state = 1;
          break;
        }
        if (s < 8 && P < 4) PC_STAMP(2 * (P * 8 + (s & 7)));
        // candidates this round may take: leading ones above tol, within the panel and n
        int mmax = 1;
        while (mmax < kBP && mmax < kNB - k && j + mmax < n && cv[mmax] > tol && cp[mmax] != INT_MAX) ++mmax;
        // B: each chosen candidate's owner publishes its row of the block (A'(p_a, p_b)) and its
        // panel values; a single candidate at a panel's first column needs neither
        {  // (always: the chosen pivots' exact diagonals come with their block rows)
#pragma unroll
          for (int t = 0; t < kBP; ++t) {
            if (t < mmax && lane < R && fi == cp[t]) {  // this lane holds candidate t's row
              unsigned long long* sb = slot_b(a, s, t);
              put(sb + kBP + kNB, bits_of(d));
#pragma unroll
              for (int b = 0; b < kBP; ++b)
                if (b < mmax) put(sb + b, bits_of(rows[lane * N + cp[b]]));
#pragma unroll
              for (int q = 0; q < kNB; ++q)
                if (q < k) put(sb + kBP + q, bits_of(Lr[q]));
            }
          }
          // poll: word w = t * kBW + e over the needed ones, two per lane, into sBv
          bool ok = true;
          unsigned long long bw[2];
          bool need[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int wd = lane + 64 * h;
            const int t = wd / kBW, e = wd - t * kBW;
            need[h] = t < mmax && ((e < kBP && e < mmax) || (e >= kBP && e - kBP < k) || e == kBP + kNB);
            bw[h] = need[h] ? get(slot_b(a, s, t) + e) : 0ull;
          }
          for (unsigned it = 0;; ++it) {  // one round trip per pass over the late words
            const bool pend = (need[0] && bw[0] == kSent) || (need[1] && bw[1] == kSent);
            if (!__any(pend)) break;
            if (it > kSpin || ((it & 31) == 31 && __hip_atomic_load((pg_u32*)abort_w, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_AGENT) != 0u)) {
              if (it > kSpin) __hip_atomic_store((pg_u32*)abort_w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              ok = false;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const int wd = lane + 64 * h;
              const int t = wd / kBW, e = wd - t * kBW;
              if (need[h] && bw[h] == kSent) bw[h] = get(slot_b(a, s, t) + e);
            }
          }
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int wd = lane + 64 * h;
            if (wd < kBP * kBW) sBv[wd] = need[h] ? dbl(bw[h]) : 0.0;
          }
          if (__any(!ok)) {
            state = 2;
            break;
          }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // (one wave: its LDS stores land before its reads)
        // the block's factor with relaxed acceptance (uniform: every lane the same values)
        double lb[kBP][kBP];
#pragma unroll
        for (int t = 0; t < kBP; ++t)
#pragma unroll
          for (int b = 0; b < kBP; ++b) lb[t][b] = 0.0;
        double cx[kBP];  // the chosen pivots' exact Schur diagonals
#pragma unroll
        for (int t = 0; t < kBP; ++t) cx[t] = sBv[t * kBW + kBP + kNB];
        if (!(cx[0] > tol)) {  // (the exact diagonal: the ranking word dropped its low bits)
          state = 1;
          break;
        }
        lb[0][0] = sqrt(cx[0]);
        int m = 1;
#pragma unroll
        for (int t = 1; t < kBP; ++t) {
          if (t < mmax && m == t) {
            double dd = cx[t];
#pragma unroll
            for (int b = 0; b < kBP; ++b) {
              if (b < t) {
                double x = sBv[t * kBW + b];
                // all 16 panel terms, unconditionally: the words past k are zero (a runtime-bounded
                // loop waited an LDS round trip per term)
#pragma unroll
                for (int q = 0; q < kNB; ++q) x = fma(-sBv[t * kBW + kBP + q], sBv[b * kBW + kBP + q], x);
#pragma unroll
                for (int c = 0; c < kBP; ++c)
                  if (c < b) x = fma(-lb[t][c], lb[b][c], x);
                lb[t][b] = x / lb[b][b];
                dd = fma(-lb[t][b], lb[t][b], dd);
              }
            }
            if (dd > tol && dd >= kEta * cx[0]) {
              lb[t][t] = sqrt(dd);
              m = t + 1;
            }
          }
        }
        // this lane's row: its m new column values
        double lr[kBP];
#pragma unroll
        for (int t = 0; t < kBP; ++t) {
          double l = 0.0;
          if (t < m && live) {
            if (fi == cp[t]) {
              l = lb[t][t];
              live = false;
            } else {
              double x = rows[lane * N + cp[t]];
#pragma unroll
              for (int q = 0; q < kNB; ++q) x = fma(-Lr[q], sBv[t * kBW + kBP + q], x);  // (Lr past k: 0)
#pragma unroll
              for (int b = 0; b < kBP; ++b)
                if (b < t) x = fma(-lr[b], lb[t][b], x);
              l = x / lb[t][t];
              d = fma(-l, l, d);
            }
          }
          lr[t] = l;
          if (t < m) {
            Lr[k + t] = l;
            if (lane < R && fi < n) put(a.w + static_cast<int64_t>(j + t) * N + fi, bits_of(l));
            if (g == 0 && lane == 0) a.piv[j + t] = cp[t];
          }
        }
        if (s < 8 && P < 4) PC_STAMP(2 * (P * 8 + (s & 7)) + 1);
        j += m;
        k += m;
        rank = j;
        ++s;
        if (j < n) {
          publish_top(a, s, d, live, fi, k == kNB);
          if (!poll_top(a, s, cv, cp, abort_w)) {
            state = 2;
            break;
          }
        }
      }
      if (lane < R) {
#pragma unroll
        for (int q = 0; q < kNB; ++q) sL[lane][q] = Lr[q];
      }
#pragma unroll
      for (int q = 0; q < kNB; ++q) Lr[q] = 0.0;
      if (state == 0 && j >= n) state = 1;
      if (lane == 0) {
        s_state = state;
        if (state != 0 && g == 0) {
          a.info[0] = rank;
          if (state == 2) atomicOr(&a.info[1], 2);
        }
        // every workgroup's W stores of the panel drained before its next-round candidates,
        // which this wave has seen: one acquire, then the update reads the panel plainly
        if (state == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (s_state != 0) break;
    if (P < 4) PC_STAMP(64 + 2 * P);
    // rank-16 panel update of the LDS rows: A'[r][m] -= sum_q L[r][q] W[j0 + q][m] (plain,
    // L2-served loads behind the acquire: the 256 KB panel is fetched once per XCD; write-through
    // loads of it from every workgroup took 26 us per panel at D = 2048)
    for (int m0 = tid; m0 < n; m0 += 4 * kPT) {
      double b[4][kNB];
      const double* wd = reinterpret_cast<const double*>(a.w);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int m = m0 + u * kPT;
#pragma unroll
        for (int q = 0; q < kNB; ++q) b[u][q] = m < n ? wd[static_cast<int64_t>(j0 + q) * N + m] : 0.0;
      }
      for (int r = 0; r < R; ++r) {
        // the row's 16 panel values once per row (one LDS wait), then 4 independent FMA chains
        double c[kNB], acc[4];
#pragma unroll
        for (int q = 0; q < kNB; ++q) c[q] = sL[r][q];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = (m0 + u * kPT < n) ? rows[r * N + m0 + u * kPT] : 0.0;
#pragma unroll
        for (int q = 0; q < kNB; ++q)
#pragma unroll
          for (int u = 0; u < 4; ++u) acc[u] = fma(-c[q], b[u][q], acc[u]);
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (m0 + u * kPT < n) rows[r * N + m0 + u * kPT] = acc[u];
      }
    }
    __syncthreads();
    if (P < 4) PC_STAMP(64 + 2 * P + 1);
  }
}

int pc_cu_count() {
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return cus;
}

int pc_grid(int64_t n) { return static_cast<int>(n < pc_cu_count() ? n : pc_cu_count()); }

}  // namespace

int pivchol_padded(int64_t n) { return static_cast<int>((n + 63) / 64 * 64); }

int64_t pivchol_slot_words(int64_t n) {
  const int64_t G = n < 1 ? 1 : pc_grid(n);
  return G + n * G * kAW + n * kBP * kBW;  // tolerance words, A slots per round, B slots per round
}

// trace (optional, >= 80 words, s_memrealtime 100 MHz, workgroup 0): [2 (8 P + s % 8)] round start
// (candidates known) / [+1] its W rows stored, for panels P < 4; [64 + 2 P] / [+1] panel P's
// update start / end
int launch_pivchol(const double* A, int64_t lda, int64_t n, unsigned long long* slots, double* w, int* piv, int* info,
                   unsigned* ctl, hipStream_t stream, unsigned long long* trace) {
  if (n < 1 || n > kNMax) return 4;
  const int G = pc_grid(n);
  const int R = static_cast<int>((n + G - 1) / G);
  if (R > kRMax) return 4;
  const int N = pivchol_padded(n);
  if (hipMemsetAsync(ctl, 0, sizeof(unsigned), stream) != hipSuccess) return 2;
  if (hipMemsetAsync(info, 0, 2 * sizeof(int), stream) != hipSuccess) return 2;
  if (hipMemsetAsync(slots, 0xff, static_cast<size_t>(pivchol_slot_words(n)) * 8, stream) != hipSuccess) return 2;
  if (hipMemsetAsync(w, 0xff, static_cast<size_t>(N) * N * 8, stream) != hipSuccess) return 2;
  PcArgs a{A, lda, static_cast<int>(n), N, R, slots, reinterpret_cast<unsigned long long*>(w), piv, info, ctl, trace};
  void* args[] = {&a};
  if (hipLaunchCooperativeKernel(reinterpret_cast<const void*>(&pivchol_kernel), dim3(G), dim3(kPT), args, 0,
                                 stream) != hipSuccess) {
    (void)hipGetLastError();
    return 3;
  }
  return 0;
}

}  // namespace tea
