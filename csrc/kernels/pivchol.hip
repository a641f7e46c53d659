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
// column steps for its rows:
//  * every workgroup publishes its best (Schur diagonal, feature) candidate, together with that
//    feature's values in the current 16-column panel, to its own slot of the step;
//  * each wave 0 reads all G candidates (lanes poll 4 slots each), reduces them to the pivot p
//    with DPP row reductions and gfx950's permlane16 / permlane32 swaps (every workgroup gets
//    the same p: a total order, ties to the lower feature), reads the winner's panel values,
//    and forms its rows' column values l_i = (A'[i][p] - L[i][panel] . L[p][panel]) / sqrt(d_p)
//    locally (A'[i][p] = A'[p][i] is its own LDS row), publishing them as row j of W;
//  * after 16 columns all 4 waves apply the panel's rank-16 update to the LDS rows, reading the
//    panel's W rows (256 KB, the same for every workgroup).
// One cross-CU exchange per column (the candidates; the winner's panel values ride along), no
// trailing-matrix traffic to HBM.  Hand-offs are sentinel words (round 3's K9b form: the slots and
// W are filled with all-one bytes, a NaN pattern no stored value carries, and every value is
// written once with an agent-scope store; consumers poll until none is the sentinel).  Every spin
// is bounded and raises an abort word; the host then falls back to eigh.
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
constexpr int kSlotW = 2 + kNB;  // candidate slot: Schur diagonal, feature, its panel values
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

__device__ __forceinline__ unsigned long long* slot(const PcArgs& a, int j, int g) {
  return a.slots + gridDim.x + (static_cast<int64_t>(j) * gridDim.x + g) * kSlotW;
}

#define PC_STAMP(idx)                                                                         \
  do {                                                                                        \
    if (a.trace != nullptr && blockIdx.x == 0 && lane == 0) a.trace[(idx)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

// wave 0: publish this workgroup's candidate for step j (k = its column within the panel: the
// candidate's first k panel values ride along)
__device__ __forceinline__ void publish(const PcArgs& a, int j, int k, double d, bool live, int fi, const double (&Lr)[kNB]) {
  const int lane = threadIdx.x & 63;
  double v = live ? d : -HUGE_VAL;
  int i = live ? fi : INT_MAX;
  if (v != v) {  // a NaN diagonal never wins (the NaN is reported through info)
    v = -HUGE_VAL;
    i = INT_MAX;
  }
  wave_argmax(v, i);
  unsigned long long* s = slot(a, j, blockIdx.x);
  if (i != INT_MAX && fi == i) {
#pragma unroll
    for (int q = 0; q < kNB; ++q)
      if (q < k) put(s + 2 + q, bits_of(Lr[q]));
  }
  // at a panel's first step, the wave's write-through W stores of the panel drain before its
  // candidate is visible: a workgroup that has seen these candidates may read the panel's W rows
  // with plain loads after one acquire (the panel update).  (A drain on every step cost ~1 us.)
  if (k == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    put(s, bits_of(v));
    put(s + 1, static_cast<unsigned long long>(static_cast<unsigned>(i)));
  }
}

// wave 0: the G candidates of step j (4 slots per lane, loads issued together) -> the pivot
__device__ __forceinline__ bool poll_candidates(const PcArgs& a, int j, double& dp, int& p, unsigned* abort_w) {
  const int lane = threadIdx.x & 63, G = gridDim.x;
  unsigned long long vb[4], ib[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gg = lane + 64 * u;
    vb[u] = gg < G ? get(slot(a, j, gg)) : bits_of(-HUGE_VAL);
    ib[u] = gg < G ? get(slot(a, j, gg) + 1) : static_cast<unsigned long long>(INT_MAX);
  }
  bool ok = true;
  dp = -HUGE_VAL;
  p = INT_MAX;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int gg = lane + 64 * u;
    if (gg < G) {
      ok = ok && wait_word(slot(a, j, gg), vb[u], abort_w);
      ok = ok && wait_word(slot(a, j, gg) + 1, ib[u], abort_w);
    }
    if (better(dbl(vb[u]), static_cast<int>(ib[u]), dp, p)) {
      dp = dbl(vb[u]);
      p = static_cast<int>(ib[u]);
    }
  }
  wave_argmax(dp, p);
  return !__any(!ok);
}

__global__ __launch_bounds__(kPT) void pivchol_kernel(PcArgs a) {
  __shared__ double rows[kRMax * kNMax];
  __shared__ double sL[kRMax][kNB];
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
  double dp = -HUGE_VAL;  // wave 0: the current step's pivot (value, feature)
  int p = INT_MAX;
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
    publish(a, 0, 0, d, live, fi, Lr);
    if (!poll_candidates(a, 0, dp, p, abort_w) && lane == 0) s_state = 2;
  }
  __syncthreads();

  for (int P = 0; s_state == 0; ++P) {
    const int j0 = P * kNB;
    if (tid < 64) {
      int state = 0;
      for (int k = 0; k < kNB; ++k) {  // (k uniform: Lr[k] is register-indexed)
        const int j = j0 + k;
        if (j >= n) {
          state = 1;
          break;
        }
        if (k < 8 && P < 4) PC_STAMP(2 * (P * 8 + k));
        if (!(dp > tol)) {  // every remaining Schur diagonal <= tol (or none left): rank j
          rank = j;
          state = 1;
          break;
        }
        // the winner's panel values (published with its candidate)
        double x = 0.0;
        if (k > 0) {
          bool ok = true;
          const unsigned long long* ws = slot(a, j, p / R) + 2;
          unsigned long long b = kSent;
          if (lane < k) {
            b = get(ws + lane);
            ok = wait_word(ws + lane, b, abort_w);
            x = dbl(b);
          }
          if (__any(!ok)) {
            state = 2;
            break;
          }
        }
        double t = (lane < R) ? rows[lane * N + p] : 0.0;
        for (int q = 0; q < k; ++q) t = fma(-Lr[q], __shfl(x, q), t);
        const double sq = sqrt(dp);
        double l = 0.0;
        if (live) {
          if (fi == p) {
            l = sq;
            live = false;
          } else {
            l = t / sq;
            d = fma(-l, l, d);
          }
        }
        Lr[k] = l;
        if (lane < R && fi < n) put(a.w + static_cast<int64_t>(j) * N + fi, bits_of(l));
        if (g == 0 && lane == 0) a.piv[j] = p;
        rank = j + 1;
        if (k < 8 && P < 4) PC_STAMP(2 * (P * 8 + k) + 1);
        if (j + 1 < n) {
          publish(a, j + 1, k + 1 < kNB ? k + 1 : 0, d, live, fi, Lr);
          if (!poll_candidates(a, j + 1, dp, p, abort_w)) {
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
      if (state == 0 && j0 + kNB >= n) state = 1;
      if (lane == 0) {
        s_state = state;
        if (state != 0 && g == 0) {
          a.info[0] = rank;
          if (state == 2) atomicOr(&a.info[1], 2);
        }
        // every workgroup's step j0 + 15 W stores drained before its step j0 + 16 candidate,
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
    bool ok = true;
    if (__syncthreads_or(!ok) != 0) {
      if (tid == 0 && g == 0) atomicOr(&a.info[1], 2);
      break;
    }
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
  return G + n * G * kSlotW;
}

// trace (optional, >= 80 words, s_memrealtime 100 MHz, workgroup 0): [2 (8 P + k)] step start
// (pivot known) / [+1] its W row stored, for steps k < 8 of panels P < 4; [64 + 2 P] / [+1] panel
// P's update start / end
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
