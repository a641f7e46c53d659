// K3c: precision-recall curve emission and recall at fixed precision over score-sorted rows.
//
// Replaces the reference's post-sort chains
//   precision_recall_curve.py:156-182 (multiclass: diff != 0 -> pad -> flip -> masked select
//     -> cumsum x2 -> divide -> nan_to_num -> pad -> masked select, one .tolist() of sizes)
//   precision_recall_curve.py:207-231 (binary / per label: the same per row, plus a
//     torch.isnan(recall[0]) host read per row)
//   recall_at_fixed_precision.py:131-156 (max recall with precision >= p, best threshold; a
//     Python loop over labels for multilabel)
// with device passes over the K3a-sorted rows (the sort carries the target / label payload,
// so no gather):
//   1 count : per 1024-sample tile: totals of a = t, b = 1 - t (FP64) and the number of
//             tie-group tails (descending key i is a tail iff key[i+1] != key[i] or i = n-1,
//             the reference's `diff != 0` mask).
//   2 scan  : one block per row: exclusive scans of the tile totals and tail counts; row
//             totals P, N and G_r (tie groups) -> sizes[r].
//   curves  : the host reads sizes once (the reference's one .tolist()), allocates the exact
//             outputs and
//   3 emit  : per tile, LDS block scans give TP / FP at every tail and its global group index
//             g; tail g of row r lands at ascending position G_r - 1 - g:
//               precision = f32(TP) / f32(TP + FP), recall = f32(TP) / f32(P) (1 if P = 0,
//               the reference's nan_to_num), threshold = key;
//             block 0 writes the row's final (precision 1, recall 0) point.
//   RAFP (no host sync at all):
//   3' emit : per group, recall and threshold into [rows, n] scratch (descending group order);
//             the block's last group with precision >= f32(p) -> atomicMax gstar[r].
//   4  find : recall is non-decreasing along the descending scan, so the maximum over the
//             qualifying points is recall[gstar] and the points that reach it are one run of
//             groups; the run's first group (its highest threshold) -> atomicMin glo[r].
//   5  final: max recall, |best threshold| (the appended point, recall 0 / threshold -1,
//             competes when the maximum is 0), as the reference's torch.max over the masks.
// Precision and recall are rounded exactly as the reference's int64 / int64 true division in
// float32 (both operands rounded to f32, one IEEE division), so the curves match bit for bit.
#include "tea_common.h"
#include "tea_kernels.h"
#include "tea_scan.h"

namespace tea {

namespace {

using namespace k3;

// the reference's tie test is `sorted.diff() != 0`: adjacent +-inf (inf - inf = NaN) and NaNs
// start new groups, -0.0 and 0.0 share one; for finite keys x - y == 0 iff x == y
template <typename K>
__device__ __forceinline__ bool same_key(K x, K y) { return x - y == K(0); }

// per tile: (sum a, sum b) and the tie-group tail count; (!DIRECT) the gathered ab copy
template <typename K, bool DIRECT>
__global__ __launch_bounds__(kT) void curve_count_kernel(AucScanArgs a) {
  const int r = blockIdx.y;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  float2* ab = reinterpret_cast<float2*>(a.ab) + static_cast<int64_t>(r) * a.n;
  double sa = 0.0, sb = 0.0;
  int tails = 0;
  // clamped unconditional loads, masked after (a per-lane `if (i < n)` around loads compiles
  // to a branch + vmcnt(0) per element)
  float2 vv[kPer];
  K kc[kPer], kn[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = base + k * kT + threadIdx.x;  // coalesced
    const int64_t ic = i < a.n ? i : a.n - 1;
    vv[k] = sample_ab(a, r, ic);
    kc[k] = key_at<K>(a, r, ic);
    kn[k] = key_at<K>(a, r, ic + 1 < a.n ? ic + 1 : ic);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = base + k * kT + threadIdx.x;
    if (i < a.n) {
      if constexpr (!DIRECT) ab[i] = vv[k];
      sa += vv[k].x;
      sb += vv[k].y;
      tails += (i == a.n - 1 || !same_key<K>(kn[k], kc[k])) ? 1 : 0;
    }
  }
  __shared__ double lds[2][kT / 64];
  __shared__ int ldc[kT / 64];
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  tails = wave_sum(tails);
  if (lane_id() == 0) {
    lds[0][threadIdx.x >> 6] = sa;
    lds[1][threadIdx.x >> 6] = sb;
    ldc[threadIdx.x >> 6] = tails;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    D2 s{0.0, 0.0};
    int c = 0;
    for (int w = 0; w < kT / 64; ++w) {
      s = {s.x + lds[0][w], s.y + lds[1][w]};
      c += ldc[w];
    }
    const int64_t t = static_cast<int64_t>(r) * gridDim.x + blockIdx.x;
    reinterpret_cast<D2*>(a.tsum)[t] = s;
    a.tcnt[t] = c;
  }
}

// one block per row: exclusive scans of the tile totals / tail counts; row totals and G_r
__global__ __launch_bounds__(kT) void curve_scan_kernel(AucScanArgs a, int ntiles) {
  const int r = blockIdx.x;
  const int64_t row = static_cast<int64_t>(r) * ntiles;
  const D2* ts = reinterpret_cast<const D2*>(a.tsum) + row;
  D2* st = reinterpret_cast<D2*>(a.tstart) + row;
  __shared__ D2 lds[kT / 64];
  D2 carry{0.0, 0.0}, ccarry{0.0, 0.0};
  for (int b = 0; b < ntiles; b += kT) {
    const int t = b + threadIdx.x;
    const D2 v = t < ntiles ? ts[t] : D2{0.0, 0.0};
    const D2 c = {t < ntiles ? static_cast<double>(a.tcnt[row + t]) : 0.0, 0.0};
    D2 tot, ctot;
    const D2 ex = block_excl_scan(v, lds, tot);
    const D2 cex = block_excl_scan(c, lds, ctot);
    if (t < ntiles) {
      st[t] = d2add(carry, ex);
      a.cstart[row + t] = static_cast<int32_t>(ccarry.x + cex.x);
    }
    carry = d2add(carry, tot);
    ccarry = d2add(ccarry, ctot);
  }
  if (threadIdx.x == 0) {
    reinterpret_cast<D2*>(a.totals)[r] = carry;
    a.sizes[r] = static_cast<int64_t>(ccarry.x);
    if (a.gstar) {
      a.gstar[r] = -1;
      a.glo[r] = 0x7fffffff;
    }
  }
}

__device__ __forceinline__ float f32_recall(double tp, double P) {
  return P == 0.0 ? 1.f : static_cast<float>(tp) / static_cast<float>(P);
}

// per tile: TP / FP at every tail and its group index; curve points (RAFP=false) or the
// RAFP scratch + last qualifying group (RAFP=true)
template <typename K, bool DIRECT, bool RAFP>
__global__ __launch_bounds__(kT) void curve_emit_kernel(AucScanArgs a) {
  const int r = blockIdx.y;
  const int ntiles = gridDim.x;
  const int64_t tile = static_cast<int64_t>(r) * ntiles + blockIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  const float2* ab = reinterpret_cast<const float2*>(a.ab) + static_cast<int64_t>(r) * a.n;
  __shared__ D2 lds[kT / 64];
  __shared__ int s_best[kT / 64];

  const int j0 = threadIdx.x * kPer;
  const int64_t i0 = base + j0;
  K key[kPer];
  float2 v[kPer];
  // clamped unconditional loads, masked after
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = i0 + k < a.n ? i0 + k : a.n - 1;
    key[k] = key_at<K>(a, r, i);
    v[k] = load_ab<DIRECT>(a, ab, r, i);
  }
  K next_key = key_at<K>(a, r, i0 + kPer < a.n ? i0 + kPer : a.n - 1);
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const bool ok = i0 + k < a.n;
    key[k] = ok ? key[k] : K(0);
    v[k] = ok ? v[k] : make_float2(0.f, 0.f);
  }
  next_key = (i0 + kPer < a.n) ? next_key : K(0);
  const D2 t0 = reinterpret_cast<const D2*>(a.tstart)[tile];
  const int g0 = a.cstart[tile];
  const D2 tot_row = reinterpret_cast<const D2*>(a.totals)[r];
  const double P = tot_row.x;
  const int64_t G = a.sizes[r];

  bool tail[kPer];
  double la = 0.0, lb = 0.0, lc = 0.0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = i0 + k;
    const K nk = (k + 1 < kPer) ? key[k + 1] : next_key;
    tail[k] = i < a.n && (i == a.n - 1 || !same_key<K>(nk, key[k]));
    la += v[k].x;
    lb += v[k].y;
    lc += tail[k] ? 1.0 : 0.0;
  }
  D2 tot, ctot;
  const D2 ex = block_excl_scan(D2{la, lb}, lds, tot);
  const D2 cex = block_excl_scan(D2{lc, 0.0}, lds, ctot);
  double tp = t0.x + ex.x, fp = t0.y + ex.y;
  int g = g0 + static_cast<int>(cex.x);
  int best = -1;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    tp += v[k].x;
    fp += v[k].y;
    if (tail[k]) {
      const float prec = static_cast<float>(tp) / static_cast<float>(tp + fp);
      const float rec = f32_recall(tp, P);
      if constexpr (RAFP) {
        const int64_t o = static_cast<int64_t>(r) * a.n + g;
        a.s_rec[o] = rec;
        static_cast<K*>(a.s_thr)[o] = key[k];
        if (prec >= a.min_precision) best = g;
      } else {
        const int64_t pos = G - 1 - g;
        const int64_t toff = a.row_off[r];
        a.out_prec[toff + r + pos] = prec;
        a.out_rec[toff + r + pos] = rec;
        static_cast<K*>(a.out_thr)[toff + pos] = key[k];
      }
      ++g;
    }
  }
  if constexpr (RAFP) {
    int m = best;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = max(m, __shfl_xor(m, o, 64));
    if (lane_id() == 0) s_best[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
      int bm = -1;
      for (int w = 0; w < kT / 64; ++w) bm = max(bm, s_best[w]);
      if (bm >= 0) atomicMax(&a.gstar[r], bm);
    }
  } else {
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the final (precision 1, recall 0) point
      const int64_t toff = a.row_off[r];
      a.out_prec[toff + r + G] = 1.f;
      a.out_rec[toff + r + G] = 0.f;
    }
  }
}

// the first group (highest threshold) whose recall equals the maximum over qualifying points
__global__ __launch_bounds__(kT) void rafp_find_kernel(AucScanArgs a) {
  const int r = blockIdx.y;
  const int64_t G = a.sizes[r];
  const int64_t g0 = static_cast<int64_t>(blockIdx.x) * kTile;
  if (g0 >= G) return;
  const int gs = a.gstar[r];
  const float maxr = gs >= 0 ? a.s_rec[static_cast<int64_t>(r) * a.n + gs] : 0.f;
  __shared__ int s_lo[kT / 64];
  int lo = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t g = g0 + k * kT + threadIdx.x;
    if (g < G && a.s_rec[static_cast<int64_t>(r) * a.n + g] == maxr) lo = min(lo, static_cast<int>(g));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) lo = min(lo, __shfl_xor(lo, o, 64));
  if (lane_id() == 0) s_lo[threadIdx.x >> 6] = lo;
  __syncthreads();
  if (threadIdx.x == 0) {
    int m = 0x7fffffff;
    for (int w = 0; w < kT / 64; ++w) m = min(m, s_lo[w]);
    if (m != 0x7fffffff) atomicMin(&a.glo[r], m);
  }
}

template <typename K>
__global__ void rafp_finalize_kernel(AucScanArgs a) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.rows) return;
  const int gs = a.gstar[r];
  const int64_t row = static_cast<int64_t>(r) * a.n;
  const float maxr = gs >= 0 ? a.s_rec[row + gs] : 0.f;
  const int lo = a.glo[r];
  K best = K(-1);  // no group reaches the maximum: only the appended point (threshold -1) does
  if (lo != 0x7fffffff) {
    best = static_cast<const K*>(a.s_thr)[row + lo];  // the run's highest threshold
    if (maxr == 0.f && best < K(-1)) best = K(-1);   // the appended point competes (NaN stays)
  }
  a.out_max_recall[r] = maxr;
  static_cast<K*>(a.out_best_thr)[r] = static_cast<K>(fabs(static_cast<double>(best)));
}

struct CurveWs {
  char* ab;
  char* tsum;
  char* tstart;
  char* totals;
  char* tcnt;
  char* cstart;
  char* gstar;
  char* glo;
  char* s_rec;
  char* s_thr;
  int64_t bytes;
};

inline int64_t up16(int64_t x) { return (x + 15) & ~int64_t(15); }

CurveWs carve(char* base, int64_t rows, int64_t n, bool rafp, bool direct) {
  const int64_t ntiles = (n + kTile - 1) / kTile;
  CurveWs w{};
  int64_t off = 0;
  auto take = [&](int64_t nb) {
    char* p = base ? base + off : nullptr;
    off += up16(nb);
    return p;
  };
  w.ab = take(direct ? 0 : rows * n * 8);
  w.tsum = take(rows * ntiles * 16);
  w.tstart = take(rows * ntiles * 16);
  w.totals = take(rows * 16);
  w.tcnt = take(rows * ntiles * 4);
  w.cstart = take(rows * ntiles * 4);
  w.gstar = take(rows * 4);
  w.glo = take(rows * 4);
  w.s_rec = take(rafp ? rows * n * 4 : 0);
  w.s_thr = take(rafp ? rows * n * 8 : 0);
  w.bytes = off + 256;
  return w;
}

void bind(AucScanArgs& a, const CurveWs& w, bool rafp) {
  a.ab = w.ab;
  a.tsum = w.tsum;
  a.tstart = w.tstart;
  a.totals = w.totals;
  a.tcnt = reinterpret_cast<int32_t*>(w.tcnt);
  a.cstart = reinterpret_cast<int32_t*>(w.cstart);
  if (rafp) {
    a.gstar = reinterpret_cast<int32_t*>(w.gstar);
    a.glo = reinterpret_cast<int32_t*>(w.glo);
    a.s_rec = reinterpret_cast<float*>(w.s_rec);
    a.s_thr = w.s_thr;
  }
}

}  // namespace

int64_t curve_workspace_bytes(int64_t rows, int64_t n, bool rafp) {
  return carve(nullptr, rows, n, rafp, false).bytes;
}

int launch_curve_count(AucScanArgs& a, void* workspace, bool rafp, hipStream_t stream) {
  if (a.n <= 0 || a.rows <= 0) return 0;
  const int ntiles = static_cast<int>((a.n + kTile - 1) / kTile);
  const bool direct = a.payload_kind != 0;
  bind(a, carve(static_cast<char*>(workspace), a.rows, a.n, rafp, direct), rafp);
  const dim3 grid(ntiles, static_cast<unsigned>(a.rows));
  const bool f64 = a.key_dt == DType::f64;
#define TEA_CNT(K, D) hipLaunchKernelGGL((curve_count_kernel<K, D>), grid, dim3(kT), 0, stream, a)
  if (f64) { if (direct) TEA_CNT(double, true); else TEA_CNT(double, false); }
  else { if (direct) TEA_CNT(float, true); else TEA_CNT(float, false); }
#undef TEA_CNT
  hipLaunchKernelGGL(curve_scan_kernel, dim3(a.rows), dim3(kT), 0, stream, a, ntiles);
  return static_cast<int>(hipGetLastError());
}

int launch_curve_emit(AucScanArgs a, void* workspace, bool rafp, hipStream_t stream) {
  if (a.n <= 0 || a.rows <= 0) return 0;
  const int ntiles = static_cast<int>((a.n + kTile - 1) / kTile);
  const bool direct = a.payload_kind != 0;
  bind(a, carve(static_cast<char*>(workspace), a.rows, a.n, rafp, direct), rafp);
  const dim3 grid(ntiles, static_cast<unsigned>(a.rows));
  const bool f64 = a.key_dt == DType::f64;
#define TEA_EMIT(K, D, R) hipLaunchKernelGGL((curve_emit_kernel<K, D, R>), grid, dim3(kT), 0, stream, a)
  if (rafp) {
    if (f64) { if (direct) TEA_EMIT(double, true, true); else TEA_EMIT(double, false, true); }
    else { if (direct) TEA_EMIT(float, true, true); else TEA_EMIT(float, false, true); }
  } else {
    if (f64) { if (direct) TEA_EMIT(double, true, false); else TEA_EMIT(double, false, false); }
    else { if (direct) TEA_EMIT(float, true, false); else TEA_EMIT(float, false, false); }
  }
#undef TEA_EMIT
  return static_cast<int>(hipGetLastError());
}

int launch_rafp(AucScanArgs a, void* workspace, hipStream_t stream) {
  if (a.n <= 0 || a.rows <= 0) return 0;
  int err = launch_curve_count(a, workspace, true, stream);
  if (err) return err;
  err = launch_curve_emit(a, workspace, true, stream);
  if (err) return err;
  const int ntiles = static_cast<int>((a.n + kTile - 1) / kTile);
  hipLaunchKernelGGL(rafp_find_kernel, dim3(ntiles, static_cast<unsigned>(a.rows)), dim3(kT), 0, stream, a);
  const int fb = static_cast<int>((a.rows + 255) / 256);
  if (a.key_dt == DType::f64) hipLaunchKernelGGL(rafp_finalize_kernel<double>, dim3(fb), dim3(256), 0, stream, a);
  else hipLaunchKernelGGL(rafp_finalize_kernel<float>, dim3(fb), dim3(256), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
