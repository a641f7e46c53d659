// K3: tie-aware scan + integrals over score-sorted samples (AUROC / AUPRC).
//
// Replaces the reference's post-sort op chains
//   auroc.py:115-152, 206-235   diff != 0 -> pad -> gather x2 -> cumsum x2 -> masked_scatter x2
//                               (host-synchronising) -> trapz -> where
//   auprc.py / precision_recall_curve.py:156-231   same prefix + per-class Python loops
// with three launches (rows of <= kFuseTiles tiles) or four that never leave the device (one
// fewer when the onesweep sort folded the tile totals, AucScanArgs::tsum_ext - opt-in, measured
// slower: profiles/k3_fold_r5.json):
//   1 tile_sums : per 1024-sample tile, the tile totals (double) of a = w*t, b = w*(1-t); when the
//                 sort carried the targets / labels (payload kinds 1, 2) they are read in place,
//                 otherwise (target, weight) are gathered through the permutation into float2 ab.
//   2 tile_scan : (long rows only) one block per row: exclusive scan of the tile totals.  Short
//                 rows fold it into tile_area: each block sums the totals of the tiles before it
//                 (<= kFuseTiles L2-resident loads), one launch and ~8 us less at 1M samples.
//   3 tile_area : per tile, LDS block scans give TP/FP at every element; prefix-max / suffix-min
//                 scans locate each sample's tie group (head / tail) inside the tile; groups that
//                 straddle a tile edge are resolved once per block by a binary search on the
//                 sorted scores plus a partial-tile reduction.  Per sample:
//                   roc += b_i * (TP(head-) + TP(tail)) / 2      (Mann-Whitney with ties)
//                   pr  += a_i * TP(tail) / (TP(tail) + FP(tail)) (average precision)
//   4 finalize  : per row: AUROC = roc / (P * N) (0.5 if degenerate), AUPRC = pr / P (0 if P = 0).
// Accumulation is in FP64 (the reference accumulates in FP32), so results are at least as
// accurate as the reference's.
#include "tea_common.h"
#include "tea_kernels.h"
#include "tea_scan.h"

namespace tea {

namespace {

using namespace k3;
constexpr int kFuseTiles = 1536;     // (<= 4) rows up to this many tiles skip the tile_scan launch
constexpr int kFusePer = kFuseTiles / kT;  // preceding-tile totals per thread in the fused prefix

template <bool DIRECT>
__global__ __launch_bounds__(kT) void tile_sums_kernel(AucScanArgs a) {
  const int r = blockIdx.y;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  double sa = 0.0, sb = 0.0;
  float2* ab = reinterpret_cast<float2*>(a.ab) + static_cast<int64_t>(r) * a.n;
  // clamped unconditional loads, the tail masked after (a per-lane `if (i < n)` around the
  // loads compiled to a branch + vmcnt(0) per element)
  float2 vv[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = base + k * kT + threadIdx.x;  // coalesced gather order
    vv[k] = sample_ab(a, r, i < a.n ? i : a.n - 1);
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = base + k * kT + threadIdx.x;
    const bool ok = i < a.n;
    if constexpr (!DIRECT) {
      if (ok) ab[i] = vv[k];
    }
    sa += ok ? vv[k].x : 0.f;
    sb += ok ? vv[k].y : 0.f;
  }
  __shared__ double lds[2][kT / 64];
  sa = wave_sum(sa);
  sb = wave_sum(sb);
  if (lane_id() == 0) {
    lds[0][threadIdx.x >> 6] = sa;
    lds[1][threadIdx.x >> 6] = sb;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    D2 s{0.0, 0.0};
    for (int w = 0; w < kT / 64; ++w) s = {s.x + lds[0][w], s.y + lds[1][w]};
    reinterpret_cast<D2*>(a.tsum)[static_cast<int64_t>(r) * gridDim.x + blockIdx.x] = s;
  }
}

// one block per row: exclusive scan of the tile totals, row totals
__global__ __launch_bounds__(kT) void tile_scan_kernel(AucScanArgs a, int ntiles) {
  const int r = blockIdx.x;
  D2* ts = reinterpret_cast<D2*>(a.tsum) + static_cast<int64_t>(r) * ntiles;
  D2* st = reinterpret_cast<D2*>(a.tstart) + static_cast<int64_t>(r) * ntiles;
  __shared__ D2 lds[kT / 64];
  const D2 init = a.init ? D2{a.init[2 * r], a.init[2 * r + 1]} : D2{0.0, 0.0};
  D2 carry = init;
  for (int b = 0; b < ntiles; b += kT) {
    const int t = b + threadIdx.x;
    const D2 v = t < ntiles ? ts[t] : D2{0.0, 0.0};
    D2 tot;
    const D2 ex = block_excl_scan(v, lds, tot);
    if (t < ntiles) st[t] = d2add(carry, ex);
    carry = d2add(carry, tot);
  }
  // totals are this shard's own P, N (the init offsets are excluded)
  if (threadIdx.x == 0) reinterpret_cast<D2*>(a.totals)[r] = D2{carry.x - init.x, carry.y - init.y};
}

// init + the totals of tiles [0, upto) of row r (block-cooperative; fused tile_scan)
__device__ D2 tiles_prefix(const AucScanArgs& a, const D2* ts, int upto, int r, D2* lds) {
  double sa = 0.0, sb = 0.0;
  for (int t = threadIdx.x; t < upto; t += kT) {
    const D2 v = ts[t];
    sa += v.x;
    sb += v.y;
  }
  D2 tot;
  block_excl_scan(D2{sa, sb}, lds, tot);
  if (a.init) tot = d2add(tot, D2{a.init[2 * r], a.init[2 * r + 1]});
  return tot;
}

// sum of a/b over [lo, hi] (inclusive, hi may be < lo -> empty) of row r, block-cooperative
template <bool DIRECT>
__device__ D2 block_range_sum(const AucScanArgs& a, const float2* ab, int r, int64_t lo, int64_t hi, D2* lds) {
  double sa = 0.0, sb = 0.0;
  for (int64_t i = lo + threadIdx.x; i <= hi; i += kT) {
    const float2 v = load_ab<DIRECT>(a, ab, r, i);
    sa += v.x;
    sb += v.y;
  }
  D2 tot;
  block_excl_scan(D2{sa, sb}, lds, tot);
  return tot;
}

template <typename K>
__device__ int64_t first_equal(const AucScanArgs& a, int r, int64_t lo, int64_t hi, K v) {
  // descending keys; first index in [lo, hi) with key == v, given key[hi] == v
  while (lo < hi) {
    const int64_t mid = lo + (hi - lo) / 2;
    if (key_at<K>(a, r, mid) > v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
template <typename K>
__device__ int64_t last_equal(const AucScanArgs& a, int r, int64_t lo, int64_t hi, K v) {
  // descending keys; last index in [lo, hi) with key == v, given key[lo] == v
  int64_t l = lo, h = hi;  // find first index with key < v in [lo, hi)
  while (l < h) {
    const int64_t mid = l + (h - l) / 2;
    if (key_at<K>(a, r, mid) < v) h = mid;
    else l = mid + 1;
  }
  return l - 1;
}

// tile start (TP, FP): from tile_scan's table, or (FUSED) summed here from the tile totals
template <bool FUSED>
__device__ __forceinline__ D2 tile_start(const AucScanArgs& a, int r, int tile, int ntiles, D2* lds) {
  if constexpr (FUSED)
    return tiles_prefix(a, reinterpret_cast<const D2*>(a.tsum) + static_cast<int64_t>(r) * ntiles, tile, r, lds);
  return reinterpret_cast<const D2*>(a.tstart)[static_cast<int64_t>(r) * ntiles + tile];
}

// row r: AUROC = roc / (P * N) (0.5 if degenerate), AUPRC = pr / P (0 if P = 0)
__device__ void finalize_row(const AucScanArgs& a, int r, int ntiles, bool fused, D2* lds) {
  const D2* ta = reinterpret_cast<const D2*>(a.tarea) + static_cast<int64_t>(r) * ntiles;
  const D2* ts = reinterpret_cast<const D2*>(a.tsum) + static_cast<int64_t>(r) * ntiles;
  double roc = 0.0, pr = 0.0, p = 0.0, q = 0.0;
  if (ntiles <= kFuseTiles) {  // every load in flight together
    D2 v[kFusePer], w[kFusePer];
#pragma unroll
    for (int u = 0; u < kFusePer; ++u) {
      const int t = u * kT + static_cast<int>(threadIdx.x);
      const int tc = t < ntiles ? t : 0;
      v[u] = ta[tc];
      w[u] = fused ? ts[tc] : D2{0.0, 0.0};
    }
#pragma unroll
    for (int u = 0; u < kFusePer; ++u) {
      const bool ok = u * kT + static_cast<int>(threadIdx.x) < ntiles;
      roc += ok ? v[u].x : 0.0;
      pr += ok ? v[u].y : 0.0;
      p += ok ? w[u].x : 0.0;
      q += ok ? w[u].y : 0.0;
    }
  } else {
    for (int t = threadIdx.x; t < ntiles; t += kT) {
      const D2 v = ta[t];
      roc += v.x;
      pr += v.y;
      if (fused) {
        const D2 u = ts[t];
        p += u.x;
        q += u.y;
      }
    }
  }
  D2 tot, pn;
  block_excl_scan(D2{roc, pr}, lds, tot);
  block_excl_scan(D2{p, q}, lds, pn);
  if (threadIdx.x == 0) {
    if (!fused) pn = reinterpret_cast<const D2*>(a.totals)[r];  // this shard's own P, N
    if (a.out_raw) {
      a.out_raw[4 * r] = tot.x;
      a.out_raw[4 * r + 1] = tot.y;
      a.out_raw[4 * r + 2] = pn.x;
      a.out_raw[4 * r + 3] = pn.y;
    }
    if (a.sort_fault != nullptr && *a.sort_fault != 0u) {  // the sort timed out: no wrong numbers
      const double nan = __builtin_nan("");
      tot = D2{nan, nan};
      pn = D2{nan, nan};
      if (a.out_raw) {
#pragma unroll
        for (int k = 0; k < 4; ++k) a.out_raw[4 * r + k] = nan;
      }
    }
    const double factor = pn.x * pn.y;
    if (a.out_auroc) a.out_auroc[r] = factor == 0.0 ? 0.5 : tot.x / factor;
    if (a.out_auprc) a.out_auprc[r] = pn.x == 0.0 ? 0.0 : tot.y / pn.x;
  }
}

template <typename K, bool DIRECT, bool FUSED>
__global__ __launch_bounds__(kT) void tile_area_kernel(AucScanArgs a) {
  const int r = blockIdx.y;
  const int ntiles = gridDim.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kTile;
  const int tile_n = static_cast<int>(min(static_cast<int64_t>(kTile), a.n - base));
  const float2* ab = reinterpret_cast<const float2*>(a.ab) + static_cast<int64_t>(r) * a.n;

  __shared__ double s_tpx[kTile];  // TP before each element (exclusive)
  __shared__ double s_fpi[kTile];  // FP up to each element (inclusive)
  __shared__ D2 lds[kT / 64];
  __shared__ double s_bound[3];    // TP before the entering group; TP, FP at the leaving group's tail
  __shared__ int s_flags[2];
  __shared__ int s_fb[2];          // a straddling group longer than the window: binary search
  __shared__ int s_hmax[kT / 64], s_tmin[kT / 64];
  __shared__ int64_t s_pos;

  // every global load of the tile is issued up front (one round trip): the thread's keys and
  // (a, b), its outer neighbour keys, and (fused) its share of the preceding tile totals
  const int j0 = threadIdx.x * kPer;
  const int64_t i0 = base + j0;
  K key[kPer];
  float2 v[kPer];
  // clamped unconditional loads (the tile has >= 1 sample, so base + tile_n - 1 is valid),
  // masked after: one round trip instead of one per element
  const int64_t ilast = base + tile_n - 1;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int64_t i = i0 + k < ilast ? i0 + k : ilast;
    key[k] = key_at<K>(a, r, i);
    v[k] = load_ab<DIRECT>(a, ab, r, i);
  }
  const bool live = j0 < tile_n;
  K pk0 = key_at<K>(a, r, i0 > 0 ? (i0 - 1 < ilast ? i0 - 1 : ilast) : 0);
  K nk_last = key_at<K>(a, r, i0 + kPer < a.n ? i0 + kPer : a.n - 1);
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const bool ok = j0 + k < tile_n;
    key[k] = ok ? key[k] : K(0);
    v[k] = ok ? v[k] : make_float2(0.f, 0.f);
  }
  pk0 = (live && i0 > 0) ? pk0 : K(0);
  nk_last = (live && i0 + kPer < a.n) ? nk_last : K(0);
  double pa = 0.0, pb = 0.0;
  if constexpr (FUSED) {
    // the preceding tiles' totals: every load in flight together (clamped index, masked after),
    // where a strided loop paid one round trip per 256 tiles
    const D2* ts = reinterpret_cast<const D2*>(a.tsum) + static_cast<int64_t>(r) * ntiles;
    const int upto = static_cast<int>(blockIdx.x);
    D2 q[kFusePer];
#pragma unroll
    for (int u = 0; u < kFusePer; ++u) {
      const int t = u * kT + static_cast<int>(threadIdx.x);
      q[u] = ts[t < upto ? t : 0];
    }
#pragma unroll
    for (int u = 0; u < kFusePer; ++u) {
      const bool ok = u * kT + static_cast<int>(threadIdx.x) < upto;
      pa += ok ? q[u].x : 0.0;
      pb += ok ? q[u].y : 0.0;
    }
  } else {  // tile_scan's table (one broadcast load; a block scan here cost 53 -> 62 us at 100 x 100k)
    const D2 q = reinterpret_cast<const D2*>(a.tstart)[static_cast<int64_t>(r) * ntiles + blockIdx.x];
    pa = q.x;
    pb = q.y;
  }
  double la = 0.0, lb = 0.0;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    la += v[k].x;
    lb += v[k].y;
  }
  // tie groups straddling the tile edges: thread 0 holds key(base) and key(base - 1), the
  // thread owning the tile's last sample holds it and the key after the tile
  if (threadIdx.x == 0) {
    s_flags[0] = (base > 0 && key[0] == pk0) ? 1 : 0;
    s_bound[0] = s_bound[1] = s_bound[2] = 0.0;
  }
  if (j0 + kPer == tile_n) s_flags[1] = (base + tile_n < a.n && key[kPer - 1] == nk_last) ? 1 : 0;
  if (j0 < tile_n && tile_n < j0 + kPer) s_flags[1] = 0;  // ragged last tile: nothing follows
  D2 tot;
  const D2 ex = block_excl_scan(D2{la, lb}, lds, tot);
  D2 t0{pa, pb};
  if constexpr (FUSED) {
    block_excl_scan(D2{pa, pb}, lds, t0);  // block total = the tiles before this one
    if (a.init) t0 = d2add(t0, D2{a.init[2 * r], a.init[2 * r + 1]});
  }

  bool headf[kPer], tailf[kPer];
  int my_head = -1, my_tail = kTile;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int j = j0 + k;
    const int64_t i = base + j;
    bool h = false, tl = false;
    if (j < tile_n) {
      const K pk = (k > 0) ? key[k - 1] : pk0;
      const K nk = (k + 1 < kPer) ? key[k + 1] : nk_last;
      h = (i == 0) || !(pk == key[k]);
      tl = (i == a.n - 1) || !(nk == key[k]);
    }
    headf[k] = h;
    tailf[k] = tl;
    if (h) my_head = j;
  }
#pragma unroll
  for (int k = kPer - 1; k >= 0; --k)
    if (tailf[k]) my_tail = j0 + k;
  {
    double ca = t0.x + ex.x, cb = t0.y + ex.y;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = j0 + k;
      s_tpx[j] = ca;
      ca += v[k].x;
      cb += v[k].y;
      s_fpi[j] = cb;
    }
  }
  const int w = threadIdx.x >> 6;
  const int hin = wave_incl_max(my_head);
  const int tin = wave_incl_min_rev(my_tail);
  if (lane_id() == 63) s_hmax[w] = hin;
  if (lane_id() == 0) s_tmin[w] = tin;
  __syncthreads();
  int hmax_before = -1, tmin_after = kTile;
  for (int k = 0; k < w; ++k) hmax_before = max(hmax_before, s_hmax[k]);
  for (int k = w + 1; k < kT / 64; ++k) tmin_after = min(tmin_after, s_tmin[k]);
  int h_excl = __shfl_up(hin, 1, 64);
  if (lane_id() == 0) h_excl = -1;
  h_excl = max(h_excl, hmax_before);
  int t_excl = __shfl_down(tin, 1, 64);
  if (lane_id() == 63) t_excl = kTile;
  t_excl = min(t_excl, tmin_after);

  // tie groups straddling the tile edges (block-uniform branches).  Not rare: 1M uniform f32
  // scores give ~3 % equal neighbours, so ~60 of ~1000 tiles have a straddling group, and the
  // kernel lasts as long as its slowest block.  A group that ends (starts) within kWin samples
  // beyond the edge is resolved from ONE window load: wave 0 (head side) / wave 1 (tail side)
  // load the kWin keys and (a, b) past the edge, the equal ones are the group's part there, and
  // their sums correct the tile's own prefix (TP before the group = TP before the tile - their
  // a; TP / FP at the group's tail = TP / FP at the tile's end + their a / b).  Only a group
  // covering the whole window falls back to the binary search + partial-tile reduction (~20
  // dependent global round trips: it made the kernel 19 us at 1M samples).
  constexpr int kWin = 64;
  if (threadIdx.x == 0) s_fb[0] = s_fb[1] = 0;
  __syncthreads();
  if (s_flags[0] && w == 0) {
    const K v0 = __shfl(key[0], 0, 64);  // key(base): thread 0's first sample
    const int64_t i = base - kWin + lane_id();  // base >= kTile > kWin on this path
    const K kk = key_at<K>(a, r, i);
    const float2 ab_i = load_ab<DIRECT>(a, ab, r, i);
    const bool eq = kk == v0;
    const unsigned long long m = __ballot(eq);
    const double sa = wave_sum(eq ? static_cast<double>(ab_i.x) : 0.0);
    if (lane_id() == 0) {
      if (m & 1ull) s_fb[0] = 1;  // the group may reach further back
      else s_bound[0] = t0.x - sa;
    }
  }
  if (s_flags[1] && w == 1) {
    const K v1 = key_at<K>(a, r, base + tile_n - 1);
    const int64_t i = base + tile_n + lane_id();
    const bool valid = i < a.n;
    const K kk = key_at<K>(a, r, valid ? i : a.n - 1);
    const float2 ab_i = load_ab<DIRECT>(a, ab, r, valid ? i : a.n - 1);
    const bool eq = valid && kk == v1;
    const unsigned long long m = __ballot(eq);
    const double sa = wave_sum(eq ? static_cast<double>(ab_i.x) : 0.0);
    const double sb = wave_sum(eq ? static_cast<double>(ab_i.y) : 0.0);
    if (lane_id() == 0) {
      if (m >> 63) s_fb[1] = 1;  // the group may reach further on
      else {
        s_bound[1] = t0.x + tot.x + sa;
        s_bound[2] = t0.y + tot.y + sb;
      }
    }
  }
  __syncthreads();
  if (s_fb[0]) {
    if (threadIdx.x == 0) s_pos = first_equal<K>(a, r, 0, base, key_at<K>(a, r, base));
    __syncthreads();
    const int64_t hpos = s_pos;
    const int64_t ht = hpos / kTile;
    const D2 part = block_range_sum<DIRECT>(a, ab, r, ht * kTile, hpos - 1, lds);
    const D2 hs = tile_start<FUSED>(a, r, static_cast<int>(ht), ntiles, lds);
    if (threadIdx.x == 0) s_bound[0] = hs.x + part.x;
    __syncthreads();
  }
  if (s_fb[1]) {
    if (threadIdx.x == 0)
      s_pos = last_equal<K>(a, r, base + tile_n, a.n, key_at<K>(a, r, base + tile_n - 1));
    __syncthreads();
    const int64_t epos = s_pos;
    const int64_t et = epos / kTile;
    const D2 part = block_range_sum<DIRECT>(a, ab, r, et * kTile, epos, lds);
    const D2 es = tile_start<FUSED>(a, r, static_cast<int>(et), ntiles, lds);
    if (threadIdx.x == 0) {
      s_bound[1] = es.x + part.x;
      s_bound[2] = es.y + part.y;
    }
    __syncthreads();
  }

  // per-sample credit (group head: last head <= j; group tail: first tail >= j)
  int ntail[kPer];
  {
    int nt = t_excl;
#pragma unroll
    for (int k = kPer - 1; k >= 0; --k) {
      if (tailf[k]) nt = j0 + k;
      ntail[k] = nt;
    }
  }
  const double tile_tp_end = t0.x + tot.x;
  double roc = 0.0, pr = 0.0;
  int cur_head = h_excl;
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int j = j0 + k;
    if (headf[k]) cur_head = j;
    if (j < tile_n) {
      const int tail = ntail[k];
      const double tps = (cur_head >= 0) ? s_tpx[cur_head] : s_bound[0];
      double tpe, fpe;
      if (tail < tile_n) {
        tpe = (tail + 1 < tile_n) ? s_tpx[tail + 1] : tile_tp_end;
        fpe = s_fpi[tail];
      } else {
        tpe = s_bound[1];
        fpe = s_bound[2];
      }
      roc += static_cast<double>(v[k].y) * 0.5 * (tps + tpe);
      const double den = tpe + fpe;
      if (v[k].x != 0.f && den != 0.0) pr += static_cast<double>(v[k].x) * (tpe / den);
    }
  }
  D2 area;
  block_excl_scan(D2{roc, pr}, lds, area);
  if (threadIdx.x == 0)
    reinterpret_cast<D2*>(a.tarea)[static_cast<int64_t>(r) * ntiles + blockIdx.x] = area;
}

// one block per row.  (A "last block finalises" fold inside tile_area was measured: the
// agent-scope release / acquire fences it needs per block - the XCDs' L2s are not coherent -
// doubled tile_area, 16 -> 34 us at 1M samples; a separate launch costs ~4 us.)
__global__ __launch_bounds__(kT) void finalize_kernel(AucScanArgs a, int ntiles, int fused) {
  __shared__ D2 lds[kT / 64];
  finalize_row(a, blockIdx.x, ntiles, fused != 0, lds);
}

}  // namespace

int64_t auc_scan_workspace_bytes(int64_t rows, int64_t n) {
  const int64_t ntiles = (n + kTile - 1) / kTile;
  return rows * n * 8 + rows * ntiles * 16 * 3 + rows * 16 + 256;
}

int launch_auc_scan(AucScanArgs a, void* workspace, hipStream_t stream) {
  if (a.n <= 0 || a.rows <= 0) return 0;
  const int ntiles = static_cast<int>((a.n + kTile - 1) / kTile);
  char* ws = static_cast<char*>(workspace);
  a.ab = ws;
  ws += a.rows * a.n * 8;
  ws = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(ws) + 15) & ~uintptr_t(15));
  a.tsum = ws;
  ws += a.rows * ntiles * 16;
  a.tstart = ws;
  ws += a.rows * ntiles * 16;
  a.tarea = ws;
  ws += a.rows * ntiles * 16;
  a.totals = ws;
  const dim3 grid(ntiles, static_cast<unsigned>(a.rows));
  // fused prefix: single / few rows only - it lengthens every block's dependency chain (an extra
  // block reduction before the scan), which 100 rows x 98 tiles paid for with +12 us per call
  const bool direct = a.payload_kind != 0, fused = ntiles <= kFuseTiles && a.rows <= 4;
  const bool f64 = a.key_dt == DType::f64;
  if (a.tsum_ext != nullptr) {
    // the sort's last pass already added the tile totals (RadixArgs::fold_ab): no tile_sums launch
    if (!direct) return -2;
    a.tsum = const_cast<void*>(a.tsum_ext);
  } else if (direct) {
    hipLaunchKernelGGL(tile_sums_kernel<true>, grid, dim3(kT), 0, stream, a);
  } else {
    hipLaunchKernelGGL(tile_sums_kernel<false>, grid, dim3(kT), 0, stream, a);
  }
  if (!fused) hipLaunchKernelGGL(tile_scan_kernel, dim3(a.rows), dim3(kT), 0, stream, a, ntiles);
#define TEA_AREA(K, D, F) hipLaunchKernelGGL((tile_area_kernel<K, D, F>), grid, dim3(kT), 0, stream, a)
  if (f64) {
    if (direct) { if (fused) TEA_AREA(double, true, true); else TEA_AREA(double, true, false); }
    else { if (fused) TEA_AREA(double, false, true); else TEA_AREA(double, false, false); }
  } else {
    if (direct) { if (fused) TEA_AREA(float, true, true); else TEA_AREA(float, true, false); }
    else { if (fused) TEA_AREA(float, false, true); else TEA_AREA(float, false, false); }
  }
#undef TEA_AREA
  hipLaunchKernelGGL(finalize_kernel, dim3(a.rows), dim3(kT), 0, stream, a, ntiles, fused ? 1 : 0);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
