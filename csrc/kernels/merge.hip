// K3m: merge-path merge of two descending-sorted (score, payload) runs.
//
// SURVEY.md §5.7 "sorted-run gather + merge": after a distributed sync every rank holds the
// ranks' samples as R runs that each rank already sorted (BinaryAUROC / BinaryAUPRC sort
// their local samples in _prepare_for_merge_state).  Merging R sorted runs costs log2(R)
// streaming passes instead of a full radix sort of the union (4 passes of histogram +
// scatter) - and the merged order is exactly what K3's scan consumes.
//
// Two launches per run pair; each 256-thread merge block owns kTile = 2048 consecutive outputs:
//  1. merge_splits_kernel: the merge-path split of every tile boundary (output diagonal
//     q * kTile), one wave per diagonal, by a 64-ary search: every round the wave probes 64
//     evenly spaced candidates in global memory at once and a ballot popcount narrows the
//     range 64x - ~4 rounds of one load, no barriers, all diagonals of the pass in flight
//     together.  (v1: a 23-load dependent binary search by one thread of each merge block,
//     ~120 us per 8M pass; v2: a 128-ary block search inside the merge block, ~79 us - the
//     search latency sat on every merge block's critical path.)
//  2. A[a0, a1) and B[b0, b1) staged in LDS with coalesced loads (la + lb = 2048);
//  3. every thread finds its own 8-output diagonal split inside LDS and merges 8 outputs
//     into an LDS output tile;
//  4. coalesced write-out of the 2048 keys and payloads.
// Order: descending, NaN first (as torch.sort / K3a), ties keep A before B (stable), so each
// run's internal order survives.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kMT = 256;
constexpr int kPerThread = 8;
constexpr int kTile = kMT * kPerThread;

// x goes before y in descending order with NaN first
__device__ __forceinline__ bool before(float x, float y) {
  const bool xn = x != x, yn = y != y;
  if (xn || yn) return xn && !yn;
  return x > y;
}

// merge-path split for output diagonal d of A[0, na) and B[0, nb): the number of A elements
// among the first d outputs (ties: A first) = the smallest m in [lo, hi) with
// before(B[d - m - 1], A[m]), or hi.  Sequential binary search (LDS operands).
template <typename LoadA, typename LoadB>
__device__ __forceinline__ int64_t path_split(int64_t d, int64_t na, int64_t nb, LoadA la, LoadB lb) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;
    if (!before(lb(d - mid - 1), la(mid))) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// one wave per diagonal q: splits[q] = number of A elements among the first min(q kTile, n)
// outputs.  P(m) = A[m] goes before-or-ties B[d - m - 1] is true for a prefix of [lo, hi); the
// answer is the first m where it is false (or hi).
__global__ __launch_bounds__(kMT) void merge_splits_kernel(const float* __restrict__ ka, int64_t na,
                                                           const float* __restrict__ kb, int64_t nb,
                                                           int64_t* __restrict__ splits, int64_t ndiag) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * (kMT / kWave) + (threadIdx.x >> 6);
  if (q >= ndiag) return;  // whole wave
  const int lane = threadIdx.x & 63;
  const int64_t d = min(na + nb, q * kTile);
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {  // wave-uniform
    const int64_t step = (hi - lo + kWave - 1) / kWave;
    const int64_t p = lo + static_cast<int64_t>(lane) * step;
    const bool pred = p < hi && !before(kb[d - p - 1], ka[p]);
    const int t = __popcll(__ballot(pred));  // monotone: the first t probes are true
    const int64_t nlo = t == 0 ? lo : lo + static_cast<int64_t>(t - 1) * step + 1;
    const int64_t nhi = min(hi, lo + static_cast<int64_t>(t) * step);
    lo = nlo;
    hi = max(nlo, nhi);
  }
  if (lane == 0) splits[q] = lo;
}

__global__ __launch_bounds__(kMT) void merge_path_kernel(const float* __restrict__ ka, const uint32_t* __restrict__ va,
                                                         int64_t na, uint32_t base_a, const float* __restrict__ kb,
                                                         const uint32_t* __restrict__ vb, int64_t nb, uint32_t base_b,
                                                         const int64_t* __restrict__ splits, float* __restrict__ ko,
                                                         uint32_t* __restrict__ vo) {
  __shared__ float sk[kTile];      // A window then B window
  __shared__ uint32_t sv[kTile];
  __shared__ float ok_[kTile];     // merged output tile
  __shared__ uint32_t ov[kTile];
  const int64_t n = na + nb;
  const int64_t d0 = static_cast<int64_t>(blockIdx.x) * kTile;
  const int64_t d1 = min(n, d0 + kTile);
  const int64_t a0 = splits[blockIdx.x], a1 = splits[blockIdx.x + 1];
  const int64_t b0 = d0 - a0, b1 = d1 - a1;
  const int la = static_cast<int>(a1 - a0), lb = static_cast<int>(b1 - b0);

  // 2. stage the windows (A at [0, la), B at [la, la + lb))
  for (int i = threadIdx.x; i < la; i += kMT) {
    sk[i] = ka[a0 + i];
    sv[i] = va ? va[a0 + i] : base_a + static_cast<uint32_t>(a0 + i);
  }
  for (int i = threadIdx.x; i < lb; i += kMT) {
    sk[la + i] = kb[b0 + i];
    sv[la + i] = vb ? vb[b0 + i] : base_b + static_cast<uint32_t>(b0 + i);
  }
  __syncthreads();

  // 3. per-thread split and 8-way sequential merge into the LDS output tile
  const float* A = sk;
  const float* B = sk + la;
  const int t0 = threadIdx.x * kPerThread;
  const int tot = la + lb;
  if (t0 < tot) {
    int i = static_cast<int>(path_split(t0, la, lb, [&](int64_t k) { return A[k]; }, [&](int64_t k) { return B[k]; }));
    int j = t0 - i;
    const int tout = min(kPerThread, tot - t0);
    for (int k = 0; k < tout; ++k) {
      const bool take_a = j >= lb || (i < la && !before(B[j], A[i]));
      const int src = take_a ? i : la + j;
      ok_[t0 + k] = sk[src];
      ov[t0 + k] = sv[src];
      if (take_a) ++i;
      else ++j;
    }
  }
  __syncthreads();

  // 4. coalesced write-out
  for (int i = threadIdx.x; i < tot; i += kMT) {
    ko[d0 + i] = ok_[i];
    vo[d0 + i] = ov[i];
  }
}

}  // namespace

int64_t merge_splits_count(int64_t n) { return (n + kTile - 1) / kTile + 1; }

int launch_merge_desc(const float* ka, const uint32_t* va, int64_t na, uint32_t base_a, const float* kb,
                      const uint32_t* vb, int64_t nb, uint32_t base_b, float* ko, uint32_t* vo, int64_t* splits,
                      hipStream_t stream) {
  static_assert(kTile == kMergeTile, "header tile size");
  const int64_t n = na + nb;
  if (n <= 0) return 0;
  const int64_t blocks = (n + kTile - 1) / kTile;
  const int64_t ndiag = blocks + 1;
  const int64_t sblocks = (ndiag + kMT / kWave - 1) / (kMT / kWave);
  hipLaunchKernelGGL(merge_splits_kernel, dim3(static_cast<unsigned>(sblocks)), dim3(kMT), 0, stream, ka, na, kb, nb,
                     splits, ndiag);
  hipLaunchKernelGGL(merge_path_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kMT), 0, stream, ka, va, na, base_a,
                     kb, vb, nb, base_b, splits, ko, vo);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
