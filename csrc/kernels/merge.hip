// K3m: merge-path merge of two descending-sorted (score, payload) runs.
//
// SURVEY.md §5.7 "sorted-run gather + merge": after a distributed sync every rank holds the
// ranks' samples as R runs that each rank already sorted (BinaryAUROC / BinaryAUPRC sort
// their local samples in _prepare_for_merge_state).  Merging R sorted runs costs log2(R)
// streaming passes instead of a full radix sort of the union (4 passes of histogram +
// scatter) - and the merged order is exactly what K3's scan consumes.
//
// One launch per run pair: each 256-thread block owns kPerBlock = 2048 consecutive output
// positions.  Thread 0 finds the block's merge-path split (a, b) with a + b = start by a
// binary search on the cross diagonal (O(log n) global probes), the block stages
// A[a, a + 2048) and B[b, b + 2048) in LDS, every thread finds its own 8-element diagonal
// split inside LDS and merges 8 outputs sequentially.  Order: descending, NaN first (as
// torch.sort / K3a), ties keep A before B (stable), so each run's internal order survives.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kMT = 256;
constexpr int kPerThread = 8;
constexpr int kPerBlock = kMT * kPerThread;

// x goes before y in descending order with NaN first
__device__ __forceinline__ bool before(float x, float y) {
  const bool xn = x != x, yn = y != y;
  if (xn || yn) return xn && !yn;
  return x > y;
}

// merge-path split for output diagonal d of A[0, na) and B[0, nb): the number of A elements
// among the first d outputs (ties: A first)
template <typename LoadA, typename LoadB>
__device__ __forceinline__ int64_t path_split(int64_t d, int64_t na, int64_t nb, LoadA la, LoadB lb) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) / 2;  // mid A elements taken, d - mid - 1 is the B index probed
    // take A[mid] iff it is not after B[d - mid - 1]: A[mid] >= B[d-mid-1] in merge order
    if (!before(lb(d - mid - 1), la(mid))) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kMT) void merge_path_kernel(const float* __restrict__ ka, const uint32_t* __restrict__ va,
                                                         int64_t na, const float* __restrict__ kb,
                                                         const uint32_t* __restrict__ vb, int64_t nb,
                                                         float* __restrict__ ko, uint32_t* __restrict__ vo) {
  __shared__ float sk[2 * kPerBlock];
  __shared__ uint32_t sv[2 * kPerBlock];
  __shared__ int64_t s_split[2];
  const int64_t n = na + nb;
  const int64_t d0 = static_cast<int64_t>(blockIdx.x) * kPerBlock;
  const int64_t d1 = min(n, d0 + kPerBlock);
  if (threadIdx.x < 2) {
    const int64_t d = threadIdx.x == 0 ? d0 : d1;
    s_split[threadIdx.x] = path_split(d, na, nb, [&](int64_t i) { return ka[i]; }, [&](int64_t i) { return kb[i]; });
  }
  __syncthreads();
  const int64_t a0 = s_split[0], a1 = s_split[1];
  const int64_t b0 = d0 - a0, b1 = d1 - a1;
  const int la = static_cast<int>(a1 - a0), lb = static_cast<int>(b1 - b0);
  for (int i = threadIdx.x; i < la; i += kMT) {
    sk[i] = ka[a0 + i];
    sv[i] = va[a0 + i];
  }
  for (int i = threadIdx.x; i < lb; i += kMT) {
    sk[kPerBlock + i] = kb[b0 + i];
    sv[kPerBlock + i] = vb[b0 + i];
  }
  __syncthreads();
  const float* A = sk;
  const float* B = sk + kPerBlock;
  const int64_t t0 = static_cast<int64_t>(threadIdx.x) * kPerThread;
  if (t0 >= la + lb) return;
  int i = static_cast<int>(path_split(t0, la, lb, [&](int64_t k) { return A[k]; }, [&](int64_t k) { return B[k]; }));
  int j = static_cast<int>(t0) - i;
  const int64_t tout = min(static_cast<int64_t>(kPerThread), static_cast<int64_t>(la + lb) - t0);
  for (int k = 0; k < tout; ++k) {
    const bool take_a = j >= lb || (i < la && !before(B[j], A[i]));
    const int src = take_a ? i : kPerBlock + j;
    ko[d0 + t0 + k] = sk[src];
    vo[d0 + t0 + k] = sv[src];
    if (take_a) ++i;
    else ++j;
  }
}

}  // namespace

int launch_merge_desc(const float* ka, const uint32_t* va, int64_t na, const float* kb, const uint32_t* vb, int64_t nb,
                      float* ko, uint32_t* vo, hipStream_t stream) {
  const int64_t n = na + nb;
  if (n <= 0) return 0;
  const unsigned blocks = static_cast<unsigned>((n + kPerBlock - 1) / kPerBlock);
  hipLaunchKernelGGL(merge_path_kernel, dim3(blocks), dim3(kMT), 0, stream, ka, va, na, kb, vb, nb, ko, vo);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
