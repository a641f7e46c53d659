// K10b: segmented streaming top-k for RetrievalPrecision (SURVEY.md §5.7 "streaming top-k";
// reference torcheval/metrics/ranking/retrieval_precision.py:136-166 loops over queries on
// the host: `i in indexes`, cat + topk + gather per query).
//
// One update merges a batch (scores x, targets t, query ids q) into per-query state rows
// topk[Q, k] / target[Q, k] / count[Q] (best first, padded with -inf / 0):
//  1. retrieval_hist_kernel: per-query batch counts (LDS-privatised histogram, one global
//     atomic per non-zero bin per block);
//  2. retrieval_scan_kernel: exclusive scan of the counts -> segment starts (one block);
//  3. retrieval_scatter_kernel: every valid sample is ranked among its block's samples of the
//     same query (LDS atomics), each (block, query) reserves its range with ONE global atomic,
//     and the sample's (order key, batch index) lands in its query's segment;
//  4. retrieval_select_kernel: one wave per query selects the top-k of old row + segment by
//     k rounds of a wave-wide max over packed keys (order key << 32 | ~position) strictly
//     below the previous pick - no marking, no sort.  Ties keep the reference's cat order:
//     old entries first, then batch order (position = slot for old entries, k + batch index
//     for new ones).  NaN ranks highest and -0 ties +0, as torch.topk.
// Samples whose query id is outside [0, Q) are ignored.  k <= 64 (one pick per lane).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kRB = 256;       // hist / scatter block
constexpr int kRPer = 16;      // samples per thread in hist / scatter
constexpr int kRTile = kRB * kRPer;

__device__ __forceinline__ uint32_t order_key(float v) {
  uint32_t b = __float_as_uint(v);
  if (v != v) b = 0x7fc00000u;  // canonical +NaN: above +inf
  if (b == 0x80000000u) b = 0u;  // -0 ties +0
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

__device__ __forceinline__ int64_t query_of(const RetrievalArgs& a, int64_t i) {
  return a.q ? a.q[i] : 0;
}

__global__ __launch_bounds__(kRB) void retrieval_hist_kernel(RetrievalArgs a) {
  extern __shared__ int hist[];  // [Q]
  for (int j = threadIdx.x; j < a.Q; j += kRB) hist[j] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRTile;
#pragma unroll 4
  for (int r = 0; r < kRPer; ++r) {
    const int64_t i = base + static_cast<int64_t>(r) * kRB + threadIdx.x;
    if (i < a.n) {
      const int64_t q = query_of(a, i);
      if (q >= 0 && q < a.Q) atomicAdd(&hist[q], 1);
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.Q; j += kRB)
    if (hist[j]) atomicAdd(&a.counts[j], hist[j]);
}

// one block: offsets[j] = sum_{i<j} counts[i]; cursor = offsets; counts re-zeroed (the
// workspace stays zeroed between calls)
__global__ __launch_bounds__(1024) void retrieval_scan_kernel(RetrievalArgs a) {
  __shared__ int wsum[1024 / kWave];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 <= a.Q; c0 += 1024) {
    const int64_t j = c0 + threadIdx.x;
    const int v = j < a.Q ? a.counts[j] : 0;
    // block exclusive scan of v
    int x = v;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(x, o, kWave);
      if (lane >= o) x += y;
    }
    if (lane == kWave - 1) wsum[w] = x;
    __syncthreads();
    if (w == 0) {
      int s = lane < 1024 / kWave ? wsum[lane] : 0;
#pragma unroll
      for (int o = 1; o < 1024 / kWave; o <<= 1) {
        const int y = __shfl_up(s, o, kWave);
        if (lane >= o) s += y;
      }
      if (lane < 1024 / kWave) wsum[lane] = s;
    }
    __syncthreads();
    const int incl = x + (w ? wsum[w - 1] : 0);
    const int excl = carry + incl - v;
    if (j <= a.Q) {
      a.offsets[j] = excl;
      if (j < a.Q) {
        a.cursor[j] = excl;
        a.counts[j] = 0;
      }
    }
    __syncthreads();
    if (threadIdx.x == 1023) carry += incl;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kRB) void retrieval_scatter_kernel(RetrievalArgs a) {
  extern __shared__ int lds[];  // [Q] local counts, then [Q] reserved bases
  int* cnt = lds;
  int* basep = lds + a.Q;
  for (int j = threadIdx.x; j < a.Q; j += kRB) cnt[j] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRTile;
  int rank[kRPer];
  int qq[kRPer];
#pragma unroll
  for (int r = 0; r < kRPer; ++r) {
    const int64_t i = base + static_cast<int64_t>(r) * kRB + threadIdx.x;
    qq[r] = -1;
    rank[r] = 0;
    if (i < a.n) {
      const int64_t q = query_of(a, i);
      if (q >= 0 && q < a.Q) {
        qq[r] = static_cast<int>(q);
        rank[r] = atomicAdd(&cnt[q], 1);
      }
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < a.Q; j += kRB)
    basep[j] = cnt[j] ? atomicAdd(&a.cursor[j], cnt[j]) : 0;
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRPer; ++r) {
    if (qq[r] < 0) continue;
    const int64_t i = base + static_cast<int64_t>(r) * kRB + threadIdx.x;
    const int pos = basep[qq[r]] + rank[r];
    a.rec_key[pos] = order_key(a.x[i]);
    a.rec_idx[pos] = static_cast<uint32_t>(i);
  }
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t y = __shfl_xor(v, o, kWave);
    v = y > v ? y : v;
  }
  return v;
}

__global__ __launch_bounds__(kRB) void retrieval_select_kernel(RetrievalArgs a) {
  const int64_t q = static_cast<int64_t>(blockIdx.x) * (kRB / kWave) + (threadIdx.x >> 6);
  if (q >= a.Q) return;  // whole wave
  const int lane = threadIdx.x & 63;
  const int k = a.k;
  float* trow = a.topk + q * k;
  float* grow = a.target_state + q * k;
  const int64_t old = a.count[q] < k ? a.count[q] : k;
  const int s0 = a.offsets[q], s1 = a.offsets[q + 1];
  const int c = s1 - s0;
  // candidate packed keys: old slot j -> (key(topk[j]) << 32) | ~j ; batch -> ~(k + idx)
  uint64_t prev = ~0ull;
  float my_val = -__builtin_inff(), my_tgt = 0.f;
  const int64_t total = old + c;
  const int picks = total < k ? static_cast<int>(total) : k;
  for (int r = 0; r < picks; ++r) {
    uint64_t best = 0;
    for (int64_t j = lane; j < old; j += kWave) {
      const uint64_t pk = (static_cast<uint64_t>(order_key(trow[j])) << 32) | static_cast<uint32_t>(~static_cast<uint32_t>(j));
      if (pk < prev && pk > best) best = pk;
    }
    for (int j = lane; j < c; j += kWave) {
      const uint32_t pos = static_cast<uint32_t>(k) + a.rec_idx[s0 + j];
      const uint64_t pk = (static_cast<uint64_t>(a.rec_key[s0 + j]) << 32) | static_cast<uint32_t>(~pos);
      if (pk < prev && pk > best) best = pk;
    }
    best = wave_max_u64(best);
    prev = best;
    if (lane == r) {
      const uint32_t pos = ~static_cast<uint32_t>(best & 0xffffffffu);
      if (pos < static_cast<uint32_t>(k)) {
        my_val = trow[pos];
        my_tgt = grow[pos];
      } else {
        const int64_t i = pos - static_cast<uint32_t>(k);
        my_val = a.x[i];
        my_tgt = a.t[i];
      }
    }
  }
  // every read of the old row is done (the wave's shuffles ordered them): write the new row
  if (lane < k) {
    trow[lane] = lane < picks ? my_val : -__builtin_inff();
    grow[lane] = lane < picks ? my_tgt : 0.f;
  }
  if (lane == 0) {
    const int64_t nc = a.count[q] + c;
    a.count[q] = nc < k ? nc : k;
  }
}

}  // namespace

int retrieval_lds_bytes(int64_t Q) { return static_cast<int>(2 * Q * 4); }

int launch_retrieval_topk(const RetrievalArgs& a, hipStream_t stream) {
  if (a.Q <= 0) return 0;
  if (a.k < 1 || a.k > kWave || 2 * a.Q * 4 > kRetrievalMaxLds) return -1;
  const unsigned blocks = static_cast<unsigned>((a.n + kRTile - 1) / kRTile);
  if (a.n > 0) {
    hipLaunchKernelGGL(retrieval_hist_kernel, dim3(blocks), dim3(kRB), static_cast<size_t>(a.Q * 4), stream, a);
  }
  hipLaunchKernelGGL(retrieval_scan_kernel, dim3(1), dim3(1024), 0, stream, a);
  if (a.n > 0) {
    hipLaunchKernelGGL(retrieval_scatter_kernel, dim3(blocks), dim3(kRB), static_cast<size_t>(2 * a.Q * 4), stream, a);
  }
  const unsigned sel = static_cast<unsigned>((a.Q + kRB / kWave - 1) / (kRB / kWave));
  hipLaunchKernelGGL(retrieval_select_kernel, dim3(sel), dim3(kRB), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
