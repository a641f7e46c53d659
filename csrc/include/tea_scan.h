// Shared device helpers of the K3 family (sortscan.hip: AUROC / AUPRC scan; curves.hip: PR
// curve emission and recall at fixed precision): tile geometry, FP64 pair scans over 64-wide
// waves, and the per-sample (a, b) = (w t, w (1 - t)) loads through the sort's payload.
#pragma once

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {
namespace k3 {

constexpr int kT = 256;              // threads per block
constexpr int kPer = 4;              // samples per thread (1024-sample tiles: ~1000 blocks at 1M;
                                     // measured: 512- and 2048-sample tiles are 5-6% slower end to end)
constexpr int kTile = kT * kPer;     // samples per tile

struct alignas(16) D2 {
  double x, y;
};

__device__ __forceinline__ D2 d2add(D2 a, D2 b) { return {a.x + b.x, a.y + b.y}; }

__device__ __forceinline__ D2 wave_incl_scan(D2 v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double x = __shfl_up(v.x, o, 64);
    const double y = __shfl_up(v.y, o, 64);
    if (lane >= o) {
      v.x += x;
      v.y += y;
    }
  }
  return v;
}

// exclusive block scan of one D2 per thread (blockDim = kT)
__device__ __forceinline__ D2 block_excl_scan(D2 v, D2* lds /* >= 4 */, D2& total) {
  const D2 inc = wave_incl_scan(v);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 63) lds[w] = inc;
  __syncthreads();
  D2 off{0.0, 0.0};
  total = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < kT / 64; ++k) {
    if (k < w) off = d2add(off, lds[k]);
    total = d2add(total, lds[k]);
  }
  __syncthreads();
  return {off.x + inc.x - v.x, off.y + inc.y - v.y};
}

__device__ __forceinline__ int wave_incl_max(int v) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(v, o, 64);
    if (lane >= o) v = max(v, u);
  }
  return v;
}
__device__ __forceinline__ int wave_incl_min_rev(int v) {  // suffix min across lanes
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_down(v, o, 64);
    if (lane + o < 64) v = min(v, u);
  }
  return v;
}

template <typename K>
__device__ __forceinline__ K key_at(const AucScanArgs& a, int r, int64_t i) {
  return static_cast<const K*>(a.sorted)[r * a.key_stride + i];
}

__device__ __forceinline__ float2 sample_ab(const AucScanArgs& a, int r, int64_t i) {
  if (a.payload_kind == 1) {  // unweighted binary: the sort carried the target itself
    const float t = __uint_as_float(static_cast<uint32_t>(a.order32[r * a.order_stride + i]));
    return make_float2(t, 1.f - t);
  }
  if (a.payload_kind == 2) {  // one-vs-rest: the sort carried the class label
    const float t = a.order32[r * a.order_stride + i] == r ? 1.f : 0.f;
    return make_float2(t, 1.f - t);
  }
  const int64_t src = a.order32 ? static_cast<int64_t>(a.order32[r * a.order_stride + i])
                                : a.order[r * a.order_stride + i];
  float t;
  if (a.class_mode) {
    t = load_as_i64(a.target, a.tg_dt, src) == r ? 1.f : 0.f;
  } else {
    t = load_as_f32(a.target, a.tg_dt, r * a.target_stride + src);
  }
  const float w = a.weight ? load_as_f32(a.weight, a.w_dt, r * a.weight_stride + src) : 1.f;
  return make_float2(w * t, w * (1.f - t));
}

// (a, b) of sorted sample i: in place for payload kinds 1 / 2, else the gathered ab copy
template <bool DIRECT>
__device__ __forceinline__ float2 load_ab(const AucScanArgs& a, const float2* ab, int r, int64_t i) {
  if constexpr (DIRECT) return sample_ab(a, r, i);
  return ab[i];
}

}  // namespace k3
}  // namespace tea
