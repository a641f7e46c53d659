// K10: rank-of-target scores.
//
// Replaces the reference's per-sample ranking chain (ranking/hit_rate.py,
// ranking/reciprocal_rank.py):
//     y = gather(input, -1, target[:, None]);  rank = (input > y).sum(-1)
//     hit = (rank < k).float()    |    rr = 1 / (rank + 1), 0 where rank >= k
// i.e. a gather kernel, a [N, C] bool temporary, a reduction and 2-3 elementwise kernels, with
// ONE pass over the [N, C] scores that writes the float score per row.
//
// Layout (gfx950): the same row-per-wave streaming as K1 - for C >= 64 every lane issues all of
// its 16-B loads of a 64*VEC*4-column chunk before comparing, so a whole row chunk is in flight;
// rows are grid-strided over ~one wave per row.  Rows with C < 64 would leave lanes idle, so they
// take a thread-per-row kernel.  Comparisons are IEEE ``>`` exactly as ATen's (a NaN target score
// ranks 0, NaN candidates never count).  An out-of-range target never faults: its row scores NaN
// and bit 0 of ``err`` is set (surfaced by the metric at compute / under validate).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kChunkLoads = 4;

template <int KIND>
__device__ __forceinline__ float ld1(const void* row, int64_t col) {
  if constexpr (KIND == 0) return static_cast<const float*>(row)[col];
  const uint16_t b = static_cast<const uint16_t*>(row)[col];
  return KIND == 1 ? bf16_to_f32(b) : f16_to_f32(b);
}

// count of v > xt over VEC consecutive columns starting at col (16-B load)
template <int KIND, int VEC>
__device__ __forceinline__ int gt_vec(const void* row, int col, float xt) {
  if constexpr (KIND == 0 && VEC == 4) {
    const float4 x = *reinterpret_cast<const float4*>(static_cast<const float*>(row) + col);
    return (x.x > xt) + (x.y > xt) + (x.z > xt) + (x.w > xt);
  } else if constexpr (VEC == 8) {
    const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(row) + col);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
    int c = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint16_t lo = static_cast<uint16_t>(w[e] & 0xffffu), hi = static_cast<uint16_t>(w[e] >> 16);
      c += ((KIND == 1 ? bf16_to_f32(lo) : f16_to_f32(lo)) > xt);
      c += ((KIND == 1 ? bf16_to_f32(hi) : f16_to_f32(hi)) > xt);
    }
    return c;
  } else {
    return ld1<KIND>(row, col) > xt;
  }
}

__device__ __forceinline__ float score_of(int mode, int64_t rank, int k) {
  if (mode == 0) return rank < k ? 1.f : 0.f;
  return (k > 0 && rank >= k) ? 0.f : 1.f / (static_cast<float>(rank) + 1.f);
}

template <int KIND, int VEC>
__global__ __launch_bounds__(kBlock) void rank_wide_kernel(RankArgs a) {
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  constexpr int STEP = kWave * VEC;
  constexpr int CHUNK = STEP * kChunkLoads;
  const int lane = lane_id();
  const int C = static_cast<int>(a.c);
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wave_id(); row < a.n;
       row += nwaves) {
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELSIZE;
    const int64_t t = load_as_i64(a.target, a.tg_dt, row);
    const bool t_ok = t >= 0 && t < C;
    const float xt = ld1<KIND>(rp, t_ok ? t : 0);
    int cnt = 0;
    for (int base = 0; base < C; base += CHUNK) {
      int part[kChunkLoads];
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u) {
        const int col = base + u * STEP + lane * VEC;
        part[u] = col < C ? gt_vec<KIND, VEC>(rp, col, xt) : 0;
      }
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u) cnt += part[u];
    }
    cnt = wave_sum(cnt);
    if (lane == 0) {
      a.out[row] = t_ok ? score_of(a.mode, cnt, a.k) : __builtin_nanf("");
      if (!t_ok && a.err) atomicOr(a.err, 1);
    }
  }
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void rank_narrow_kernel(RankArgs a) {
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; row < a.n; row += stride) {
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELSIZE;
    const int64_t t = load_as_i64(a.target, a.tg_dt, row);
    const bool t_ok = t >= 0 && t < a.c;
    const float xt = ld1<KIND>(rp, t_ok ? t : 0);
    int cnt = 0;
    for (int col = 0; col < a.c; ++col) cnt += ld1<KIND>(rp, col) > xt;
    a.out[row] = t_ok ? score_of(a.mode, cnt, a.k) : __builtin_nanf("");
    if (!t_ok && a.err) atomicOr(a.err, 1);
  }
}

template <int KIND, int VEC>
int launch_wide(const RankArgs& a, hipStream_t s) {
  int64_t blocks = (a.n + kWavesPerBlock - 1) / kWavesPerBlock;
  blocks = blocks < 1 ? 1 : (blocks > 16384 ? 16384 : blocks);
  hipLaunchKernelGGL((rank_wide_kernel<KIND, VEC>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, s, a);
  return static_cast<int>(hipGetLastError());
}

template <int KIND>
int launch_kind(const RankArgs& a, hipStream_t s) {
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  constexpr int VEC = 16 / ELSIZE;
  if (a.c < kWave) {
    int64_t blocks = (a.n + kBlock - 1) / kBlock;
    blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
    hipLaunchKernelGGL((rank_narrow_kernel<KIND>), dim3(static_cast<unsigned>(blocks)), dim3(kBlock), 0, s, a);
    return static_cast<int>(hipGetLastError());
  }
  const bool aligned = (reinterpret_cast<uintptr_t>(a.input) % 16 == 0) && (a.row_stride % VEC == 0) &&
                       (a.c % VEC == 0);
  return aligned ? launch_wide<KIND, VEC>(a, s) : launch_wide<KIND, 1>(a, s);
}

}  // namespace

int launch_rank_scores(const RankArgs& a, hipStream_t stream) {
  if (a.n == 0) return 0;
  switch (a.in_dt) {
    case DType::f32: return launch_kind<0>(a, stream);
    case DType::bf16: return launch_kind<1>(a, stream);
    case DType::f16: return launch_kind<2>(a, stream);
    default: return -1;
  }
}

}  // namespace tea
