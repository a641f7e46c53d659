// K2: multilabel accuracy counts.
//
// Replaces accuracy.py:388-445: ``torch.where(input < thr, 0, 1)`` (or ``zeros.scatter_(topk)``
// for the top-k variant) materialising an [N, L] label matrix, followed by one or two
// comparisons, an ``all``/``max`` reduction and a ``sum`` per criteria - 4-7 full passes.
// Here one wave64 owns a row: it streams the row's scores and targets once (16-B loads when
// aligned), derives the predicted labels in registers, evaluates every criteria flag with
// wave ballots, and the per-block row count goes through the sharded fold (tea_fold.h) into
// the float32 ``num_correct`` state; block 0 also adds the update's total.  Top-k keeps the
// row in registers (R values per lane, C <= 64 R) and selects k maxima with packed
// (order-preserving key, ~index) u64 wave reductions - ties resolve to the lowest index and
// NaN ranks highest, as in torch.topk.
#include "tea_common.h"
#include "tea_fold.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kB = 256;
constexpr int kWpb = kB / kWave;

enum Criteria { kExact = 0, kHamming = 1, kOverlap = 2, kContain = 3, kBelong = 4 };

struct RowFlags {
  uint32_t eq = 0;  // elements with pred == target
  bool all_eq = true, any_both1 = false, all_both0 = true, all_ge = true, all_le = true;
  __device__ __forceinline__ void add(float p, float t) {
    const bool e = p == t;
    eq += e;
    all_eq &= e;
    any_both1 |= (p == 1.f) & (t == 1.f);
    all_both0 &= (p == 0.f) & (t == 0.f);
    all_ge &= (p - t) >= 0.f;
    all_le &= (p - t) <= 0.f;
  }
};

__device__ __forceinline__ bool wave_all(bool v) { return __ballot(!v) == 0ull; }
__device__ __forceinline__ bool wave_any(bool v) { return __ballot(v) != 0ull; }

// per-row result (valid in every lane)
__device__ __forceinline__ uint32_t row_correct(const RowFlags& f, int criteria) {
  switch (criteria) {
    case kHamming: return static_cast<uint32_t>(wave_sum(static_cast<int>(f.eq)));
    case kExact: return wave_all(f.all_eq) ? 1u : 0u;
    case kOverlap: return (wave_any(f.any_both1) ? 1u : 0u) + (wave_all(f.all_both0) ? 1u : 0u);
    case kContain: return wave_all(f.all_ge) ? 1u : 0u;
    default: return wave_all(f.all_le) ? 1u : 0u;
  }
}

template <int KIND>
__device__ __forceinline__ float ld_x(const void* p, int64_t i) {
  if constexpr (KIND == 0) return static_cast<const float*>(p)[i];
  const uint16_t b = static_cast<const uint16_t*>(p)[i];
  return KIND == 1 ? bf16_to_f32(b) : f16_to_f32(b);
}

template <int KIND>
__device__ __forceinline__ void ld_x4(const void* p, int64_t i, float (&v)[4]) {
  if constexpr (KIND == 0) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else {
    const uint2 q = *reinterpret_cast<const uint2*>(static_cast<const uint16_t*>(p) + i);
    const uint16_t h[4] = {static_cast<uint16_t>(q.x), static_cast<uint16_t>(q.x >> 16),
                           static_cast<uint16_t>(q.y), static_cast<uint16_t>(q.y >> 16)};
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = KIND == 1 ? bf16_to_f32(h[e]) : f16_to_f32(h[e]);
  }
}

// target kinds: 0 f32, 1 i64, 2 i32, 3 u8/bool
template <int TK>
__device__ __forceinline__ float ld_t(const void* p, int64_t i) {
  if constexpr (TK == 0) return static_cast<const float*>(p)[i];
  if constexpr (TK == 1) return static_cast<float>(static_cast<const int64_t*>(p)[i]);
  if constexpr (TK == 2) return static_cast<float>(static_cast<const int32_t*>(p)[i]);
  return static_cast<float>(static_cast<const uint8_t*>(p)[i]);
}

template <int TK>
__device__ __forceinline__ void ld_t4(const void* p, int64_t i, float (&v)[4]) {
  if constexpr (TK == 0) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + i);
    v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
  } else if constexpr (TK == 1) {
    const longlong2* q = reinterpret_cast<const longlong2*>(static_cast<const int64_t*>(p) + i);
    const longlong2 a = q[0], b = q[1];
    v[0] = static_cast<float>(a.x); v[1] = static_cast<float>(a.y);
    v[2] = static_cast<float>(b.x); v[3] = static_cast<float>(b.y);
  } else if constexpr (TK == 2) {
    const int4 q = *reinterpret_cast<const int4*>(static_cast<const int32_t*>(p) + i);
    v[0] = static_cast<float>(q.x); v[1] = static_cast<float>(q.y);
    v[2] = static_cast<float>(q.z); v[3] = static_cast<float>(q.w);
  } else {
    const uint32_t q = *reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(p) + i);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = static_cast<float>((q >> (8 * e)) & 0xffu);
  }
}

__device__ __forceinline__ void block_fold(const MultilabelArgs& a, uint32_t mine) {
  __shared__ uint32_t lds[kWpb];
  if (lane_id() == 0) lds[threadIdx.x >> 6] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < kWpb; ++k) s += lds[k];
    if (a.fold_ws) fold_count(a.fold_ws, s, a.num_correct);
    else if (s) atomicAdd(a.num_correct, static_cast<float>(s));
    if (blockIdx.x == 0 && a.num_total) atomicAdd(a.num_total, static_cast<float>(a.total));
  }
}

// ---- threshold mode: stream the row once
template <int KIND, int TK, bool VEC>
__global__ __launch_bounds__(kB) void ml_threshold_kernel(MultilabelArgs a) {
  const int lane = lane_id();
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kWpb;
  uint32_t mine = 0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWpb + wave_id(); row < a.n; row += nw) {
    const int64_t xo = row * a.x_row_stride, to = row * a.t_row_stride;
    RowFlags f;
    if constexpr (VEC) {
      for (int64_t c = static_cast<int64_t>(lane) * 4; c < a.c; c += kWave * 4) {
        float xv[4], tv[4];
        ld_x4<KIND>(a.x, xo + c, xv);
        ld_t4<TK>(a.t, to + c, tv);
#pragma unroll
        for (int e = 0; e < 4; ++e) f.add(xv[e] < a.threshold ? 0.f : 1.f, tv[e]);
      }
    } else {
      for (int64_t c = lane; c < a.c; c += kWave)
        f.add(ld_x<KIND>(a.x, xo + c) < a.threshold ? 0.f : 1.f, ld_t<TK>(a.t, to + c));
    }
    const uint32_t r = row_correct(f, a.criteria);
    if (lane == 0) mine += r;
  }
  block_fold(a, mine);
}

__device__ __forceinline__ uint32_t order_key(float v) {
  uint32_t u = __float_as_uint(v);
  if (v != v) u = 0x7fc00000u;  // canonical NaN: above +inf after the flip
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long wave_max_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long w = __shfl_xor(v, o, kWave);
    v = w > v ? w : v;
  }
  return v;
}

// ---- top-k mode: row resident in registers, k packed-key wave maxima
template <int KIND, int TK, int R>
__global__ __launch_bounds__(kB) void ml_topk_kernel(MultilabelArgs a) {
  const int lane = lane_id();
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kWpb;
  uint32_t mine = 0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWpb + wave_id(); row < a.n; row += nw) {
    const int64_t xo = row * a.x_row_stride, to = row * a.t_row_stride;
    // scores AND targets are loaded up front, so the target loads overlap the score loads and
    // the top-k selection (v1 loaded targets after the selection: their latency was exposed)
    uint32_t key[R];
    float tv[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t j = lane + static_cast<int64_t>(kWave) * r;
      key[r] = j < a.c ? order_key(ld_x<KIND>(a.x, xo + j)) : 0u;
      tv[r] = j < a.c ? ld_t<TK>(a.t, to + j) : 0.f;
    }
    uint32_t sel = 0;
    for (int it = 0; it < a.k; ++it) {
      unsigned long long best = 0ull;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint32_t j = static_cast<uint32_t>(lane + kWave * r);
        if (!((sel >> r) & 1u) && j < a.c) {
          const unsigned long long cand = (static_cast<unsigned long long>(key[r]) << 32) | (~j);
          best = cand > best ? cand : best;
        }
      }
      best = wave_max_u64(best);
      const uint32_t win = ~static_cast<uint32_t>(best & 0xffffffffull);
      if (static_cast<int>(win % kWave) == lane) sel |= 1u << (win / kWave);
    }
    RowFlags f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int64_t j = lane + static_cast<int64_t>(kWave) * r;
      if (j < a.c) f.add(((sel >> r) & 1u) ? 1.f : 0.f, tv[r]);
    }
    const uint32_t res = row_correct(f, a.criteria);
    if (lane == 0) mine += res;
  }
  block_fold(a, mine);
}

// vectorised top-k: a lane owns 4 consecutive columns per 256-column round (16-B score
// loads, 2 x 16-B int64 target loads): 4x fewer memory instructions than the scalar layout,
// which ran at 33 us for 8192 x 1000 against 17 us for the (vectorised) threshold mode
template <int KIND, int TK, int RV>
__global__ __launch_bounds__(kB) void ml_topk_vec_kernel(MultilabelArgs a) {
  const int lane = lane_id();
  const int64_t nw = static_cast<int64_t>(gridDim.x) * kWpb;
  uint32_t mine = 0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWpb + wave_id(); row < a.n; row += nw) {
    const int64_t xo = row * a.x_row_stride, to = row * a.t_row_stride;
    uint32_t key[RV][4];
    float tv[RV][4];
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      const int64_t j = static_cast<int64_t>(r) * kWave * 4 + lane * 4;
      if (j < a.c) {
        float xv[4];
        ld_x4<KIND>(a.x, xo + j, xv);
        ld_t4<TK>(a.t, to + j, tv[r]);
#pragma unroll
        for (int e = 0; e < 4; ++e) key[r][e] = order_key(xv[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          key[r][e] = 0u;
          tv[r][e] = 0.f;
        }
      }
    }
    uint32_t sel = 0;
    for (int it = 0; it < a.k; ++it) {
      unsigned long long best = 0ull;
#pragma unroll
      for (int r = 0; r < RV; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t j = static_cast<uint32_t>(r * kWave * 4 + lane * 4 + e);
          if (!((sel >> (r * 4 + e)) & 1u) && j < a.c) {
            const unsigned long long cand = (static_cast<unsigned long long>(key[r][e]) << 32) | (~j);
            best = cand > best ? cand : best;
          }
        }
      best = wave_max_u64(best);
      const uint32_t win = ~static_cast<uint32_t>(best & 0xffffffffull);
      if (static_cast<int>((win % (kWave * 4)) / 4) == lane) sel |= 1u << ((win / (kWave * 4)) * 4 + win % 4);
    }
    RowFlags f;
#pragma unroll
    for (int r = 0; r < RV; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t j = static_cast<int64_t>(r) * kWave * 4 + lane * 4 + e;
        if (j < a.c) f.add(((sel >> (r * 4 + e)) & 1u) ? 1.f : 0.f, tv[r][e]);
      }
    const uint32_t res = row_correct(f, a.criteria);
    if (lane == 0) mine += res;
  }
  block_fold(a, mine);
}

template <int KIND, int TK>
int launch_kinds(const MultilabelArgs& a, int grid, hipStream_t s) {
  const int xes = KIND == 0 ? 4 : 2;
  const int tes = TK == 0 ? 4 : TK == 1 ? 8 : TK == 2 ? 4 : 1;
  const bool vec = a.c % 4 == 0 && a.x_row_stride % 4 == 0 && a.t_row_stride % 4 == 0 &&
                   reinterpret_cast<uintptr_t>(a.x) % (4 * xes) == 0 &&
                   reinterpret_cast<uintptr_t>(a.t) % (4 * tes < 16 ? 4 * tes : 16) == 0;
  if (a.k > 0 && vec && a.c <= 8 * kWave * 4) {
    const int64_t RV = (a.c + kWave * 4 - 1) / (kWave * 4);
    if (RV <= 1) hipLaunchKernelGGL((ml_topk_vec_kernel<KIND, TK, 1>), dim3(grid), dim3(kB), 0, s, a);
    else if (RV <= 2) hipLaunchKernelGGL((ml_topk_vec_kernel<KIND, TK, 2>), dim3(grid), dim3(kB), 0, s, a);
    else if (RV <= 4) hipLaunchKernelGGL((ml_topk_vec_kernel<KIND, TK, 4>), dim3(grid), dim3(kB), 0, s, a);
    else hipLaunchKernelGGL((ml_topk_vec_kernel<KIND, TK, 8>), dim3(grid), dim3(kB), 0, s, a);
    return 0;
  }
  if (a.k > 0) {
    const int64_t R = (a.c + kWave - 1) / kWave;
    if (R <= 4) hipLaunchKernelGGL((ml_topk_kernel<KIND, TK, 4>), dim3(grid), dim3(kB), 0, s, a);
    else if (R <= 8) hipLaunchKernelGGL((ml_topk_kernel<KIND, TK, 8>), dim3(grid), dim3(kB), 0, s, a);
    else if (R <= 16) hipLaunchKernelGGL((ml_topk_kernel<KIND, TK, 16>), dim3(grid), dim3(kB), 0, s, a);
    else if (R <= 32) hipLaunchKernelGGL((ml_topk_kernel<KIND, TK, 32>), dim3(grid), dim3(kB), 0, s, a);
    else return -2;
    return 0;
  }
  if (vec) hipLaunchKernelGGL((ml_threshold_kernel<KIND, TK, true>), dim3(grid), dim3(kB), 0, s, a);
  else hipLaunchKernelGGL((ml_threshold_kernel<KIND, TK, false>), dim3(grid), dim3(kB), 0, s, a);
  return 0;
}

template <int KIND>
int launch_tk(const MultilabelArgs& a, int grid, hipStream_t s) {
  switch (a.t_dt) {
    case DType::f32: return launch_kinds<KIND, 0>(a, grid, s);
    case DType::i64: return launch_kinds<KIND, 1>(a, grid, s);
    case DType::i32: return launch_kinds<KIND, 2>(a, grid, s);
    case DType::u8:
    case DType::b8: return launch_kinds<KIND, 3>(a, grid, s);
    default: return -1;
  }
}

}  // namespace

int multilabel_max_topk_cols() { return 32 * kWave; }

int launch_multilabel(const MultilabelArgs& a, hipStream_t stream) {
  if (a.n <= 0) return 0;
  const int grid = stream_grid(a.n, kWpb, 2048);
  int rc;
  switch (a.x_dt) {
    case DType::f32: rc = launch_tk<0>(a, grid, stream); break;
    case DType::bf16: rc = launch_tk<1>(a, grid, stream); break;
    case DType::f16: rc = launch_tk<2>(a, grid, stream); break;
    default: return -1;
  }
  if (rc != 0) return rc;
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
