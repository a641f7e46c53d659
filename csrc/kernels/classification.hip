// K1: fused classification counts.
//
// Replaces the reference's eager op chains
//   accuracy.py:260-278   argmax -> eq -> long -> sum / scatter_(add) x2
//   precision.py:115-139  argmax -> 3 x scatter_(add)
//   recall.py:156-181, f1_score.py:166-193, confusion_matrix.py:219-234 (vstack + sparse_coo
//   + to_dense)
// with ONE streaming pass over the [N, C] score matrix that writes straight into the metric
// state tensors (no temporaries, no host syncs).
//
// Layout / mapping (gfx950):
//  * one wave64 per row, grid-stride over rows; a row is read with 16-B loads per lane
//    (float4 for f32, 8 x 16-bit for bf16/f16), four loads in flight per lane before the
//    compare chain, so a 256-thread block keeps 16 KB of HBM reads outstanding.
//  * argmax reduces (value, index) across the wave with xor-shuffles, torch.argmax tie/NaN
//    semantics (first index, NaN is max).  top-k (k > 1) uses rank-of-target = #(x > x_t).
//  * micro counts: per-block LDS reduction -> ONE float atomic per block.  Per-class
//    histograms / confusion matrix: one lane per row issues the scatter atomics (targets are
//    spread over C addresses, so contention is low).
//  * invalid targets / predictions never fault: they are skipped and flagged in ``err``
//    (bit 0: target out of range, bit 1: predicted label out of range); the Python layer
//    checks the flag where the reference would have raised.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kUnroll = 4;

template <int KIND, int VEC>
struct RowLoader;

// f32
template <>
struct RowLoader<0, 4> {
  static __device__ __forceinline__ void load(const void* row, int col, float (&v)[4]) {
    const float4 x = *reinterpret_cast<const float4*>(static_cast<const float*>(row) + col);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
  }
  static __device__ __forceinline__ float one(const void* row, int64_t col) {
    return static_cast<const float*>(row)[col];
  }
};
template <>
struct RowLoader<0, 1> {
  static __device__ __forceinline__ void load(const void* row, int col, float (&v)[1]) {
    v[0] = static_cast<const float*>(row)[col];
  }
  static __device__ __forceinline__ float one(const void* row, int64_t col) {
    return static_cast<const float*>(row)[col];
  }
};
// bf16 (KIND 1) / f16 (KIND 2)
template <int KIND>
__device__ __forceinline__ float h16(uint16_t b) {
  return KIND == 1 ? bf16_to_f32(b) : f16_to_f32(b);
}
template <int KIND>
struct RowLoader16x8 {
  static __device__ __forceinline__ void load(const void* row, int col, float (&v)[8]) {
    const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(row) + col);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = h16<KIND>(static_cast<uint16_t>(w[e] & 0xffffu));
      v[2 * e + 1] = h16<KIND>(static_cast<uint16_t>(w[e] >> 16));
    }
  }
  static __device__ __forceinline__ float one(const void* row, int64_t col) {
    return h16<KIND>(static_cast<const uint16_t*>(row)[col]);
  }
};
template <>
struct RowLoader<1, 8> : RowLoader16x8<1> {};
template <>
struct RowLoader<2, 8> : RowLoader16x8<2> {};
template <int KIND>
struct RowLoader16x1 {
  static __device__ __forceinline__ void load(const void* row, int col, float (&v)[1]) {
    v[0] = h16<KIND>(static_cast<const uint16_t*>(row)[col]);
  }
  static __device__ __forceinline__ float one(const void* row, int64_t col) {
    return h16<KIND>(static_cast<const uint16_t*>(row)[col]);
  }
};
template <>
struct RowLoader<1, 1> : RowLoader16x1<1> {};
template <>
struct RowLoader<2, 1> : RowLoader16x1<2> {};

__device__ __forceinline__ int64_t load_target(const void* tgt, DType dt, int64_t i) {
  return dt == DType::i64 ? static_cast<const int64_t*>(tgt)[i] : load_as_i64(tgt, dt, i);
}

// Per-row bookkeeping shared by the score and label kernels (executed by one lane).
__device__ __forceinline__ void row_epilogue(const ClsCountsArgs& a, int64_t t, int64_t pred,
                                             bool correct) {
  const int64_t C = a.num_classes;
  const bool t_ok = t >= 0 && t < C;
  const bool p_ok = pred >= 0 && pred < C;
  if (a.err) {
    if (!t_ok && (a.cls_label || a.cls_correct || a.confusion || a.check_target)) atomicOr(a.err, 1);
    if (!p_ok && (a.cls_pred || a.confusion)) atomicOr(a.err, 2);
  }
  if (t_ok) {
    if (a.cls_correct && correct) atomicAdd(a.cls_correct + t, 1.f);
    if (a.cls_label) atomicAdd(a.cls_label + t, 1.f);
  }
  if (p_ok && a.cls_pred) atomicAdd(a.cls_pred + pred, 1.f);
  if (t_ok && p_ok && a.confusion) atomicAdd(a.confusion + t * C + pred, 1.f);
}

__device__ __forceinline__ void block_flush_micro(const ClsCountsArgs& a, int correct_lane0) {
  __shared__ int lds[kWavesPerBlock];
  if (lane_id() == 0) lds[threadIdx.x >> 6] = correct_lane0;
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) s += lds[w];
    if (a.micro_correct && s) atomicAdd(a.micro_correct, static_cast<float>(s));
    if (a.micro_total && blockIdx.x == 0) atomicAdd(a.micro_total, static_cast<float>(a.n));
  }
}

template <int KIND, int VEC, bool TOPK>
__global__ __launch_bounds__(kBlock) void cls_scores_kernel(ClsCountsArgs a) {
  using L = RowLoader<KIND, VEC>;
  const int lane = lane_id();
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  const int elsize = KIND == 0 ? 4 : 2;
  const int C = static_cast<int>(a.c);
  int correct_acc = 0;

  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wave_id(); row < a.n;
       row += nwaves) {
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * elsize;
    const int64_t t = load_target(a.target, a.tg_dt, row);
    bool correct;
    int64_t pred = -1;
    if constexpr (!TOPK) {
      float bv = -__builtin_huge_valf();
      int bi = 0x7fffffff;
      constexpr int STEP = kWave * VEC;
      for (int base = 0; base < C; base += STEP * kUnroll) {
        float v[kUnroll][VEC];
        bool ok[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const int col = base + u * STEP + lane * VEC;
          ok[u] = col < C;
          if (ok[u]) L::load(rp, col, v[u]);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          if (ok[u]) {
            const int col = base + u * STEP + lane * VEC;
#pragma unroll
            for (int e = 0; e < VEC; ++e)
              if (argmax_better(v[u][e], col + e, bv, bi)) {
                bv = v[u][e];
                bi = col + e;
              }
          }
        }
      }
      wave_argmax(bv, bi);
      pred = bi;
      correct = pred == t;
    } else {
      const bool t_ok = t >= 0 && t < C;
      const float xt = t_ok ? L::one(rp, t) : __builtin_nanf("");
      int cnt = 0;
      constexpr int STEP = kWave * VEC;
      for (int base = 0; base < C; base += STEP * kUnroll) {
        float v[kUnroll][VEC];
        bool ok[kUnroll];
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
          const int col = base + u * STEP + lane * VEC;
          ok[u] = col < C;
          if (ok[u]) L::load(rp, col, v[u]);
        }
#pragma unroll
        for (int u = 0; u < kUnroll; ++u)
          if (ok[u]) {
#pragma unroll
            for (int e = 0; e < VEC; ++e) cnt += v[u][e] > xt;
          }
      }
      cnt = wave_sum(cnt);
      correct = t_ok && cnt < a.k;
    }
    if (lane == 0) {
      correct_acc += correct;
      row_epilogue(a, t, pred, correct);
    }
  }
  block_flush_micro(a, correct_acc);
}

// 1-D integer label predictions: elementwise compare + histograms.
__global__ __launch_bounds__(kBlock) void cls_labels_kernel(ClsCountsArgs a) {
  int correct_acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride) {
    const int64_t p = load_as_i64(a.input, a.in_dt, i);
    const int64_t t = load_target(a.target, a.tg_dt, i);
    const bool correct = p == t;
    correct_acc += correct;
    row_epilogue(a, t, p, correct);
  }
  correct_acc = wave_sum(correct_acc);
  block_flush_micro(a, correct_acc);
}

// Binary: thresholded scores vs targets -> [tp, fp, tn, fn] (+ optional weights).
__global__ __launch_bounds__(kBlock) void binary_counts_kernel(BinaryCountsArgs a) {
  float tp = 0.f, fp = 0.f, tn = 0.f, fn = 0.f;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride) {
    const float x = load_as_f32(a.input, a.in_dt, i);
    const double t = load_as_f64(a.target, a.tg_dt, i);
    const int pred = (x < a.threshold) ? 0 : 1;
    const float w = a.weight ? load_as_f32(a.weight, a.w_dt, i) : 1.f;
    if (pred == 1) {
      if (t == 1.0) tp += w;
      else if (t == 0.0) fp += w;
      else fp += a.strict_binary ? 0.f : w;
    } else {
      if (t == 0.0) tn += w;
      else if (t == 1.0) fn += w;
      else fn += a.strict_binary ? 0.f : w;
    }
  }
  tp = wave_sum(tp);
  fp = wave_sum(fp);
  tn = wave_sum(tn);
  fn = wave_sum(fn);
  __shared__ float lds[4][kWavesPerBlock];
  if (lane_id() == 0) {
    const int w = threadIdx.x >> 6;
    lds[0][w] = tp;
    lds[1][w] = fp;
    lds[2][w] = tn;
    lds[3][w] = fn;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) s += lds[threadIdx.x][w];
    float* dst = a.out[threadIdx.x];
    if (dst && s != 0.f) atomicAdd(dst, s);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.total) atomicAdd(a.total, static_cast<float>(a.n));
}

template <int KIND, int VEC>
void launch_scores(const ClsCountsArgs& a, int grid, hipStream_t s) {
  if (a.k > 1)
    hipLaunchKernelGGL((cls_scores_kernel<KIND, VEC, true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((cls_scores_kernel<KIND, VEC, false>), dim3(grid), dim3(kBlock), 0, s, a);
}

}  // namespace

int launch_cls_counts(const ClsCountsArgs& a, hipStream_t stream) {
  if (a.n <= 0) {
    return 0;
  }
  const int cap = a.max_blocks > 0 ? a.max_blocks : 1024;
  if (a.c > 0) {
    const int grid = stream_grid(a.n, kWavesPerBlock, cap);
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.input);
    switch (a.in_dt) {
      case DType::f32: {
        const bool vec = (a.c % 4 == 0) && (a.row_stride % 4 == 0) && (base % 16 == 0);
        vec ? launch_scores<0, 4>(a, grid, stream) : launch_scores<0, 1>(a, grid, stream);
        break;
      }
      case DType::bf16: {
        const bool vec = (a.c % 8 == 0) && (a.row_stride % 8 == 0) && (base % 16 == 0);
        vec ? launch_scores<1, 8>(a, grid, stream) : launch_scores<1, 1>(a, grid, stream);
        break;
      }
      case DType::f16: {
        const bool vec = (a.c % 8 == 0) && (a.row_stride % 8 == 0) && (base % 16 == 0);
        vec ? launch_scores<2, 8>(a, grid, stream) : launch_scores<2, 1>(a, grid, stream);
        break;
      }
      default:
        return -1;  // caller falls back / converts
    }
  } else {
    const int grid = stream_grid(a.n, kBlock, cap);
    hipLaunchKernelGGL(cls_labels_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  }
  return static_cast<int>(hipGetLastError());
}

int launch_binary_counts(const BinaryCountsArgs& a, hipStream_t stream) {
  if (a.n <= 0) return 0;
  const int cap = a.max_blocks > 0 ? a.max_blocks : 1024;
  const int grid = stream_grid(a.n, kBlock * 4, cap);
  hipLaunchKernelGGL(binary_counts_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
