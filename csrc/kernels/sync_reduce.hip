// C3: fused cross-rank reduction of a gathered metric-state buffer.
//
// The small-state sync (torcheval_amd/parallel/state_buffer.py) all-gathers every rank's
// contiguous state buffer in ONE RCCL all_gather_into_tensor: rows [ws][row_bytes].  This
// kernel then reduces every (op, dtype) segment of that row layout across the ws rows in one
// launch (the ATen form is one launch per segment plus a cat), writing the merged buffer the
// synced metric's states are views of.  Ranks are folded in ascending order with the same
// arithmetic on every rank, so all ranks get bit-identical states.
//
// Replaces reference torcheval/metrics/toolkit.py:371-391 (pickled all_gather_object of the
// whole metric followed by merge_state on each rank).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kBlock = 256;

template <typename T>
__device__ __forceinline__ T ld(const uint8_t* p) {
  return *reinterpret_cast<const T*>(p);
}
template <typename T>
__device__ __forceinline__ void st(uint8_t* p, T v) {
  *reinterpret_cast<T*>(p) = v;
}

// NaN-propagating max / min (torch.amax / amin semantics)
template <typename F>
__device__ __forceinline__ F fmax_nan(F a, F b) {
  return (a != a) ? a : (b != b) ? b : (b > a ? b : a);
}
template <typename F>
__device__ __forceinline__ F fmin_nan(F a, F b) {
  return (a != a) ? a : (b != b) ? b : (b < a ? b : a);
}

// Reduce element e of one segment over the ws rows (rank 0 first).
template <typename T, typename Acc>
__device__ __forceinline__ void reduce_elem(const SegReduceArgs& a, int64_t byte, int op) {
  const uint8_t* p = a.rows + byte;
  Acc acc = static_cast<Acc>(ld<T>(p));
  for (int r = 1; r < a.ws; ++r) {
    const Acc v = static_cast<Acc>(ld<T>(p + r * a.row_bytes));
    if (op == 0) acc = acc + v;
    else if (op == 1) acc = fmax_nan(acc, v);
    else acc = fmin_nan(acc, v);
  }
  st<T>(a.out + byte, static_cast<T>(acc));
}

__device__ __forceinline__ void reduce_bytes16(const SegReduceArgs& a, int64_t byte, int dt, int op) {
  // bf16 / f16: accumulate in float, round once (torch's sum(0) on a [ws, n] half tensor)
  const uint8_t* p = a.rows + byte;
  auto cvt = [dt](uint16_t b) { return dt == static_cast<int>(DType::bf16) ? bf16_to_f32(b) : f16_to_f32(b); };
  float acc = cvt(ld<uint16_t>(p));
  for (int r = 1; r < a.ws; ++r) {
    const float v = cvt(ld<uint16_t>(p + r * a.row_bytes));
    if (op == 0) acc += v;
    else if (op == 1) acc = fmax_nan(acc, v);
    else acc = fmin_nan(acc, v);
  }
  uint16_t o;
  if (dt == static_cast<int>(DType::bf16)) {
    const __bf16 h = static_cast<__bf16>(acc);
    __builtin_memcpy(&o, &h, 2);
  } else {
    const _Float16 h = static_cast<_Float16>(acc);
    __builtin_memcpy(&o, &h, 2);
  }
  st<uint16_t>(a.out + byte, o);
}

__global__ __launch_bounds__(kBlock) void seg_reduce_kernel(SegReduceArgs a) {
  const int64_t total = a.first[a.nseg];
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t g = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; g < total; g += stride) {
    int s = 0;
    while (g >= a.first[s + 1]) ++s;  // nseg <= kSegMax: a short scan
    const int64_t e = g - a.first[s];
    const int dt = a.dtype[s], op = a.op[s];
    switch (static_cast<DType>(dt)) {
      case DType::f32: reduce_elem<float, float>(a, a.off[s] + e * 4, op); break;
      case DType::f64: reduce_elem<double, double>(a, a.off[s] + e * 8, op); break;
      case DType::i64: reduce_elem<int64_t, int64_t>(a, a.off[s] + e * 8, op); break;
      case DType::i32: reduce_elem<int32_t, int32_t>(a, a.off[s] + e * 4, op); break;
      case DType::i16: reduce_elem<int16_t, int16_t>(a, a.off[s] + e * 2, op); break;
      case DType::i8: reduce_elem<int8_t, int8_t>(a, a.off[s] + e, op); break;
      case DType::u8: reduce_elem<uint8_t, uint8_t>(a, a.off[s] + e, op); break;
      case DType::b8: {  // logical or (sum / max) and logical and (min)
        const uint8_t* p = a.rows + a.off[s] + e;
        uint8_t acc = p[0] != 0;
        for (int r = 1; r < a.ws; ++r) {
          const uint8_t v = p[r * a.row_bytes] != 0;
          acc = op == 2 ? (acc & v) : (acc | v);
        }
        a.out[a.off[s] + e] = acc;
        break;
      }
      case DType::bf16:
      case DType::f16: reduce_bytes16(a, a.off[s] + e * 2, dt, op); break;
    }
  }
}

// Snapshot of a large-state region plus this rank's device error flag in the same f32 SUM
// all-reduce: the flag words (uint32) go as exact (hi16, lo16) float pairs into this rank's slot
// of a [ws][words][2] block whose other slots are zero, so the SUM delivers every rank's flag
// and the collective that gathered flags separately is gone.
__global__ __launch_bounds__(kBlock) void snapshot_flags_kernel(const float4* __restrict__ src, float4* __restrict__ dst,
                                                                int64_t n4, const int* __restrict__ err, int words,
                                                                int rank, int ws) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
  if (blockIdx.x == 0) {
    float* slots = reinterpret_cast<float*>(dst + n4);
    for (int j = threadIdx.x; j < ws * words * 2; j += kBlock) {
      const int r = j / (2 * words), w = (j / 2) % words, half = j % 2;
      float v = 0.f;
      if (r == rank && err) {
        const uint32_t u = static_cast<uint32_t>(err[w]);
        v = static_cast<float>(half == 0 ? (u >> 16) : (u & 0xffffu));
      }
      slots[j] = v;
    }
  }
}

// [ws][words][2] summed slots -> int32 [words]: elementwise max over ranks (the engine's "max"
// flag merge), rank order irrelevant
__global__ void merge_flag_slots_kernel(const float* __restrict__ slots, int* __restrict__ out, int words, int ws) {
  const int w = threadIdx.x;
  if (w >= words) return;
  uint32_t m = 0;
  for (int r = 0; r < ws; ++r) {
    const uint32_t hi = static_cast<uint32_t>(slots[(r * words + w) * 2]);
    const uint32_t lo = static_cast<uint32_t>(slots[(r * words + w) * 2 + 1]);
    const uint32_t u = (hi << 16) | lo;
    m = u > m ? u : m;
  }
  out[w] = static_cast<int>(m);
}

}  // namespace

int launch_snapshot_flags(const void* src, void* dst, int64_t bytes, const int* err, int words, int rank, int ws,
                          hipStream_t stream) {
  if (bytes % 16 != 0 || words < 1 || words > 7 || ws < 1 || rank < 0 || rank >= ws) return -1;
  const int64_t n4 = bytes / 16;
  const int grid = stream_grid(n4 > 0 ? n4 : 1, kBlock, 1024);
  hipLaunchKernelGGL(snapshot_flags_kernel, dim3(grid), dim3(kBlock), 0, stream, static_cast<const float4*>(src),
                     static_cast<float4*>(dst), n4, err, words, rank, ws);
  return static_cast<int>(hipGetLastError());
}

int launch_merge_flag_slots(const float* slots, int* out, int words, int ws, hipStream_t stream) {
  if (words < 1 || words > 7 || ws < 1) return -1;
  hipLaunchKernelGGL(merge_flag_slots_kernel, dim3(1), dim3(kWave), 0, stream, slots, out, words, ws);
  return static_cast<int>(hipGetLastError());
}

int launch_seg_reduce(const SegReduceArgs& a, hipStream_t stream) {
  if (a.nseg <= 0 || a.nseg > kSegMax || a.ws <= 0) return -1;
  const int64_t total = a.first[a.nseg];
  if (total <= 0) return 0;
  const int grid = stream_grid(total, kBlock, 1024);
  hipLaunchKernelGGL(seg_reduce_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
