// Shared device helpers for torcheval_amd HIP kernels (gfx950 / CDNA4 only).
//
// Conventions
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
//  * loads are 16 B per lane (Guideline 13): float4 for f32, 8 x 16-bit for bf16/f16.
//  * kernels take raw pointers + a DType tag; the pybind layer (csrc/bindings.cpp) owns the
//    torch::Tensor plumbing so kernel TUs compile in seconds (no torch headers here).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "tea_types.h"

namespace tea {

constexpr int kWave = 64;

// ------------------------------------------------------------------ scalar conversions
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}
__device__ __forceinline__ float f16_to_f32(uint16_t b) {
  _Float16 h;
  __builtin_memcpy(&h, &b, 2);
  return static_cast<float>(h);
}

// Load element i of a typed buffer as float (scalar path).
__device__ __forceinline__ float load_as_f32(const void* p, DType dt, int64_t i) {
  switch (dt) {
    case DType::f32: return static_cast<const float*>(p)[i];
    case DType::f16: return f16_to_f32(static_cast<const uint16_t*>(p)[i]);
    case DType::bf16: return bf16_to_f32(static_cast<const uint16_t*>(p)[i]);
    case DType::f64: return static_cast<float>(static_cast<const double*>(p)[i]);
    case DType::i64: return static_cast<float>(static_cast<const int64_t*>(p)[i]);
    case DType::i32: return static_cast<float>(static_cast<const int32_t*>(p)[i]);
    case DType::u8: return static_cast<float>(static_cast<const uint8_t*>(p)[i]);
    case DType::b8: return static_cast<float>(static_cast<const uint8_t*>(p)[i] != 0);
    case DType::i8: return static_cast<float>(static_cast<const int8_t*>(p)[i]);
    case DType::i16: return static_cast<float>(static_cast<const int16_t*>(p)[i]);
  }
  return 0.f;
}

__device__ __forceinline__ double load_as_f64(const void* p, DType dt, int64_t i) {
  if (dt == DType::f64) return static_cast<const double*>(p)[i];
  if (dt == DType::i64) return static_cast<double>(static_cast<const int64_t*>(p)[i]);
  return static_cast<double>(load_as_f32(p, dt, i));
}

__device__ __forceinline__ int64_t load_as_i64(const void* p, DType dt, int64_t i) {
  switch (dt) {
    case DType::i64: return static_cast<const int64_t*>(p)[i];
    case DType::i32: return static_cast<const int32_t*>(p)[i];
    case DType::u8: return static_cast<const uint8_t*>(p)[i];
    case DType::b8: return static_cast<const uint8_t*>(p)[i] != 0;
    case DType::i8: return static_cast<const int8_t*>(p)[i];
    case DType::i16: return static_cast<const int16_t*>(p)[i];
    default: return static_cast<int64_t>(load_as_f64(p, dt, i));
  }
}

// ------------------------------------------------------------------ wave reductions
__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }
__device__ __forceinline__ int wave_id() {
  return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, kWave));
  return v;
}

// torch.argmax semantics: NaN is the maximum; ties (and NaN ties) keep the lowest index.
__device__ __forceinline__ bool argmax_better(float v2, int i2, float v, int i) {
  const bool n2 = v2 != v2, n = v != v;
  if (n2 != n) return n2;
  if (n2 && n) return i2 < i;
  return (v2 > v) || (v2 == v && i2 < i);
}

__device__ __forceinline__ void wave_argmax(float& v, int& i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o, kWave);
    const int i2 = __shfl_xor(i, o, kWave);
    if (argmax_better(v2, i2, v, i)) {
      v = v2;
      i = i2;
    }
  }
}

// Block-wide sum of one value per thread into thread 0 (blockDim <= 1024, multiple of 64).
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* lds /* >= 16 entries */) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) lds[w] = v;
  __syncthreads();
  T s = T(0);
  if (threadIdx.x == 0) {
    const int nw = blockDim.x >> 6;
    for (int k = 0; k < nw; ++k) s += lds[k];
  }
  return s;
}

// Grid sizing for streaming kernels: enough waves to fill 256 CUs, capped (Guideline 11).
inline int stream_grid(int64_t work_items, int items_per_block, int cap) {
  int64_t g = (work_items + items_per_block - 1) / items_per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

}  // namespace tea
