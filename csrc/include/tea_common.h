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

// ------------------------------------------------------------------ 16-B loads at 4-B alignment
// gfx950 serves a global_load_dwordx4 from any 4-B-aligned address at the aligned rate
// (csrc/bench/unaligned_probe.hip, profiles/unaligned_probe_r5.txt: 8192 x 1001 f32 rows 6.0-6.1 us
// vs 5.9 us for 8192 x 1000; a column walk 5.8 us at both widths).  Rows of an odd width therefore
// keep 16-B loads: the type below tells the compiler the address is only 4-B aligned (so it must
// not assume more), and the load is still one dwordx4.
typedef float f4u_t __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ float4 load_f4u(const float* p) {
  const f4u_t v = *reinterpret_cast<const f4u_t*>(p);
  return make_float4(v.x, v.y, v.z, v.w);
}

// ------------------------------------------------------------------ write-through hand-off
// Per-block partials handed to the block that arrives last on a ticket, inside one launch
// (MI355X_MICROARCH.md, visibility table row 1): every partial is stored write-through (sc1:
// an agent-scope relaxed atomic store, GLOBAL address space so it is never a flat store),
// every storing wave drains (vmcnt(0)), the workgroup barrier, then ONE lane adds to the
// ticket; the block whose add returns the last count reads the partials with sc1 loads only.
// No release / acquire fence (each costs a buffer_wbl2 / buffer_inv of ~1.7 us).
typedef __attribute__((address_space(1))) unsigned long long wt_u64;
typedef __attribute__((address_space(1))) unsigned wt_u32;

__device__ __forceinline__ void wt_store(double* p, double v) {
  __hip_atomic_store((wt_u64*)(p), static_cast<unsigned long long>(__double_as_longlong(v)),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double wt_load(const double* p) {
  return __longlong_as_double(static_cast<long long>(
      __hip_atomic_load((wt_u64*)(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)));
}
__device__ __forceinline__ void wt_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Called by EVERY thread after its write-through stores: drains, joins the barrier, and returns
// (block-uniformly) whether this block drew the last of `expected` tickets.  The last block
// resets the ticket (self-cleaning workspace) and may then wt_load every partial.
__device__ __forceinline__ bool wt_arrive_last(unsigned* ticket, unsigned expected) {
  __shared__ int s_last;
  wt_drain();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add((wt_u32*)(ticket), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const bool last = t == expected - 1;
    if (last) __hip_atomic_store((wt_u32*)(ticket), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last ? 1 : 0;
  }
  __syncthreads();
  return s_last != 0;
}

// Deferred-mode partial: ADD v to a pending slot this block alone writes in this launch, as a
// no-return FP64 atomic (global_atomic_add_f64): fire and forget, where a plain += would wait a
// full memory round trip for the old value at the end of every block.  One writer per slot per
// launch and stream-ordered launches keep the sums deterministic.
__device__ __forceinline__ void pend_add(double* p, double v) { unsafeAtomicAdd(p, v); }

// Grid sizing for streaming kernels: enough waves to fill 256 CUs, capped (Guideline 11).
inline int stream_grid(int64_t work_items, int items_per_block, int cap) {
  int64_t g = (work_items + items_per_block - 1) / items_per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

}  // namespace tea
