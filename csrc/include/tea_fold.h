// Grid-wide fold of per-block partial counts WITHOUT same-address atomic storms.
//
// Measured on MI355X (csrc/bench/k1_variants.hip, bs=8192 x C=1000 argmax-accuracy):
//   one float atomicAdd per block into ONE address, 2048 blocks  ->  +23 us (serialised at
//   the memory-side atomic unit, ~10 ns each); a release/acquire "last arriver" fold -> +47 us
//   (agent-scope fences per block).  This relaxed sharded fold costs +0.5 us.
//
// Scheme: blocks are hashed onto S shards (blockIdx % S).  Each shard is ONE 64-bit cell
// {hi 32: arrivals, lo 32: integer partial sum}.  A block adds (1 << 32) | partial with a
// single returning atomic; the value it gets back tells it whether it is the shard's last
// arriver and, if so, the shard's full sum (the count and the value travel in the same
// atomic, so no memory ordering between two locations is needed).  The last arriver resets
// the cell for the next launch and adds the shard total to the destination float with one
// atomic: S destination atomics per launch instead of gridDim.x.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tea {

constexpr int kFoldShards = 64;
constexpr int kFoldStride = 8;  // u64 elements between cells (64 B)

// ws: [nvals][kFoldShards * kFoldStride] u64 cells, zero-initialised once, self-cleaning.
__device__ __forceinline__ void fold_count(unsigned long long* ws, uint32_t partial, float* dst) {
  const int s = blockIdx.x % kFoldShards;
  const uint32_t members =
      gridDim.x / kFoldShards + ((gridDim.x % kFoldShards) > static_cast<uint32_t>(s) ? 1u : 0u);
  unsigned long long* cell = ws + s * kFoldStride;
  const unsigned long long inc = (1ull << 32) | partial;
  const unsigned long long old =
      __hip_atomic_fetch_add(cell, inc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (static_cast<uint32_t>(old >> 32) == members - 1) {
    const uint32_t total = static_cast<uint32_t>(old & 0xffffffffull) + partial;
    __hip_atomic_store(cell, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (total) atomicAdd(dst, static_cast<float>(total));
  }
}

}  // namespace tea
