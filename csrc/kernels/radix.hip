// K3a: segmented descending LSD radix sort of f32 scores with an int32 permutation payload
// (SURVEY.md §7.3 K3 "segmented descending radix sort").
//
// Replaces torch.sort(descending=True) in the AUROC / AUPRC pipelines: on MI355X that call
// costs ~230 us for 1M scores (rocPRIM onesweep + a post-processing pass + an index iota /
// gather pass), i.e. most of binary_auroc's time.  Here:
//   * keys are mapped to order-preserving u32 (sign flip, NaN canonicalised to +NaN so it
//     sorts first like torch, -0 folded into +0) and complemented so an ascending LSD sort
//     yields descending scores; the permutation payload is generated in the first pass (no
//     iota kernel) and the last pass writes the scores back as floats;
//   * 4 passes x 8 bits; each pass = upsweep (per-tile digit histogram, tile-major rows of
//     1 KB, plus one atomic per non-zero digit into the count of its group of kGroup tiles) ->
//     downsweep (each block forms its digit bases from the <= ngroups group counts and the
//     < kGroup tile counts before it in its group - no scan launch: v2 ran a digit-parallel scan
//     kernel between the two, 4 launches and ~20 us per 1M-key sort - then a stable scatter).  Tiles are 2048 or 4096 keys (256 threads x 8 or 16 rounds,
//     coalesced, see radix_sort_rounds); each thread loads all of its keys up front so the loads overlap (v1 loaded per round
//     and ran a single-block serial scan: ~60 us per pass at 1M).  Stable in-tile ranking uses wave64 "match" masks
//     built from 8 ballots: each lane's rank among equal digits is popc(peers & lanes_below),
//     per-wave digit counts are combined in wave order through LDS, so the scatter is stable
//     (LSD correctness) and contention-free even when every key shares a digit (typical for
//     probabilities, whose top byte is nearly constant);
//   * rows are independent segments: histogram/scan/offsets are per row, so a [C, n]
//     one-vs-rest score matrix is sorted in the same 12 launches.
#include <algorithm>
#include <cstdlib>

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kRT = 256;
// keys per thread (R) per tile of 256 * R keys, chosen per sort by radix_sort_rounds():
// 1M keys: 8 rounds (2048-key tiles, 512 blocks) 100 us vs 114 us at 16 (half the blocks
// leaves CUs idle); 100 rows x 100k: 16 rounds 402 vs 422 us (longer digit runs per tile,
// so fuller write lines, and half the blocks' fixed cost)
constexpr int kBigSort = 4 << 20;  // total keys from which 16 rounds win
constexpr int kBins = 256;
constexpr int kRWaves = kRT / 64;
constexpr int kGroup = 32;  // tiles per group count

__device__ __forceinline__ uint32_t f2key_desc(float f) {
  uint32_t u = __float_as_uint(f);
  if (f != f) u = 0x7fc00000u;      // canonical +NaN: first in descending order (torch.sort)
  if (u == 0x80000000u) u = 0u;     // -0 == +0
  const uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~asc;
}

__device__ __forceinline__ float key2f_desc(uint32_t k) {
  const uint32_t asc = ~k;
  const uint32_t u = (asc & 0x80000000u) ? (asc & 0x7fffffffu) : ~asc;
  return __uint_as_float(u);
}

__device__ __forceinline__ uint32_t load_key(const RadixArgs& a, const uint32_t* keys_in, int pass,
                                             int64_t row, int64_t i) {
  if (pass == 0) return f2key_desc(a.in[row * a.in_row_stride + i]) ^ a.key_xor;
  return keys_in[row * a.n + i];
}

// lanes (among `active`) holding the same 8-bit digit as this lane.  Per bit: one signed
// bit-field extract (0 / -1), the ballot, and an xnor + and per 32-bit half - the select form
// (`bit ? ones : ~ones`) compiled to ~9 VALU per bit, and at 10M keys the downsweep is
// VALU-bound on this match (SQ_INSTS_VALU ~2350 per wave, profiles/pmc_k3_multiclass_10m_r3.txt)
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t active) {
  uint32_t lo = static_cast<uint32_t>(active), hi = static_cast<uint32_t>(active >> 32);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_sbfe(static_cast<int>(d), b, 1));
    const uint64_t ones = __ballot(m != 0u);
    lo &= ~(static_cast<uint32_t>(ones) ^ m);
    hi &= ~(static_cast<uint32_t>(ones >> 32) ^ m);
  }
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// pass-0 payload carried instead of the source index, converted per element from the
// caller's dtype PT (compile-time, so the 16 up-front loads stay batched): KIND 1 -> f32 bits of
// the value (binary targets), KIND 2 -> int32 of the value (class labels)
template <typename PT, int KIND>
__device__ __forceinline__ uint32_t first_payload(const RadixArgs& a, int64_t row, int64_t i) {
  if constexpr (sizeof(PT) == 8) {
    // int64 targets / labels: only the low dword is loaded (one VGPR per element, no 64-bit
    // convert); binary targets and class labels both fit in int32
    const int32_t lo = static_cast<const int32_t*>(a.payload)[2 * (row * a.payload_row_stride + i)];
    if constexpr (KIND == 1) return __float_as_uint(static_cast<float>(lo));
    return static_cast<uint32_t>(lo);
  }
  const PT x = static_cast<const PT*>(a.payload)[row * a.payload_row_stride + i];
  if constexpr (KIND == 1) return __float_as_uint(static_cast<float>(x));
  return static_cast<uint32_t>(static_cast<int32_t>(x));
}

// keys of this thread's 16 striped rounds, loaded up front so the loads overlap
template <int kRounds>
__device__ __forceinline__ void load_tile(const RadixArgs& a, const uint32_t* keys_in, const uint32_t* vals_in,
                                          int pass, int64_t row, int tile, uint32_t (&k)[kRounds],
                                          uint32_t (&v)[kRounds], bool want_vals) {
  constexpr int kRTile = kRT * kRounds;
  const int64_t t0 = static_cast<int64_t>(tile) * kRTile + threadIdx.x;
  // every load from a clamped (valid) index, the tail masked afterwards: a per-lane
  // `if (i < n) load` compiled to a branch and a vmcnt(0) per round - kRounds serial round
  // trips instead of one
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int64_t i = t0 + j * kRT;
    const int64_t ic = i < a.n ? i : a.n - 1;
    k[j] = load_key(a, keys_in, pass, row, ic);
    v[j] = want_vals ? vals_in[row * a.n + ic] : 0u;
  }
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const bool ok = t0 + j * kRT < a.n;
    k[j] = ok ? k[j] : 0u;
    v[j] = ok ? v[j] : 0u;
  }
}

// hist layout: [row][tile][digit] (each block writes 1 KB contiguously).  Measured: the
// digit-major alternative (coalesced scan reads, strided upsweep stores) made the scan 12%
// faster and the upsweep 27% slower - 2.40 vs 2.31 ms per 20 1M-sample binary_auroc calls
template <int kRounds>
__global__ __launch_bounds__(kRT) void radix_upsweep_kernel(RadixArgs a, const uint32_t* keys_in, int pass) {
  constexpr int kRTile = kRT * kRounds;
  const int64_t row = blockIdx.y;
  const int tile = blockIdx.x;
  const int shift = 8 * pass;
  // LDS histograms fed by plain per-lane LDS atomics (counting needs no ranks, so no 8-ballot
  // digit match): kHCopies copies indexed by lane % kHCopies, so one atomic instruction has at
  // most 64 / kHCopies lanes on one address.  With one copy per wave, the top byte of [0, 1)
  // scores (half of them 0x3f) put ~32 lanes on one bin and the pass-3 upsweep took 31 us at
  // 100 x 100k (9.7 us for the uniform low bytes); 32 copies measured slower (16.1 vs 13.0 us
  // mean: the 32 KB of LDS costs occupancy)
  constexpr int kHCopies = 16;
  __shared__ uint32_t h[kHCopies][kBins + 1];  // +1: one digit's copies sit in different banks
#pragma unroll
  for (int q = 0; q < kHCopies; ++q) h[q][threadIdx.x] = 0;
  uint32_t k[kRounds], v[kRounds];
  load_tile(a, keys_in, nullptr, pass, row, tile, k, v, false);
  __syncthreads();
  const int hc = threadIdx.x % kHCopies;
  const int64_t t0 = static_cast<int64_t>(tile) * kRTile + threadIdx.x;
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    if (t0 + j * kRT < a.n) atomicAdd(&h[hc][(k[j] >> shift) & 0xffu], 1u);
  }
  __syncthreads();
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < kHCopies; ++q) c += h[q][threadIdx.x];
  a.hist[(row * a.tiles + tile) * kBins + threadIdx.x] = c;
  if (c) atomicAdd(&a.groups[pass * a.region + (row * a.ngroups + tile / kGroup) * kBins + threadIdx.x], c);
  // self-cleaning group counts (no memset launch): clear the region consumed last - the previous
  // pass's, or for pass 0 what the previous sort left in region 3
  const int64_t cells = pass > 0 ? a.rows * a.ngroups * kBins : static_cast<int64_t>(*a.dirty);
  uint32_t* prev = a.groups + (pass > 0 ? pass - 1 : 3) * a.region;
  const int64_t nb = static_cast<int64_t>(gridDim.x) * gridDim.y;
  for (int64_t q = (row * gridDim.x + tile) * kRT + threadIdx.x; q < cells; q += nb * kRT) prev[q] = 0u;
}

// Downsweep: wave w owns the contiguous sub-tile [w * 1024, (w + 1) * 1024) of the tile
// (round j = 64 consecutive keys), so (wave, round, lane) IS the source order and every
// wave ranks its keys with wave-private digit counters - no block barrier inside the loop.
// Then: wave-ordered offsets + per-tile digit starts (one barrier), keys/values are placed in
// LDS in sorted tile order, and written out with consecutive threads writing consecutive
// addresses of each digit run (coalesced; v1 scattered 4-byte writes straight to HBM).
// VMODE: 0 = values from the previous pass, 1 = source index (pass 0), 2 = caller payload of
// dtype PT (pass 0); separate instantiations keep the payload conversion out of passes 1-3
template <int kRounds, int VMODE, typename PT = uint32_t, int KIND = 0>
__global__ __launch_bounds__(kRT) void radix_downsweep_kernel(RadixArgs a, const uint32_t* keys_in,
                                                              const uint32_t* vals_in, uint32_t* keys_out,
                                                              uint32_t* vals_out, int pass) {
  constexpr int kRTile = kRT * kRounds;
  const int64_t row = blockIdx.y;
  const int tile = blockIdx.x;
  const int shift = 8 * pass;
  const bool last = pass == 3;
  constexpr int kSub = kRTile / kRWaves;  // keys per wave
  __shared__ uint32_t base[kBins];        // global (row-relative) start of each digit's run
  __shared__ uint32_t tstart[kBins];      // start of each digit inside the sorted tile
  __shared__ uint32_t wc[kRWaves][kBins]; // per-wave digit counts -> per-wave offsets
  __shared__ uint32_t wsum[kRWaves];
  __shared__ uint32_t sk[kRTile], sv[kRTile];
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t tbase = static_cast<int64_t>(tile) * kRTile;
  const int64_t wbase = tbase + static_cast<int64_t>(w) * kSub;
  uint32_t k[kRounds], v[kRounds], r[kRounds];
  // clamped unconditional loads, tail masked afterwards (see load_tile)
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int64_t i = wbase + j * 64 + lane;
    const int64_t ic = i < a.n ? i : a.n - 1;
    k[j] = load_key(a, keys_in, pass, row, ic);
    if constexpr (VMODE == 0) v[j] = vals_in[row * a.n + ic];
    else if constexpr (VMODE == 1) v[j] = static_cast<uint32_t>(i);
    else v[j] = first_payload<PT, KIND>(a, row, ic);
  }
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const bool ok = wbase + j * 64 + lane < a.n;
    k[j] = ok ? k[j] : 0u;
    v[j] = ok ? v[j] : 0u;
  }
#pragma unroll
  for (int q = 0; q < kBins / 64; ++q) wc[w][lane + 64 * q] = 0;
  {  // digit bases = exclusive scan of the row's digit totals + this tile's prefix in the digit:
     // totals and the prefix of whole groups from the group counts, the rest from the tile
     // counts of this tile's own group (all independent, L2-resident loads)
    const uint32_t* G = a.groups + pass * a.region + row * a.ngroups * kBins + threadIdx.x;
    const int mg = tile / kGroup;
    uint32_t tot = 0, pre = 0;
    // fixed-trip, fully unrolled chunks: every load of a chunk is in flight at once
    for (int g0 = 0; g0 < a.ngroups; g0 += 16) {
      uint32_t v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = G[static_cast<int64_t>(min(g0 + q, a.ngroups - 1)) * kBins];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = g0 + q < a.ngroups ? v[q] : 0u;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        tot += v[q];
        pre += g0 + q < mg ? v[q] : 0u;
      }
    }
    const uint32_t* H = a.hist + (row * a.tiles + static_cast<int64_t>(mg) * kGroup) * kBins + threadIdx.x;
    const int in_group = tile - mg * kGroup;  // tiles of this group before this one
    uint32_t hv[kGroup];
    const int qmax = min(kGroup, a.tiles - mg * kGroup) - 1;  // last tile of this group
#pragma unroll
    for (int q = 0; q < kGroup; ++q) hv[q] = H[static_cast<int64_t>(min(q, qmax)) * kBins];
#pragma unroll
    for (int q = 0; q < kGroup; ++q) hv[q] = q < in_group ? hv[q] : 0u;
#pragma unroll
    for (int q = 0; q < kGroup; ++q) pre += hv[q];
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q)
      if (q < w) off += wsum[q];
    base[threadIdx.x] = off + inc - tot + pre;
  }
  // wave-local stable ranks (wave-private counters; a wave's LDS ops are in program order)
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const bool valid = wbase + j * 64 + lane < a.n;
    const uint64_t active = __ballot(valid);
    const uint32_t d = (k[j] >> shift) & 0xffu;
    const uint64_t peers = match_digit(d, active);
    const uint64_t pb = peers & below;
    r[j] = wc[w][d] + static_cast<uint32_t>(__popcll(pb));
    if (valid && pb == 0ull)  // the lowest lane of the digit's peers advances its counter
      wc[w][d] += static_cast<uint32_t>(__popcll(peers));
  }
  __syncthreads();
  {  // thread t owns digit t: per-wave exclusive offsets, tile count, tile-start scan
    const int t = threadIdx.x;
    uint32_t o = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q) {
      const uint32_t c = wc[q][t];
      wc[q][t] = o;
      o += c;
    }
    uint32_t inc = o;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t u = __shfl_up(inc, s2, 64);
      if (lane >= s2) inc += u;
    }
    __syncthreads();  // wsum reuse
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q)
      if (q < w) off += wsum[q];
    tstart[t] = off + inc - o;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    if (wbase + j * 64 + lane < a.n) {
      const uint32_t d = (k[j] >> shift) & 0xffu;
      const uint32_t p = tstart[d] + wc[w][d] + r[j];
      sk[p] = k[j];
      sv[p] = v[j];
    }
  }
  __syncthreads();
  if (last && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    *a.dirty = static_cast<uint32_t>(a.rows * a.ngroups * kBins);  // for the next sort's pass 0
  const int64_t tn64 = a.n - tbase;
  const int tn = static_cast<int>(tn64 < kRTile ? tn64 : kRTile);
  if (tn == kRTile) {
    // full tile: every LDS read of the write-out issued before the dependent ones and all the
    // stores after (a rolled loop paid sk -> base / tstart -> store round trips per element)
    uint32_t kk[kRounds], vv[kRounds];
    int32_t pb[kRounds];  // base - tile start of the element's digit (may be negative)
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      kk[j] = sk[threadIdx.x + j * kRT];
      vv[j] = sv[threadIdx.x + j * kRT];
    }
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      const uint32_t d = (kk[j] >> shift) & 0xffu;
      pb[j] = static_cast<int32_t>(base[d]) - static_cast<int32_t>(tstart[d]);
    }
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      const int64_t pos = row * a.n + static_cast<int64_t>(pb[j]) + (threadIdx.x + j * kRT);
      if (last) {
        a.out_sorted[pos] = key2f_desc(kk[j] ^ a.key_xor);
        a.out_order[pos] = static_cast<int32_t>(vv[j]);
      } else {
        keys_out[pos] = kk[j];
        vals_out[pos] = vv[j];
      }
    }
    return;
  }
  for (int p = threadIdx.x; p < tn; p += kRT) {
    const uint32_t key = sk[p];
    const uint32_t d = (key >> shift) & 0xffu;
    const int64_t pos = row * a.n + base[d] + (p - tstart[d]);
    if (last) {
      a.out_sorted[pos] = key2f_desc(key ^ a.key_xor);
      a.out_order[pos] = static_cast<int32_t>(sv[p]);
    } else {
      keys_out[pos] = key;
      vals_out[pos] = sv[p];
    }
  }
}

// ---------------------------------------------------------------- onesweep
// The same sort in 5 launches instead of 8: ONE histogram kernel reads every key once and
// counts all four digits (the row totals each pass needs for its digit starts), then each pass
// ranks its tile exactly as the downsweep above and gets its tiles-before prefix in the same
// launch (decoupled look-back, Merrill & Garland / Adinets & Merrill "onesweep"), so the four
// upsweep launches and their second read of the keys are gone.
//   * a tile waits only on lower-numbered tiles of its row, and workgroups are dispatched in
//     blockIdx order per XCD, so the lowest unfinished tile never waits on an undispatched one;
//   * look-back without chained prefixes: each tile publishes its per-digit count (the data is
//     the flag: bit 31 = ready) and adds it, with an arrival count, into its group's word (32
//     tiles per group); a tile's prefix is the sum of the complete groups before its own plus
//     the counts of the tiles before it in its group - <= 2 x 16 independent agent-scope loads
//     per digit at <= 1024 tiles a row, every round trip in flight together (a chained
//     inclusive-prefix look-back serialises hops when all tiles start at once, as they do here);
//   * every hand-off word is an agent-scope (write-through) store / atomic and an agent-scope
//     load (the XCDs' L2s are not coherent), relaxed: the words carry the data themselves;
//   * self-cleaning: the status and group planes alternate between passes and each pass clears
//     the plane the previous pass used, up to the extent recorded for it (so a later sort of
//     another shape never reads stale flags); the last tile of each row in pass 3 clears the
//     row's digit totals once every tile of the row has consumed them (its look-back saw all
//     of them publish, and each publishes only after its digit-start scan).  Every spin is
//     bounded (a timeout sets hdr[8]).
#ifdef TEA_RADIX_TRACE  // csrc/bench/k3_pass_trace.hip: s_memrealtime per phase, thread 0 of every block
__device__ unsigned long long* g_radix_trace;
#define RDX_TRACE(i)                                                                             \
  do {                                                                                           \
    if (threadIdx.x == 0) g_radix_trace[(static_cast<size_t>(pass) * 4096 + blockIdx.x) * 8 + (i)] = \
        __builtin_amdgcn_s_memrealtime();                                                        \
  } while (0)
#define BKT_TRACE(region, i)                                                                     \
  do {                                                                                           \
    if (threadIdx.x == 0) g_radix_trace[(static_cast<size_t>(region) * 4096 + blockIdx.x) * 8 + (i)] = \
        __builtin_amdgcn_s_memrealtime();                                                        \
  } while (0)
#else
#define RDX_TRACE(i) \
  do {               \
  } while (0)
#define BKT_TRACE(region, i) \
  do {                       \
  } while (0)
#endif
#ifdef TEA_RADIX_TRACE
#define BKT_NBITS(v) g_radix_trace[(static_cast<size_t>(7) * 4096 + blockIdx.x) * 8] = (v)
#else
#define BKT_NBITS(v) (void)(v)
#endif
constexpr int kOSMaxTiles = 1024;
constexpr uint32_t kReady = 0x80000000u;
constexpr int kHistKeys = 16;  // keys per thread per round of the histogram kernel
constexpr int kGCopies = 8;    // copies of the digit totals (histogram block % 8): 8x fewer
                               // same-address device atomics (256 blocks on one address: ~5 us)

typedef __attribute__((address_space(1))) unsigned os_u32;
typedef __attribute__((address_space(1))) unsigned long long os_u64;

__device__ __forceinline__ void os_put(uint32_t* p, uint32_t v) {
  __hip_atomic_store((os_u32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t os_get(const uint32_t* p) {
  return __hip_atomic_load((os_u32*)(const_cast<uint32_t*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long os_get64(const unsigned long long* p) {
  return __hip_atomic_load((os_u64*)(const_cast<unsigned long long*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void os_add64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_fetch_add((os_u64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// all four digit histograms of the row's keys, one read: LDS counts (kC copies per digit, one
// per lane % kC, against same-bin contention on the near-constant top byte), then one device
// atomic per non-zero (digit, bin) into copy (block % kGCopies) of the row totals
__global__ __launch_bounds__(kRT) void onesweep_hist_kernel(RadixArgs a, int64_t per_block) {
  constexpr int kC = 8;
  __shared__ uint32_t h[4][kC][kBins + 1];
  // this sort's look-back timeout word starts clear (the passes run after this launch); the
  // previous sort's word goes to the host first (RadixArgs::os_watch)
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    if (a.os_watch != nullptr) a.os_watch[0] = a.os_hdr[8];
    a.os_hdr[8] = 0u;
  }
  for (int q = threadIdx.x; q < 4 * kC * (kBins + 1); q += kRT) (&h[0][0][0])[q] = 0u;
  __syncthreads();
  const int64_t row = blockIdx.y;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * per_block;
  const int64_t hi = lo + per_block < a.n ? lo + per_block : a.n;
  const int c = threadIdx.x % kC;
  const float* in = a.in + row * a.in_row_stride;
  for (int64_t i0 = lo; i0 < hi; i0 += kRT * kHistKeys) {
    uint32_t k[kHistKeys];
#pragma unroll
    for (int j = 0; j < kHistKeys; ++j) {  // clamped loads, all in flight; the tail masked below
      const int64_t i = i0 + j * kRT + threadIdx.x;
      k[j] = f2key_desc(in[i < hi ? i : hi - 1]) ^ a.key_xor;
    }
#pragma unroll
    for (int j = 0; j < kHistKeys; ++j) {
      if (i0 + j * kRT + threadIdx.x < hi) {
#pragma unroll
        for (int p = 0; p < 4; ++p) atomicAdd(&h[p][c][(k[j] >> (8 * p)) & 0xffu], 1u);
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < kC; ++q) v += h[p][q][threadIdx.x];
    if (v) atomicAdd(&a.os_g[((row * kGCopies + blockIdx.x % kGCopies) * 4 + p) * kBins + threadIdx.x], v);
  }
}

// K3 tile-sum fold (RadixArgs::fold_ab), run by the last pass once its sorted tile is staged in
// LDS: positions rise monotonically through the staged tile (digit runs in digit order, each
// run contiguous in the row), so each digit's run splits into <= 2 + run / 1024 pieces by
// 1024-sample output tile.  Prefix sums of (a, b) over the staged tile (thread-contiguous chunks,
// one block scan) give every piece's sums; thread d adds its run's pieces with device atomics
// (a few per block for probability scores, whose top byte takes a handful of values).
constexpr int kFoldShift = 10;  // k3::kTile = 1024-sample tiles of the scan

template <int kRounds>
__device__ __forceinline__ void fold_tile_sums(const RadixArgs& a, int64_t row, const uint32_t* sv, int tn,
                                               const uint32_t* tstart, const uint32_t* base, uint32_t cnt,
                                               double* fa, double* fb, double (*fw)[kRWaves]) {
  const int t = threadIdx.x, lane = lane_id(), w = t >> 6;
  float va[kRounds];
  double ca = 0.0, cb = 0.0;
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int p = t * kRounds + j;
    float x = 0.f;
    if (p < tn) {
      const uint32_t v = sv[p];
      x = a.payload_kind == 1 ? __uint_as_float(v)
                              : (static_cast<int64_t>(static_cast<int32_t>(v)) == row ? 1.f : 0.f);
      cb += static_cast<double>(1.f - x);
    }
    va[j] = x;
    ca += x;
  }
  double ia = ca, ib = cb;  // inclusive wave scans
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double ua = __shfl_up(ia, o, 64), ub = __shfl_up(ib, o, 64);
    if (lane >= o) {
      ia += ua;
      ib += ub;
    }
  }
  if (lane == 63) {
    fw[0][w] = ia;
    fw[1][w] = ib;
  }
  __syncthreads();
  double ra = ia - ca, rb = ib - cb;
#pragma unroll
  for (int q = 0; q < kRWaves; ++q) {
    if (q < w) {
      ra += fw[0][q];
      rb += fw[1][q];
    }
  }
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int p = t * kRounds + j;
    fa[p] = ra;
    fb[p] = rb;
    ra += va[j];
    rb += p < tn ? static_cast<double>(1.f - va[j]) : 0.0;
  }
  if (t == kRT - 1) {
    fa[kRT * kRounds] = ra;
    fb[kRT * kRounds] = rb;
  }
  __syncthreads();
  if (cnt == 0 || (a.fold_probe & 1)) return;
  const int64_t g0 = base[t], g1 = g0 + cnt;  // row-relative positions of this digit's run
  const int s0 = static_cast<int>(tstart[t]);
  double* out = a.fold_ab + row * a.fold_otiles * 2;
  for (int64_t ot = g0 >> kFoldShift; ot <= (g1 - 1) >> kFoldShift; ++ot) {
    const int64_t lo = max(g0, ot << kFoldShift), hi = min(g1, (ot + 1) << kFoldShift);
    const int ps = s0 + static_cast<int>(lo - g0), pe = s0 + static_cast<int>(hi - g0);
    atomicAdd(out + 2 * ot, fa[pe] - fa[ps]);
    atomicAdd(out + 2 * ot + 1, fb[pe] - fb[ps]);
  }
}

// one pass: load + rank as radix_downsweep_kernel, then publish / look back, then scatter
// bucket of a key in splitter-bucket mode: the number of the 255 ascending splitters below it
// (spl[255] = ~0u is never below a key): 8 LDS probes, monotone in the key
__device__ __forceinline__ uint32_t bkt_of(uint32_t key, const uint32_t* spl) {
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 128; step > 0; step >>= 1) lo += spl[lo + step - 1] < key ? step : 0u;
  return lo;
}

template <int kRounds, int VMODE, typename PT = uint32_t, int KIND = 0, bool FOLD = false, bool BKT = false>
__global__ __launch_bounds__(kRT) void onesweep_pass_kernel(RadixArgs a, const uint32_t* keys_in,
                                                            const uint32_t* vals_in, uint32_t* keys_out,
                                                            uint32_t* vals_out, int pass) {
  constexpr int kRTile = kRT * kRounds;
  constexpr int kSub = kRTile / kRWaves;
  __shared__ uint32_t base[kBins];
  __shared__ uint32_t tstart[kBins];
  __shared__ uint32_t wc[kRWaves][kBins];
  __shared__ uint32_t wsum[kRWaves];
  __shared__ uint32_t sk[kRTile], sv[kRTile];
  __shared__ double fa[FOLD ? kRTile + 1 : 1], fb[FOLD ? kRTile + 1 : 1];
  __shared__ double fw[2][kRWaves];
  __shared__ uint32_t sspl[BKT ? kBins : 1];
  __shared__ uint8_t sdg[BKT ? kRTile : 1];  // bucket mode: the staged keys' buckets (one search per key)
  uint32_t my_cnt = 0;  // this tile's count of digit threadIdx.x
  // tile id = blockIdx: workgroups are dispatched in order per XCD, so the lowest unfinished
  // tile only ever waits on finished ones.  (Ids from a counter ticket, the textbook guard,
  // cost 512 serialised same-address atomics per launch: 18.9 vs 13.2 us per pass at 1M,
  // profiles/k3_onesweep_r5.json.)
  const int64_t id = blockIdx.x;
  const int64_t row = id / a.tiles;
  const int tile = static_cast<int>(id - row * a.tiles);
  const int shift = 8 * pass;
  const bool last = pass == 3;
  if constexpr (BKT) sspl[threadIdx.x] = threadIdx.x < kBins - 1 ? a.bkt_spl[row * kBins + threadIdx.x] : ~0u;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t tbase = static_cast<int64_t>(tile) * kRTile;
  const int64_t wbase = tbase + static_cast<int64_t>(w) * kSub;
  RDX_TRACE(0);
  uint32_t k[kRounds], v[kRounds], r[kRounds];
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const int64_t i = wbase + j * 64 + lane;
    const int64_t ic = i < a.n ? i : a.n - 1;
    k[j] = load_key(a, keys_in, pass, row, ic);
    if constexpr (VMODE == 0) v[j] = vals_in[row * a.n + ic];
    else if constexpr (VMODE == 1) v[j] = static_cast<uint32_t>(i);
    else v[j] = first_payload<PT, KIND>(a, row, ic);
  }
  // the row's digit totals (histogram kernel) -> exclusive scan over the digits
  uint32_t gtot = 0;
#pragma unroll
  for (int c = 0; c < kGCopies; ++c) gtot += a.os_g[((row * kGCopies + c) * 4 + pass) * kBins + threadIdx.x];
  if constexpr (BKT) {
    if (tile == 0) a.bkt_cnt[row * kBins + threadIdx.x] = gtot;  // the bucket sizes, for the LDS stage
  }
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const bool ok = wbase + j * 64 + lane < a.n;
    k[j] = ok ? k[j] : 0u;
    v[j] = ok ? v[j] : 0u;
  }
#pragma unroll
  for (int q = 0; q < kBins / 64; ++q) wc[w][lane + 64 * q] = 0;
  uint32_t gb;
  {
    uint32_t inc = gtot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q)
      if (q < w) off += wsum[q];
    gb = off + inc - gtot;
  }
  // wave-local stable ranks (as radix_downsweep_kernel)
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t dj[BKT ? kRounds : 1];
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    const bool valid = wbase + j * 64 + lane < a.n;
    const uint64_t active = __ballot(valid);
    uint32_t d;
    if constexpr (BKT) {
      d = bkt_of(k[j], sspl);
      dj[j] = d;
    } else {
      d = (k[j] >> shift) & 0xffu;
    }
    const uint64_t peers = match_digit(d, active);
    const uint64_t pb = peers & below;
    r[j] = wc[w][d] + static_cast<uint32_t>(__popcll(pb));
    if (valid && pb == 0ull) wc[w][d] += static_cast<uint32_t>(__popcll(peers));
  }
  __syncthreads();
  RDX_TRACE(1);
  const int P = pass & 1;
  {  // thread t owns digit t
    const int t = threadIdx.x;
    uint32_t o = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q) {
      const uint32_t c = wc[q][t];
      wc[q][t] = o;
      o += c;
    }
    my_cnt = o;
    // publish this tile's count (ready-flagged) and add it to the group's word
    const int ngroups = static_cast<int>(a.ngroups);
    uint32_t* st = a.os_status + P * a.os_splane + row * a.tiles * kBins;
    unsigned long long* ga = a.os_gacc + P * a.os_gplane + row * static_cast<int64_t>(ngroups) * kBins;
    const int g = tile / kGroup;
    os_put(st + static_cast<int64_t>(tile) * kBins + t, kReady | o);
    os_add64(ga + static_cast<int64_t>(g) * kBins + t, (1ull << 32) | o);
    RDX_TRACE(2);
    uint32_t inc = o;
#pragma unroll
    for (int s2 = 1; s2 < 64; s2 <<= 1) {
      const uint32_t u = __shfl_up(inc, s2, 64);
      if (lane >= s2) inc += u;
    }
    // clear the planes the previous pass used (the next pass uses them), up to their extents
    {
      const int64_t nthr = static_cast<int64_t>(gridDim.x) * kRT;
      const int64_t me = id * kRT + t;
      uint32_t* so = a.os_status + (P ^ 1) * a.os_splane;
      const int64_t se = a.os_hdr[4 + (P ^ 1)];
      for (int64_t q = me; q < se; q += nthr) so[q] = 0u;
      unsigned long long* go = a.os_gacc + (P ^ 1) * a.os_gplane;
      const int64_t ge = a.os_hdr[6 + (P ^ 1)];
      for (int64_t q = me; q < ge; q += nthr) go[q] = 0ull;
      // pass 0 zeroes the tile-sum fold the last pass adds into (stream order separates them)
      if (VMODE != 0 && a.fold_ab != nullptr) {
        const int64_t fe = a.rows * a.fold_otiles * 2;
        for (int64_t q = me; q < fe; q += nthr) a.fold_ab[q] = 0.0;
      }
    }
    // tiles-before prefix: whole groups before this tile's group, then the group's earlier tiles
    uint32_t pre = 0;
    int spins = 0;
    for (int g0 = 0; g0 < g; g0 += 16) {
      unsigned long long gv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) gv[q] = os_get64(ga + static_cast<int64_t>(min(g0 + q, g - 1)) * kBins + t);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (g0 + q < g) {
          while ((gv[q] >> 32) < static_cast<unsigned long long>(kGroup) && spins < a.spin_limit) {
            ++spins;
            gv[q] = os_get64(ga + static_cast<int64_t>(g0 + q) * kBins + t);
          }
          pre += static_cast<uint32_t>(gv[q]);
        }
      }
    }
    for (int j0 = g * kGroup; j0 < tile; j0 += 16) {
      uint32_t sv2[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) sv2[q] = os_get(st + static_cast<int64_t>(min(j0 + q, tile - 1)) * kBins + t);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (j0 + q < tile) {
          while (!(sv2[q] & kReady) && spins < a.spin_limit) {
            ++spins;
            sv2[q] = os_get(st + static_cast<int64_t>(j0 + q) * kBins + t);
          }
          pre += sv2[q] & ~kReady;
        }
      }
    }
    if (spins >= a.spin_limit) a.os_hdr[8] = 1u;  // surfaced: K3 scans return NaN, the next sort warns
    base[t] = gb + pre;
    // the last tile of the row: every tile of the row has consumed the digit totals
    if ((last || BKT) && tile == a.tiles - 1) {
#pragma unroll
      for (int q = 0; q < kGCopies * 4; ++q) a.os_g[(row * kGCopies * 4 + q) * kBins + t] = 0u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    RDX_TRACE(3);
    uint32_t off = 0;
#pragma unroll
    for (int q = 0; q < kRWaves; ++q)
      if (q < w) off += wsum[q];
    tstart[t] = off + inc - o;
  }
  if (id == 0 && threadIdx.x == 0) {  // this pass's extents: the next pass clears them
    a.os_hdr[4 + P] = static_cast<uint32_t>(a.rows * a.tiles * kBins);
    a.os_hdr[6 + P] = static_cast<uint32_t>(a.rows * a.ngroups * kBins);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRounds; ++j) {
    if (wbase + j * 64 + lane < a.n) {
      uint32_t d;
      if constexpr (BKT) d = dj[j];
      else d = (k[j] >> shift) & 0xffu;
      const uint32_t p = tstart[d] + wc[w][d] + r[j];
      sk[p] = k[j];
      sv[p] = v[j];
      if constexpr (BKT) sdg[p] = static_cast<uint8_t>(d);
    }
  }
  __syncthreads();
  RDX_TRACE(4);
  const int64_t tn64 = a.n - tbase;
  const int tn = static_cast<int>(tn64 < kRTile ? tn64 : kRTile);
  if constexpr (FOLD) {
    if (!(a.fold_probe & 2)) fold_tile_sums<kRounds>(a, row, sv, tn, tstart, base, my_cnt, fa, fb, fw);
  }
  if (tn == kRTile) {
    uint32_t kk[kRounds], vv[kRounds];
    int32_t pb[kRounds];
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      kk[j] = sk[threadIdx.x + j * kRT];
      vv[j] = sv[threadIdx.x + j * kRT];
    }
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      const uint32_t d = BKT ? static_cast<uint32_t>(sdg[threadIdx.x + j * kRT]) : (kk[j] >> shift) & 0xffu;
      pb[j] = static_cast<int32_t>(base[d]) - static_cast<int32_t>(tstart[d]);
    }
#pragma unroll
    for (int j = 0; j < kRounds; ++j) {
      const int64_t pos = row * a.n + static_cast<int64_t>(pb[j]) + (threadIdx.x + j * kRT);
      if (last) {
        a.out_sorted[pos] = key2f_desc(kk[j] ^ a.key_xor);
        a.out_order[pos] = static_cast<int32_t>(vv[j]);
      } else {
        keys_out[pos] = kk[j];
        vals_out[pos] = vv[j];
      }
    }
    RDX_TRACE(5);
    return;
  }
  for (int p = threadIdx.x; p < tn; p += kRT) {
    const uint32_t key = sk[p];
    const uint32_t d = BKT ? static_cast<uint32_t>(sdg[p]) : (key >> shift) & 0xffu;
    const int64_t pos = row * a.n + base[d] + (p - tstart[d]);
    if (last) {
      a.out_sorted[pos] = key2f_desc(key ^ a.key_xor);
      a.out_order[pos] = static_cast<int32_t>(sv[p]);
    } else {
      keys_out[pos] = key;
      vals_out[pos] = sv[p];
    }
  }
}

// ---------------------------------------------------------------- splitter-bucket mode (opt-in)
// binary_auroc at 1M spent ~52 of its ~82 us in the four onesweep passes (each a ~13 us latency
// chain: load + rank, look-back, staging, stores; profiles/k3_pass_trace_r5.txt).  Bucket mode
// keeps ONE such pass: 255 splitters cut the row into 256 near-equal buckets (equal-frequency
// quantiles of an 8192-key sorted sample, so the bucket sizes follow the data, not the key bits:
// probabilities, whose top key bits are nearly constant, bucket as evenly as logits), the pass
// scatters the keys stably into their buckets, and one workgroup per bucket sorts it in LDS
// (packed (key, position) bitonic sort: stable) and writes the final floats and payload.
constexpr int kBktSample = 8192;
constexpr int kBktT = 1024;      // threads of the sample / bucket kernels
constexpr int kBktFast = 8192;   // keys a bucket workgroup radix-sorts in LDS (2 x 64 KB of packed pairs)
constexpr int kBktCap = 16384;   // ... or bitonic-sorts in place (the two halves as one array)
constexpr int kBktW = kBktT / 64;

// block-wide exclusive scan of one value per thread (kBktT threads); returns the block total
__device__ __forceinline__ uint32_t bkt_block_scan(uint32_t v, uint32_t& excl, uint32_t* ws) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  uint32_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(inc, o, 64);
    if (lane >= o) inc += u;
  }
  if (lane == 63) ws[w] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < kBktW; ++q) {
    const uint32_t x = ws[q];
    off += q < w ? x : 0u;
    tot += x;
  }
  excl = off + inc - v;
  __syncthreads();
  return tot;
}

// XOR of the block's min and max key over e[0, N) (the high words): the key bits that differ
__device__ __forceinline__ uint32_t bkt_key_spread(const unsigned long long* e, int N, uint32_t* ws) {
  uint32_t mn = ~0u, mx = 0u;
  for (int i = threadIdx.x; i < N; i += kBktT) {
    const uint32_t k = static_cast<uint32_t>(e[i] >> 32);
    mn = k < mn ? k : mn;
    mx = k > mx ? k : mx;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t a = __shfl_xor(mn, o, 64), b = __shfl_xor(mx, o, 64);
    mn = a < mn ? a : mn;
    mx = b > mx ? b : mx;
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    ws[w] = mn;
    ws[kBktW + w] = mx;
  }
  __syncthreads();
  mn = ~0u;
  mx = 0u;
#pragma unroll
  for (int q = 0; q < kBktW; ++q) {
    mn = ws[q] < mn ? ws[q] : mn;
    mx = ws[kBktW + q] > mx ? ws[kBktW + q] : mx;
  }
  __syncthreads();
  return mn ^ mx;
}

// stable LSD radix sort of N <= kBktFast packed (key << 32 | value) words by their key bits
// [0, nbits), 8 bits per pass, ping-pong A <-> B; returns the buffer holding the result.  Wave w
// ranks the contiguous chunk [w C, (w + 1) C) in 64-key rounds (onesweep's match-mask ranks),
// the digit bases combine the waves in order: stable.
__device__ __forceinline__ unsigned long long* lds_radix_u64(unsigned long long* A, unsigned long long* B, int N, int nbits,
                                             uint32_t (*wcnt)[kBins], uint32_t* dbase, uint32_t* ws) {
  constexpr int kMaxR = kBktFast / kBktT;  // rounds per wave
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int C = ((N + kBktW - 1) / kBktW + 63) / 64 * 64;
  const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  for (int sh = 0; sh < nbits; sh += 8) {
    if (sh == 0) BKT_TRACE(8, 0);
    for (int q = lane; q < kBins; q += 64) wcnt[w][q] = 0u;
    __syncthreads();
    unsigned long long el[kMaxR];
    uint32_t rk[kMaxR];
#pragma unroll
    for (int r = 0; r < kMaxR; ++r) {
      const int i = w * C + r * 64 + lane;
      const bool valid = r * 64 < C && i < N;
      el[r] = valid ? A[i] : 0ull;
      const uint32_t d = static_cast<uint32_t>(el[r] >> (32 + sh)) & 0xffu;
      const uint64_t active = __ballot(valid);
      const uint64_t peers = match_digit(d, active);
      const uint64_t pb = peers & below;
      rk[r] = wcnt[w][d] + static_cast<uint32_t>(__popcll(pb));
      if (valid && pb == 0ull) wcnt[w][d] += static_cast<uint32_t>(__popcll(peers));
    }
    __syncthreads();
    if (sh == 0) BKT_TRACE(8, 1);
    uint32_t tot = 0;
    if (threadIdx.x < kBins) {
#pragma unroll
      for (int q = 0; q < kBktW; ++q) {
        const uint32_t c = wcnt[q][threadIdx.x];
        wcnt[q][threadIdx.x] = tot;
        tot += c;
      }
    }
    uint32_t ex = 0;
    bkt_block_scan(tot, ex, ws);
    if (threadIdx.x < kBins) dbase[threadIdx.x] = ex;
    __syncthreads();
    if (sh == 0) BKT_TRACE(8, 2);
#pragma unroll
    for (int r = 0; r < kMaxR; ++r) {
      const int i = w * C + r * 64 + lane;
      const uint32_t d = static_cast<uint32_t>(el[r] >> (32 + sh)) & 0xffu;
      if (r * 64 < C && i < N) B[dbase[d] + wcnt[w][d] + rk[r]] = el[r];
    }
    __syncthreads();
    if (sh == 0) BKT_TRACE(8, 3);
    unsigned long long* t = A;
    A = B;
    B = t;
  }
  return A;
}

// ascending bitonic sort of e[0, P) in place (P a power of two <= kBktCap): the tier for buckets
// between kBktFast and kBktCap keys
__device__ void lds_bitonic(unsigned long long* e, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P / 2; i += kBktT) {
        const int lo = ((i & ~(j - 1)) << 1) | (i & (j - 1));  // i-th pair (lo, lo + j)
        const int hi = lo + j;
        const unsigned long long x = e[lo], y = e[hi];
        const bool up = (lo & k) == 0;
        if ((x > y) == up) {
          e[lo] = y;
          e[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// one block per row: sorted 8192-key sample (LDS radix) -> 255 splitters (its ranks 32, 64, ...)
__global__ __launch_bounds__(kBktT) void bkt_split_kernel(RadixArgs a) {
  __shared__ unsigned long long e[2][kBktSample];
  __shared__ uint32_t wcnt[kBktW][kBins];
  __shared__ uint32_t dbase[kBins];
  __shared__ uint32_t ws[2 * kBktW];
  const int64_t row = blockIdx.x;
  const float* in = a.in + row * a.in_row_stride;
  BKT_TRACE(6, 0);
  for (int i = threadIdx.x; i < kBktSample; i += kBktT)
    e[0][i] = static_cast<unsigned long long>(f2key_desc(in[static_cast<int64_t>(i) * a.n / kBktSample]) ^ a.key_xor) << 32;
  __syncthreads();
  BKT_TRACE(6, 1);
  const uint32_t spread = bkt_key_spread(e[0], kBktSample, ws);
  const int nbits = spread ? 32 - __clz(static_cast<int>(spread)) : 0;
  const unsigned long long* s = lds_radix_u64(e[0], e[1], kBktSample, nbits, wcnt, dbase, ws);
  BKT_TRACE(6, 2);
  if (threadIdx.x < kBins - 1)
    a.bkt_spl[row * kBins + threadIdx.x] = static_cast<uint32_t>(s[(threadIdx.x + 1) * (kBktSample / kBins) - 1] >> 32);
}

// the bucket histogram into digit-total slot 0 (as onesweep_hist_kernel's pass-0 digit)
__global__ __launch_bounds__(kRT) void bkt_hist_kernel(RadixArgs a, int64_t per_block) {
  constexpr int kC = 8;
  __shared__ uint32_t h[kC][kBins + 1];
  __shared__ uint32_t spl[kBins];
  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    if (a.os_watch != nullptr) a.os_watch[0] = a.os_hdr[8];
    a.os_hdr[8] = 0u;
  }
  const int64_t row = blockIdx.y;
  for (int q = threadIdx.x; q < kC * (kBins + 1); q += kRT) (&h[0][0])[q] = 0u;
  spl[threadIdx.x] = threadIdx.x < kBins - 1 ? a.bkt_spl[row * kBins + threadIdx.x] : ~0u;
  __syncthreads();
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * per_block;
  const int64_t hi = lo + per_block < a.n ? lo + per_block : a.n;
  const int c = threadIdx.x % kC;
  const float* in = a.in + row * a.in_row_stride;
  for (int64_t i0 = lo; i0 < hi; i0 += kRT * kHistKeys) {
    uint32_t k[kHistKeys];
#pragma unroll
    for (int j = 0; j < kHistKeys; ++j) {
      const int64_t i = i0 + j * kRT + threadIdx.x;
      k[j] = f2key_desc(in[i < hi ? i : hi - 1]) ^ a.key_xor;
    }
#pragma unroll
    for (int j = 0; j < kHistKeys; ++j)
      if (i0 + j * kRT + threadIdx.x < hi) atomicAdd(&h[c][bkt_of(k[j], spl)], 1u);
  }
  __syncthreads();
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < kC; ++q) v += h[q][threadIdx.x];
  if (v) atomicAdd(&a.os_g[((row * kGCopies + blockIdx.x % kGCopies) * 4 + 0) * kBins + threadIdx.x], v);
}


// one block per (bucket, row): the bucket's keys (stably scattered by the pass into keys0 /
// vals0 at the bucket's offset) sorted in LDS as packed (key << 32 | position) pairs - equal
// keys keep their input order - then written out as the sorted floats and their payload.  A
// bucket over kBktCap keys (a tie group larger than ~n / 256 lands in one bucket at its upper
// splitter) puts the keys equal to that splitter after the LDS-sorted rest, in input order; a
// rest still over kBktCap (never for near-continuous scores) takes a slow single-workgroup LSD
// sort through keys1 / vals1.  The blocks also clear the status / group plane the pass used.
__global__ __launch_bounds__(kBktT) void bkt_sort_kernel(RadixArgs a) {
  __shared__ unsigned long long e[kBktCap];  // two kBktFast halves for the radix tier
  __shared__ uint32_t ws[2 * kBktW];
  __shared__ uint32_t hist[kBins];
  __shared__ uint32_t wcnt[kBktW][kBins];
  __shared__ uint32_t dbase[kBins];
  const int b = blockIdx.x;
  const int64_t row = blockIdx.y;
  BKT_TRACE(5, 0);
  {  // the pass's status / group plane (0), grid-stride over every block
    const int64_t nthr = static_cast<int64_t>(gridDim.x) * gridDim.y * kBktT;
    const int64_t me = (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * kBktT + threadIdx.x;
    const int64_t se = a.os_hdr[4], ge = a.os_hdr[6];
    for (int64_t q = me; q < se; q += nthr) a.os_status[q] = 0u;
    for (int64_t q = me; q < ge; q += nthr) a.os_gacc[q] = 0ull;
  }
  // this bucket's offset (exclusive scan of the bucket sizes) and size
  __shared__ uint32_t s_off;
  {
    const uint32_t cv = threadIdx.x < kBins ? a.bkt_cnt[row * kBins + threadIdx.x] : 0u;
    uint32_t ex = 0;
    bkt_block_scan(cv, ex, ws);
    if (threadIdx.x == static_cast<unsigned>(b)) s_off = ex;
    __syncthreads();
  }
  const uint32_t off = s_off;
  const uint32_t cnt = a.bkt_cnt[row * kBins + b];
  BKT_TRACE(5, 1);
  if (cnt == 0) return;
  const int64_t base = row * a.n + off;
  const uint32_t* kin = a.keys0 + base;
  const uint32_t* vin = a.vals0 + base;
  float* os = a.out_sorted + base;
  int32_t* oo = a.out_order + base;
  const uint32_t split = b < kBins - 1 ? a.bkt_spl[row * kBins + b] : ~0u;
  // keys other than the upper splitter (all of them when the bucket fits)
  const bool fits = cnt <= static_cast<uint32_t>(kBktCap);
  uint32_t m = cnt;
  if (!fits) {
    uint32_t mine = 0;
    for (uint32_t i = threadIdx.x; i < cnt; i += kBktT) mine += kin[i] != split ? 1u : 0u;
    uint32_t ex = 0;
    m = bkt_block_scan(mine, ex, ws);
  }
  if (m <= static_cast<uint32_t>(kBktCap)) {
    const bool radix = m <= static_cast<uint32_t>(kBktFast);
    int P = 64;
    while (P < static_cast<int>(m)) P <<= 1;
    const int fill = radix ? static_cast<int>(m) : P;
    if (fits) {
      for (int i = threadIdx.x; i < fill; i += kBktT)
        e[i] = i < static_cast<int>(cnt) ? (static_cast<unsigned long long>(kin[i]) << 32) | static_cast<uint32_t>(i) : ~0ull;
    } else {
      // stable compaction of the non-splitter keys, then the splitter's tie run in input order
      uint32_t done_ne = 0, done_eq = 0;
      for (uint32_t i0 = 0; i0 < cnt; i0 += kBktT) {
        const uint32_t i = i0 + threadIdx.x;
        const bool valid = i < cnt;
        const uint32_t key = valid ? kin[i] : split;
        const bool ne = valid && key != split;
        uint32_t ex_ne = 0, ex_eq = 0;
        const uint32_t t_ne = bkt_block_scan(ne ? 1u : 0u, ex_ne, ws);
        const uint32_t t_eq = bkt_block_scan(valid && !ne ? 1u : 0u, ex_eq, ws);
        if (ne) e[done_ne + ex_ne] = (static_cast<unsigned long long>(key) << 32) | i;
        if (valid && !ne) {
          os[m + done_eq + ex_eq] = key2f_desc(split ^ a.key_xor);
          oo[m + done_eq + ex_eq] = static_cast<int32_t>(vin[i]);
        }
        done_ne += t_ne;
        done_eq += t_eq;
      }
      for (int i = static_cast<int>(m) + threadIdx.x; i < fill; i += kBktT) e[i] = ~0ull;
    }
    __syncthreads();
    BKT_TRACE(5, 2);
    const unsigned long long* r = e;
    if (radix) {  // LSD over the key bits that differ inside the bucket (2-3 passes for scores)
      const uint32_t spread = bkt_key_spread(e, static_cast<int>(m), ws);
      const int nbits = spread ? 32 - __clz(static_cast<int>(spread)) : 0;
      BKT_TRACE(5, 3);
      if (threadIdx.x == 0) BKT_NBITS(nbits);
      r = lds_radix_u64(e, e + kBktFast, static_cast<int>(m), nbits, wcnt, dbase, ws);
    } else {
      lds_bitonic(e, P);
    }
    BKT_TRACE(5, 4);
    for (int i = threadIdx.x; i < static_cast<int>(m); i += kBktT) {
      const unsigned long long x = r[i];
      os[i] = key2f_desc(static_cast<uint32_t>(x >> 32) ^ a.key_xor);
      oo[i] = static_cast<int32_t>(vin[static_cast<uint32_t>(x)]);
    }
    BKT_TRACE(5, 5);
    return;
  }
  // slow path: stable LSD radix sort of the whole bucket by this workgroup alone, 8 bits per
  // pass, ping-pong keys0 / vals0 <-> keys1 / vals1 at the bucket's offset (chunks of kBktT keys
  // in order; per-wave stable ranks as the onesweep passes; running digit bases)
  uint32_t* k2 = a.keys1 + base;
  uint32_t* v2 = a.vals1 + base;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  for (int pass = 0; pass < 4; ++pass) {
    const uint32_t* ks = pass & 1 ? k2 : kin;
    const uint32_t* vs = pass & 1 ? v2 : vin;
    uint32_t* kd = pass & 1 ? const_cast<uint32_t*>(kin) : k2;
    uint32_t* vd = pass & 1 ? const_cast<uint32_t*>(vin) : v2;
    const int sh = 8 * pass;
    if (threadIdx.x < kBins) hist[threadIdx.x] = 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < cnt; i += kBktT) atomicAdd(&hist[(ks[i] >> sh) & 0xffu], 1u);
    __syncthreads();
    {
      uint32_t ex = 0;
      const uint32_t hv = threadIdx.x < kBins ? hist[threadIdx.x] : 0u;
      bkt_block_scan(hv, ex, ws);
      if (threadIdx.x < kBins) dbase[threadIdx.x] = ex;
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < cnt; i0 += kBktT) {
      const uint32_t i = i0 + threadIdx.x;
      const bool valid = i < cnt;
      const uint32_t key = valid ? ks[i] : 0u;
      const uint32_t val = valid ? vs[i] : 0u;
      for (int q = lane; q < kBins; q += 64) wcnt[w][q] = 0u;
      __syncthreads();
      const uint64_t active = __ballot(valid);
      const uint32_t d = (key >> sh) & 0xffu;
      const uint64_t peers = match_digit(d, active);
      const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
      const uint32_t rk = static_cast<uint32_t>(__popcll(peers & below));
      if (valid && (peers & below) == 0ull) wcnt[w][d] = static_cast<uint32_t>(__popcll(peers));
      __syncthreads();
      uint32_t pre = 0;
      for (int q = 0; q < w; ++q) pre += wcnt[q][d];
      if (valid) {
        const uint32_t pos = dbase[d] + pre + rk;
        kd[pos] = key;
        vd[pos] = val;
      }
      __syncthreads();
      if (threadIdx.x < kBins) {
        uint32_t add = 0;
        for (int q = 0; q < kBktW; ++q) add += wcnt[q][threadIdx.x];
        dbase[threadIdx.x] += add;
      }
      __syncthreads();
    }
    __syncthreads();
  }
  // 4 passes: the result is back in keys0 / vals0
  for (uint32_t i = threadIdx.x; i < cnt; i += kBktT) {
    os[i] = key2f_desc(kin[i] ^ a.key_xor);
    oo[i] = static_cast<int32_t>(vin[i]);
  }
}

// [n, C] row-major -> [C, n] (LDS-tiled 64 x 64 transpose; coalesced both ways)
__global__ __launch_bounds__(kRT) void transpose_kernel(const float* in, int64_t n, int64_t c, int64_t ld_in,
                                                        float* out) {
  __shared__ float t[64][65];
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * 64, c0 = static_cast<int64_t>(blockIdx.y) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += kRT / 64) {
    const int64_t i = i0 + r, cc = c0 + tx;
    t[r][tx] = (i < n && cc < c) ? in[i * ld_in + cc] : 0.f;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += kRT / 64) {
    const int64_t cc = c0 + r, i = i0 + tx;
    if (cc < c && i < n) out[cc * n + i] = t[tx][r];
  }
}

// The same transpose with 16-B accesses both ways (in 16-B aligned with ld_in % 4 == 0, out
// with n % 4 == 0): a thread loads 4 consecutive columns of a row and stores 4 consecutive
// samples of an output row (4 strided LDS reads).  One 4-byte access per element made the
// [100k, 100] case 28 us (~2.8 TB/s; profiles/rocprof_multiclass_auroc_100k_x100_kernel_stats_r3.csv).
__global__ __launch_bounds__(kRT) void transpose4_kernel(const float* in, int64_t n, int64_t c, int64_t ld_in,
                                                         float* out) {
  __shared__ float t[64][65];
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * 64, c0 = static_cast<int64_t>(blockIdx.y) * 64;
  const int q = threadIdx.x & 15, ty = threadIdx.x >> 4;  // 16 threads x 4 values per 64-wide row
  float4 v[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {  // every load issued before any LDS store
    const int64_t i = i0 + ty + 16 * p, cc = c0 + 4 * q;
    v[p] = (i < n && cc < c) ? *reinterpret_cast<const float4*>(in + i * ld_in + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = ty + 16 * p;
    t[r][4 * q] = v[p].x;
    t[r][4 * q + 1] = v[p].y;
    t[r][4 * q + 2] = v[p].z;
    t[r][4 * q + 3] = v[p].w;
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const int r = ty + 16 * p;  // output row c0 + r, samples i0 + 4q .. 4q + 3
    const int64_t cc = c0 + r, i = i0 + 4 * q;
    if (cc < c && i < n)
      *reinterpret_cast<float4*>(out + cc * n + i) = make_float4(t[4 * q][r], t[4 * q + 1][r], t[4 * q + 2][r], t[4 * q + 3][r]);
  }
}

}  // namespace

int radix_sort_rounds(int64_t rows, int64_t n) {
  // TORCHEVAL_AMD_K3_ROUNDS=8|16 forces the tiling (A/B); default: 16 from kBigSort keys
  static const int forced = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K3_ROUNDS");
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v == 8 || v == 16 ? v : 0;
  }();
  if (forced) return forced;
  return rows * n >= kBigSort ? 16 : 8;
}

int64_t radix_sort_tiles(int64_t rows, int64_t n) {
  const int64_t tile = static_cast<int64_t>(kRT) * radix_sort_rounds(rows, n);
  return (n + tile - 1) / tile;
}

int64_t radix_sort_groups(int64_t tiles) { return (tiles + kGroup - 1) / kGroup; }

int launch_transpose_f32(const float* in, int64_t n, int64_t c, int64_t ld_in, float* out, hipStream_t stream) {
  if (n <= 0 || c <= 0) return 0;
  const dim3 grid(static_cast<unsigned>((n + 63) / 64), static_cast<unsigned>((c + 63) / 64));
  // 16-B path: c and n multiples of 4 (whole float4s never straddle the edge), aligned rows
  const bool v4 = c % 4 == 0 && n % 4 == 0 && ld_in % 4 == 0 && reinterpret_cast<uintptr_t>(in) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out) % 16 == 0;
  if (v4) hipLaunchKernelGGL(transpose4_kernel, grid, dim3(kRT), 0, stream, in, n, c, ld_in, out);
  else hipLaunchKernelGGL(transpose_kernel, grid, dim3(kRT), 0, stream, in, n, c, ld_in, out);
  return static_cast<int>(hipGetLastError());
}

namespace {

template <int R>
int radix_passes(const RadixArgs& a, hipStream_t stream) {
  const dim3 grid(static_cast<unsigned>(a.tiles), static_cast<unsigned>(a.rows));
  const uint32_t* kin[4] = {nullptr, a.keys0, a.keys1, a.keys0};
  const uint32_t* vin[4] = {nullptr, a.vals0, a.vals1, a.vals0};
  uint32_t* kout[4] = {a.keys0, a.keys1, a.keys0, nullptr};
  uint32_t* vout[4] = {a.vals0, a.vals1, a.vals0, nullptr};
  for (int p = 0; p < 4; ++p) {
    hipLaunchKernelGGL(radix_upsweep_kernel<R>, grid, dim3(kRT), 0, stream, a, kin[p], p);
#define TEA_DOWNSWEEP(...) \
  hipLaunchKernelGGL((radix_downsweep_kernel<R, __VA_ARGS__>), grid, dim3(kRT), 0, stream, a, kin[p], vin[p], kout[p], vout[p], p)
    if (p > 0) {
      TEA_DOWNSWEEP(0);
    } else if (a.payload_kind == 0) {
      TEA_DOWNSWEEP(1);
    } else if (a.payload_kind == 1) {
      switch (a.payload_dt) {
        case DType::f32: TEA_DOWNSWEEP(2, float, 1); break;
        case DType::i64: TEA_DOWNSWEEP(2, int64_t, 1); break;
        case DType::i32: TEA_DOWNSWEEP(2, int32_t, 1); break;
        case DType::u8: case DType::b8: TEA_DOWNSWEEP(2, uint8_t, 1); break;
        default: return -2;
      }
    } else {
      switch (a.payload_dt) {
        case DType::i64: TEA_DOWNSWEEP(2, int64_t, 2); break;
        case DType::i32: TEA_DOWNSWEEP(2, int32_t, 2); break;
        default: return -2;
      }
    }
#undef TEA_DOWNSWEEP
  }
  return static_cast<int>(hipGetLastError());
}

template <int R>
int radix_onesweep(const RadixArgs& a, hipStream_t stream) {
  // histogram: one 4096-key round per block (245 blocks at 1M keys; many-row sorts get their
  // parallelism from the rows: 2 blocks per 100k-key row ran 13 serial rounds each)
  // TORCHEVAL_AMD_K3_HIST_ROUNDS (A/B): 4096-key rounds per histogram block (fewer blocks, fewer
  // device atomics into the digit totals, more serial rounds per block)
  static const int hist_rounds = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K3_HIST_ROUNDS");
    const int v = e != nullptr ? std::atoi(e) : 1;
    return v >= 1 && v <= 16 ? v : 1;
  }();
  const int64_t per = static_cast<int64_t>(kRT) * kHistKeys * hist_rounds;
  const dim3 hgrid(static_cast<unsigned>((a.n + per - 1) / per), static_cast<unsigned>(a.rows));
  hipLaunchKernelGGL(onesweep_hist_kernel, hgrid, dim3(kRT), 0, stream, a, per);
  const dim3 grid(static_cast<unsigned>(a.rows * a.tiles));
  const uint32_t* kin[4] = {nullptr, a.keys0, a.keys1, a.keys0};
  const uint32_t* vin[4] = {nullptr, a.vals0, a.vals1, a.vals0};
  uint32_t* kout[4] = {a.keys0, a.keys1, a.keys0, nullptr};
  uint32_t* vout[4] = {a.vals0, a.vals1, a.vals0, nullptr};
  for (int p = 0; p < 4; ++p) {
#define TEA_PASS(...) \
  hipLaunchKernelGGL((onesweep_pass_kernel<R, __VA_ARGS__>), grid, dim3(kRT), 0, stream, a, kin[p], vin[p], kout[p], vout[p], p)
    if (p == 3 && a.fold_ab != nullptr) {
      TEA_PASS(0, uint32_t, 0, true);
    } else if (p > 0) {
      TEA_PASS(0);
    } else if (a.payload_kind == 0) {
      TEA_PASS(1);
    } else if (a.payload_kind == 1) {
      switch (a.payload_dt) {
        case DType::f32: TEA_PASS(2, float, 1); break;
        case DType::i64: TEA_PASS(2, int64_t, 1); break;
        case DType::i32: TEA_PASS(2, int32_t, 1); break;
        case DType::u8: case DType::b8: TEA_PASS(2, uint8_t, 1); break;
        default: return -2;
      }
    } else {
      switch (a.payload_dt) {
        case DType::i64: TEA_PASS(2, int64_t, 2); break;
        case DType::i32: TEA_PASS(2, int32_t, 2); break;
        default: return -2;
      }
    }
#undef TEA_PASS
  }
  return static_cast<int>(hipGetLastError());
}

template <int R>
int radix_bucket(const RadixArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL(bkt_split_kernel, dim3(static_cast<unsigned>(a.rows)), dim3(kBktT), 0, stream, a);
  const int64_t per = static_cast<int64_t>(kRT) * kHistKeys;
  const dim3 hgrid(static_cast<unsigned>((a.n + per - 1) / per), static_cast<unsigned>(a.rows));
  hipLaunchKernelGGL(bkt_hist_kernel, hgrid, dim3(kRT), 0, stream, a, per);
  const dim3 grid(static_cast<unsigned>(a.rows * a.tiles));
#define TEA_BPASS(...) \
  hipLaunchKernelGGL((onesweep_pass_kernel<R, __VA_ARGS__>), grid, dim3(kRT), 0, stream, a, nullptr, nullptr, a.keys0, a.vals0, 0)
  if (a.payload_kind == 0) {
    TEA_BPASS(1, uint32_t, 0, false, true);
  } else if (a.payload_kind == 1) {
    switch (a.payload_dt) {
      case DType::f32: TEA_BPASS(2, float, 1, false, true); break;
      case DType::i64: TEA_BPASS(2, int64_t, 1, false, true); break;
      case DType::i32: TEA_BPASS(2, int32_t, 1, false, true); break;
      case DType::u8: case DType::b8: TEA_BPASS(2, uint8_t, 1, false, true); break;
      default: return -2;
    }
  } else {
    switch (a.payload_dt) {
      case DType::i64: TEA_BPASS(2, int64_t, 2, false, true); break;
      case DType::i32: TEA_BPASS(2, int32_t, 2, false, true); break;
      default: return -2;
    }
  }
#undef TEA_BPASS
  hipLaunchKernelGGL(bkt_sort_kernel, dim3(kBins, static_cast<unsigned>(a.rows)), dim3(kBktT), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

bool radix_bucket_ok(int64_t rows, int64_t n) {
  // opt-in (TORCHEVAL_AMD_K3_BUCKET=1, read per sort): measured slower than the four onesweep
  // passes at 1M (115 vs 85 us per binary_auroc, profiles/k3_bucket_attempt_r6.json) - its LDS
  // stages (the 8192-key sample sort on one CU, the per-bucket LSD) cost 5-6 us per 8-bit pass
  const char* e = std::getenv("TORCHEVAL_AMD_K3_BUCKET");
  const bool on = e != nullptr && e[0] == '1';
  // from 64k keys (below, the sample is most of the row) to 2M per row (~8k keys per bucket; the
  // LDS stage holds 16k)
  return on && radix_onesweep_ok(rows, n) && n >= (int64_t{1} << 16) && n <= (int64_t{2} << 20);
}

bool radix_onesweep_ok(int64_t rows, int64_t n) {
  // few long rows only: at 100 rows x 100k the legacy sort stays ahead (361 vs 370 us for
  // multiclass_auroc, profiles/k3_onesweep_r5.json): short rows leave the look-back little to save
  const int64_t tiles = radix_sort_tiles(rows, n);
  return rows > 0 && rows <= 8 && n > 0 && tiles <= kOSMaxTiles && rows * tiles * kBins < (int64_t{1} << 31);
}

int64_t radix_onesweep_status_words(int64_t rows, int64_t n) { return rows * radix_sort_tiles(rows, n) * kBins; }

int64_t radix_onesweep_group_words(int64_t rows, int64_t n) {
  return rows * radix_sort_groups(radix_sort_tiles(rows, n)) * kBins;
}

int launch_radix_sort_desc(const RadixArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.rows <= 0) return 0;
  if (a.tiles != radix_sort_tiles(a.rows, a.n)) return -2;  // workspace sized for another tiling
  if (a.os_hdr != nullptr) {
    if (!radix_onesweep_ok(a.rows, a.n) || a.os_splane < radix_onesweep_status_words(a.rows, a.n) ||
        a.os_gplane < radix_onesweep_group_words(a.rows, a.n))
      return -2;
    if (a.fold_ab != nullptr && ((a.payload_kind != 1 && a.payload_kind != 2) ||
                                 a.fold_otiles != ((a.n + (1 << kFoldShift) - 1) >> kFoldShift)))
      return -2;
    if (a.bkt_spl != nullptr && a.bkt_cnt != nullptr && a.fold_ab == nullptr && radix_bucket_ok(a.rows, a.n))
      return radix_sort_rounds(a.rows, a.n) == 16 ? radix_bucket<16>(a, stream) : radix_bucket<8>(a, stream);
    return radix_sort_rounds(a.rows, a.n) == 16 ? radix_onesweep<16>(a, stream) : radix_onesweep<8>(a, stream);
  }
  return radix_sort_rounds(a.rows, a.n) == 16 ? radix_passes<16>(a, stream) : radix_passes<8>(a, stream);
}

}  // namespace tea
