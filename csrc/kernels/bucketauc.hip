// K3b: bucketed one-row binary AUROC / AUPRC without a global sort (4 launches).
//
// Reference: torcheval/metrics/functional/classification/auroc.py:115-152 (sort desc -> tie
// mask -> cumsum TP/FP -> trapz) and auprc.py / precision_recall_curve.py (same prefix, then
// average precision).  Both areas only need, per tie group in descending-score order, the
// positive / negative mass of the group and of everything above it:
//   AUROC * P * N = sum_e (1 - t_e) * (TP_strictly_above(e) + t_eq(e) / 2)   (Mann-Whitney)
//   AUPRC * P     = sum_e t_e * TP_ge(e) / (TP_ge(e) + FP_ge(e))              (avg precision)
// so a sample needs the mass above its bucket (a prefix over bucket totals) plus the mass above
// it INSIDE its bucket - never a global order.  On MI355X a global radix sort costs one memory
// round trip per launch (K3a: 4 passes x 2 launches, then the K3 scan); here:
//   1 sample : one block draws S = 4B stratified scores (hash-jittered, deterministic) and
//              bitonic-sorts them with 4 keys per thread - register and DPP/shuffle stages
//              inside a wave, LDS stages only across waves - then writes B-1 splitters.
//   2 hist   : per 16K-sample tile (1024 threads x 16): bin ids (binary search over the LDS
//              splitters; a score EQUAL to splitter j gets its own "equal" bin, so a heavily
//              repeated score needs no within-bin work), LDS counts + FP64 positive mass, then
//              per non-empty bin ONE returning atomic that reserves the tile's run inside the
//              bin (and one FP64 atomic for the bin's positive mass).  Big tiles keep the
//              same-address atomic depth at n / 16K.
//   3 scatter: per tile: bin starts from the complete bin counts, every sample written to
//              start + the tile's reservation + its LDS-atomic rank (order inside a bin does not
//              matter to the sums, except for the special bins below).
//   4 local  : one block per splitter: its "between" bin, then its "equal" bin in closed form.
//              A between bin of <= 4096 samples stays in registers (16 per thread): min / max,
//              1024 sub-bins under the bin's key span, an LDS counting sort by sub-bin and a
//              pair loop inside the sample's sub-bin (~m / 1024 samples).  A sub-bin of more
//              than 64 samples over more than one key is pushed and sub-binned again under its
//              own span (each level removes >= 10 key bits), so adversarial bins cost
//              O(m * levels), never O(m^2); bins above 4096 samples run the same passes from
//              global scratch.  One extra block scans the special bins.  Per-block (U, AP) go to
//              slots; the last block to finish (returning atomic, release / acquire fences) sums
//              them in order, writes AUROC / AUPRC and re-zeroes the counters.
// Special scores follow the reference's `diff != 0` tie rule: NaN, +inf and -inf samples are
// never tied with each other (inf - inf = NaN), so their bins hold singletons in SOURCE order
// (placed by per-tile counts, not atomics) and are scanned in that order.
// All masses accumulate in FP64 (exact for 0 / 1 targets).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kSampleT = 1024;       // sample threads
constexpr int kSP = 4;               // sampled keys per thread (S <= 4096)
constexpr int kHT = 256;             // hist / scatter threads
constexpr int kHPer = 16;            // samples per thread
constexpr int kHW = kHT / kWave;     // 4 waves
constexpr int kTileN = kHT * kHPer;  // 4096: ~one tile per CU at 1M (the per-element LDS work spreads)
constexpr int kMaxB = 1024;
constexpr int kMaxBins = 2 * kMaxB + 2;
constexpr int kBinQ = (kMaxBins + kHT - 1) / kHT;  // bins per hist / scatter thread (9)
constexpr int kLT = 256;             // local threads: 4 waves, one splitter each (B = 1024: 256 blocks, one per CU)
constexpr int kLW = kLT / kWave;
constexpr int kLeaf = 64;            // largest multi-key sub-bin resolved by a pair loop

#ifdef BK_PROBE  // csrc/bench/k3b_probe.hip: per-block wall-clock stamps [kernel][block][8]
__device__ unsigned long long* g_bk_dbg;
#define BK_STAMP(kern, slot)                                                                      \
  if (threadIdx.x == 0) g_bk_dbg[((kern) * 4096 + blockIdx.x) * 8 + (slot)] = wall_clock64()
#define BK_STAMPW(unit, slot)                                                                     \
  if ((threadIdx.x & 63) == 0) g_bk_dbg[(2 * 4096 + (unit)) * 8 + (slot)] = wall_clock64()
#else
#define BK_STAMP(kern, slot)
#define BK_STAMPW(unit, slot)
#endif

constexpr uint32_t kKeyNan = 0x003fffffu, kKeyPinf = 0x007fffffu, kKeyNinf = 0xff800000u;

__device__ __forceinline__ uint32_t bk_key(float f) {  // ascending key = descending score
  uint32_t u = __float_as_uint(f);
  if (f != f) u = 0x7fc00000u;   // canonical NaN (first, as torch.sort)
  if (u == 0x80000000u) u = 0u;  // -0 ties +0
  const uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~asc;
}

__device__ __forceinline__ int bk_special(uint32_t k) {  // 0 NaN, 1 +inf, 2 -inf, -1 finite
  return k == kKeyNan ? 0 : k == kKeyPinf ? 1 : k == kKeyNinf ? 2 : -1;
}

template <typename PT>
__device__ __forceinline__ float bk_target(const void* t, int64_t i) {
  if constexpr (sizeof(PT) == 8) return static_cast<float>(static_cast<const int32_t*>(t)[2 * i]);  // low dword
  else return static_cast<float>(static_cast<const PT*>(t)[i]);
}

// bin of a key: 0 NaN, 1 +inf, nbins - 1 -inf, else 2 + 2 * lower_bound(sp) + (key == sp[lb]).
// R keys at once, step-outer: every step issues R independent LDS reads.
template <int R>
__device__ __forceinline__ void bk_bins(const uint32_t* sp, int B, int nbins, const uint32_t (&k)[R], uint32_t (&bin)[R]) {
  uint32_t idx[R];
#pragma unroll
  for (int r = 0; r < R; ++r) idx[r] = 0u;
  for (int step = B >> 1; step > 0; step >>= 1) {
#pragma unroll
    for (int r = 0; r < R; ++r) idx[r] += sp[idx[r] + step - 1] < k[r] ? static_cast<uint32_t>(step) : 0u;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int c = bk_special(k[r]);
    const uint32_t eq = (static_cast<int>(idx[r]) < B - 1 && sp[idx[r]] == k[r]) ? 1u : 0u;
    bin[r] = c >= 0 ? (c == 2 ? static_cast<uint32_t>(nbins - 1) : static_cast<uint32_t>(c)) : 2u + 2u * idx[r] + eq;
  }
}

template <typename T>
__device__ __forceinline__ T block_sum_all(T v, T* lds /* >= NT / 64 */) {  // total in every thread
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  if (lane_id() == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  T s = T(0);
  for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) s += lds[w];
  __syncthreads();
  return s;
}

// exclusive scan over the block of one value per thread; total returned through `tot`
template <typename T>
__device__ __forceinline__ T block_excl(T v, T* lds, T& tot) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  T inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const T y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  if (lane == kWave - 1) lds[w] = inc;
  __syncthreads();
  T pre = T(0), t = T(0);
  for (int q = 0; q < static_cast<int>(blockDim.x >> 6); ++q) {
    if (q < w) pre += lds[q];
    t += lds[q];
  }
  __syncthreads();
  tot = t;
  return pre + inc - v;
}

// in-place exclusive scan of len u32 in LDS (len <= kPer * blockDim)
template <int kPer>
__device__ __forceinline__ void lds_excl_scan(uint32_t* v, int len, uint32_t* lds) {
  const int j0 = threadIdx.x * kPer;
  uint32_t x[kPer], s = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    x[q] = j0 + q < len ? v[j0 + q] : 0u;
    s += x[q];
  }
  uint32_t tot;
  uint32_t run = block_excl<uint32_t>(s, lds, tot);
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (j0 + q < len) {
      v[j0 + q] = run;
      run += x[q];
    }
  __syncthreads();
}

// B <= 2 * kHT splitters into LDS, both loads in flight together
__device__ __forceinline__ void load_splitters(const BucketAucArgs& a, uint32_t* sp) {
  uint32_t v[kMaxB / kHT];
#pragma unroll
  for (int q = 0; q < kMaxB / kHT; ++q) {
    const int j = q * kHT + static_cast<int>(threadIdx.x);
    v[q] = j < a.B ? a.sp[j] : 0u;
  }
#pragma unroll
  for (int q = 0; q < kMaxB / kHT; ++q) {
    const int j = q * kHT + static_cast<int>(threadIdx.x);
    if (j < a.B) sp[j] = v[q];
  }
}

// ---------------------------------------------------------------- 1: splitters
__global__ __launch_bounds__(kSampleT) void bk_sample_kernel(BucketAucArgs a) {
  __shared__ uint32_t s[kSP * kSampleT];
  BK_STAMP(3, 0);
  const int S = a.S, T = S / kSP, tid = threadIdx.x;
  const int64_t q = a.n / S;  // stratum length (>= 4)
  uint32_t v[kSP];
  float xv[kSP];
#pragma unroll
  for (int p = 0; p < kSP; ++p) {  // every load issued before any is used (no branch between)
    const int e = tid < T ? tid * kSP + p : 0;
    uint32_t h = static_cast<uint32_t>(e) * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    xv[p] = a.x[static_cast<int64_t>(e) * q + static_cast<int64_t>(h % static_cast<uint32_t>(q))];
  }
#pragma unroll
  for (int p = 0; p < kSP; ++p) v[p] = tid < T ? bk_key(xv[p]) : 0xffffffffu;
  BK_STAMP(3, 1);
  // bitonic network over e = kSP * tid + p (ascending): j >= kSP * 64 across waves in LDS,
  // kSP <= j < kSP * 64 across lanes of a wave (shuffles), j < kSP inside the thread
  for (int k = 2; k <= S; k <<= 1) {
    int j = k >> 1;
    if (j >= kSP * kWave) {
      if (tid < T) {
#pragma unroll
        for (int p = 0; p < kSP; ++p) s[tid * kSP + p] = v[p];
      }
      __syncthreads();
      for (; j >= kSP * kWave; j >>= 1) {
        for (int i = tid; i < S / 2; i += kSampleT) {
          const int lo = 2 * i - (i & (j - 1)), hi = lo + j;
          const uint32_t x = s[lo], y = s[hi];
          if ((x > y) == ((lo & k) == 0)) {
            s[lo] = y;
            s[hi] = x;
          }
        }
        __syncthreads();
      }
      if (tid < T) {
#pragma unroll
        for (int p = 0; p < kSP; ++p) v[p] = s[tid * kSP + p];
      }
      __syncthreads();  // the next LDS stage writes s again
    }
    for (; j >= kSP; j >>= 1) {
      const int m = j / kSP;
      const bool lower = (tid & m) == 0, up = ((tid * kSP) & k) == 0;  // same for every p
#pragma unroll
      for (int p = 0; p < kSP; ++p) {
        const uint32_t o = __shfl_xor(v[p], m, kWave);
        v[p] = (lower == up) ? (o < v[p] ? o : v[p]) : (o > v[p] ? o : v[p]);
      }
    }
#pragma unroll
    for (int jj = kSP / 2; jj >= 1; jj >>= 1) {  // static register indices; j is now < kSP
      if (jj > j) continue;
#pragma unroll
      for (int p = 0; p < kSP; ++p) {
        if (p & jj) continue;
        const int pq = p | jj;
        const bool up = ((tid * kSP + p) & k) == 0;
        const uint32_t x = v[p], y = v[pq];
        const bool sw = (x > y) == up;
        v[p] = sw ? y : x;
        v[pq] = sw ? x : y;
      }
    }
  }
  BK_STAMP(3, 2);
  // splitter j = sorted[4 (j + 1)] (S / B = 4) = element 0 of thread j + 1
  if (tid >= 1 && tid < a.B) a.sp[tid - 1] = v[0];
  if (tid == 0) a.sp[a.B - 1] = 0xffffffffu;
  BK_STAMP(3, 3);
}

// ---------------------------------------------------------------- 2: counts + reservations
template <typename PT>
__global__ __launch_bounds__(kHT) void bk_hist_kernel(BucketAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* tsum = reinterpret_cast<double*>(smem);               // [nbins]
  uint32_t* cnt = reinterpret_cast<uint32_t*>(tsum + a.nbins);  // [nbins]
  uint32_t* sp = cnt + a.nbins;                                 // [B]
  BK_STAMP(0, 0);
  const int tile = blockIdx.x;
  for (int j = threadIdx.x; j < a.nbins; j += kHT) {
    cnt[j] = 0u;
    tsum[j] = 0.0;
  }
  load_splitters(a, sp);
  const int64_t t0 = static_cast<int64_t>(tile) * kTileN + threadIdx.x;
  float xs[kHPer], ts[kHPer];
#pragma unroll
  for (int r = 0; r < kHPer; ++r) {
    const int64_t i = t0 + r * kHT;
    const int64_t ic = i < a.n ? i : a.n - 1;
    xs[r] = a.x[ic];
    ts[r] = bk_target<PT>(a.t, ic);
  }
  __syncthreads();
  BK_STAMP(0, 1);
  {
    uint32_t kk[kHPer], bin[kHPer];
#pragma unroll
    for (int r = 0; r < kHPer; ++r) kk[r] = bk_key(xs[r]);
    bk_bins<kHPer>(sp, a.B, a.nbins, kk, bin);
    BK_STAMP(0, 4);
    // in-tile rank from the returning LDS atomic; (bin, rank) saves the scatter pass the search
#pragma unroll
    for (int r = 0; r < kHPer; ++r) {
      if (t0 + r * kHT < a.n) {
        const uint32_t rk = atomicAdd(&cnt[bin[r]], 1u);
        if (ts[r] != 0.f) atomicAdd(&tsum[bin[r]], static_cast<double>(ts[r]));
        a.binrank[t0 + r * kHT] = (bin[r] << 12) | rk;
      }
    }
  }
  __syncthreads();
  BK_STAMP(0, 2);
  // special-bin counts of this tile (their samples are placed in source order by prefix sums)
  if (threadIdx.x < 3) a.spc[3 * tile + threadIdx.x] = cnt[threadIdx.x == 2 ? a.nbins - 1 : threadIdx.x];
  // reserve this tile's run in every non-empty bin: all returning atomics in flight together
  uint32_t* row = a.tileoff + static_cast<int64_t>(tile) * a.nbins;
  uint32_t got[kBinQ];
#pragma unroll
  for (int q = 0; q < kBinQ; ++q) {
    const int j = q * kHT + static_cast<int>(threadIdx.x);
    const uint32_t c = j < a.nbins ? cnt[j] : 0u;
    got[q] = c ? atomicAdd(&a.cursor[j], c) : 0u;
    if (j < a.nbins && tsum[j] != 0.0) atomicAdd(&a.posmass[j], tsum[j]);
  }
#pragma unroll
  for (int q = 0; q < kBinQ; ++q) {
    const int j = q * kHT + static_cast<int>(threadIdx.x);
    if (j < a.nbins && cnt[j]) row[j] = got[q];
  }
  BK_STAMP(0, 3);
}

// ---------------------------------------------------------------- 3: scatter into bins
template <typename PT>
__global__ __launch_bounds__(kHT) void bk_scatter_kernel(BucketAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* start = reinterpret_cast<uint32_t*>(smem);  // [nbins] bin starts
  __shared__ uint32_t sord[3][kHPer * kHW];              // special samples per (class, round, wave)
  __shared__ uint32_t sprev[3];                          // special samples of earlier tiles
  __shared__ uint32_t red[kHW];
  BK_STAMP(1, 0);
  const int tile = blockIdx.x, tid = threadIdx.x;
  const int64_t t0 = static_cast<int64_t>(tile) * kTileN + tid;
  const uint32_t* row = a.tileoff + static_cast<int64_t>(tile) * a.nbins;
  const uint32_t last_bin = static_cast<uint32_t>(a.nbins - 1);
  // every global load of the pass in flight together: counts, (bin, rank), scores, targets,
  // then the tile's reservations (dependent on the bins only)
  uint32_t cv[kBinQ];
#pragma unroll
  for (int q = 0; q < kBinQ; ++q) {
    const int j = q * kHT + tid;
    cv[q] = j < a.nbins ? a.cursor[j] : 0u;
  }
  float xs[kHPer], ts[kHPer];
  uint32_t br[kHPer];
#pragma unroll
  for (int r = 0; r < kHPer; ++r) {
    const int64_t i = t0 + r * kHT;
    const int64_t ic = i < a.n ? i : a.n - 1;
    br[r] = a.binrank[ic];
    xs[r] = a.x[ic];
    ts[r] = bk_target<PT>(a.t, ic);
  }
  uint32_t c3[3] = {0u, 0u, 0u};  // special samples of the tiles before this one, per class
  for (int u = tid; u < tile; u += kHT) {
    c3[0] += a.spc[3 * u];
    c3[1] += a.spc[3 * u + 1];
    c3[2] += a.spc[3 * u + 2];
  }
  uint32_t off[kHPer];  // the tile's reservation in the sample's bin (regular bins)
#pragma unroll
  for (int r = 0; r < kHPer; ++r) {
    const uint32_t b = br[r] >> 12;
    const bool special = b < 2u || b == last_bin;
    off[r] = (t0 + r * kHT < a.n && !special) ? row[b] + (br[r] & 0xfffu) : 0u;
  }
#pragma unroll
  for (int q = 0; q < kBinQ; ++q) {
    const int j = q * kHT + tid;
    if (j < a.nbins) start[j] = cv[q];
  }
  BK_STAMP(1, 1);
  const int lane = lane_id(), w = tid >> 6;
  const uint64_t below = lane ? (~0ull >> (kWave - lane)) : 0ull;
#pragma unroll
  for (int r = 0; r < kHPer; ++r) {
    const bool valid = t0 + r * kHT < a.n;
    const uint32_t b = br[r] >> 12;
    const int cls = !valid ? -1 : b == 0u ? 0 : b == 1u ? 1 : b == last_bin ? 2 : -1;
    const uint64_t m0 = __ballot(cls == 0), m1 = __ballot(cls == 1), m2 = __ballot(cls == 2);
    if (lane == 0) {
      sord[0][r * kHW + w] = static_cast<uint32_t>(__popcll(m0));
      sord[1][r * kHW + w] = static_cast<uint32_t>(__popcll(m1));
      sord[2][r * kHW + w] = static_cast<uint32_t>(__popcll(m2));
    }
    const uint64_t mm = cls == 0 ? m0 : cls == 1 ? m1 : m2;
    if (cls >= 0) off[r] = static_cast<uint32_t>(__popcll(mm & below));  // rank among the wave's specials
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const uint32_t sum = block_sum_all<uint32_t>(c3[q], red);  // syncs: sord and start complete after this
    if (tid == 0) sprev[q] = sum;
  }
  {  // exclusive prefix over (round, wave) cells per class: source order inside the tile
    const int cell = tid & (kHPer * kHW - 1);
    uint32_t v3[3], tot;
#pragma unroll
    for (int q = 0; q < 3; ++q) v3[q] = tid < kHPer * kHW ? sord[q][cell] : 0u;
    uint32_t e3[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) e3[q] = block_excl<uint32_t>(v3[q], red, tot);
    if (tid < kHPer * kHW) {
#pragma unroll
      for (int q = 0; q < 3; ++q) sord[q][cell] = e3[q];
    }
  }
  lds_excl_scan<kBinQ>(start, a.nbins, red);  // ends with a barrier: sord and start are final
  BK_STAMP(1, 2);
#pragma unroll
  for (int r = 0; r < kHPer; ++r) {
    if (t0 + r * kHT >= a.n) continue;
    const uint32_t b = br[r] >> 12;
    uint32_t pos = start[b] + off[r], key;
    if (b < 2u || b == last_bin) {  // special: source order; the key slot carries the source index
      const int cls = b == last_bin ? 2 : static_cast<int>(b);
      pos += sprev[cls] + sord[cls][r * kHW + w];
      key = static_cast<uint32_t>(t0 + r * kHT);
    } else {
      key = bk_key(xs[r]);
    }
#ifdef BK_PROBE_LINEAR  // timing experiment only: coalesced stores to the wrong place
    pos = static_cast<uint32_t>(t0 + r * kHT);
#endif
    a.keys_out[pos] = key;
    a.t_out[pos] = ts[r];
  }
  BK_STAMP(1, 3);
}

// ---------------------------------------------------------------- 4: per-bin terms + fold
// One WAVE per splitter (its between bin, then its equal bin in closed form): no block barriers
// anywhere in the pass.  A range of <= kWCap samples is held in registers (32 per lane), sorted
// by 512 sub-bins under its own key span into wave-private LDS, and resolved by pair loops
// inside a sub-bin (~m / 256 samples); a multi-key sub-bin of more than kLeaf samples is pushed
// and sub-binned again (each level removes >= 8 key bits).  Ranges above kWCap run chunked
// passes over global memory (ping-pong with keys_tmp) with leaves staged through LDS.
constexpr int kWCap = 4096;              // range samples in registers (64 per lane): ~4x the mean bin
constexpr int kWPer = kWCap / kWave;
constexpr int kWSub = 256;               // sub-bins per pass (4 per lane)
constexpr int kWSubBits = 8;
constexpr int kWSPer = kWSub / kWave;
constexpr int kWStack = kWCap / kLeaf + 8;

// A pending range of a between bin: [s, s + c) of the bin's slice of keys_out / t_out, s = the
// samples above it inside the bin (ranges are laid out in key order), tpa = their positive mass.
struct BkItem {
  uint32_t s, c;
  double tpa;
};

struct alignas(16) WaveLds {
  uint32_t k[kWCap];
  float t[kWCap];
  double m[kWSub + 2];    // exclusive positive mass per sub-bin (m[kWSub] = range mass)
  uint32_t c[kWSub];      // counts, then cursors
  uint32_t o[kWSub + 4];  // exclusive offsets (o[kWSub] = range size)
  BkItem stack[kWStack];
};

struct Acc {
  double u = 0.0, ap = 0.0;
};

// LDS writes of this wave are visible to its other lanes after this (DS ops retire in order)
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <typename T>
__device__ __forceinline__ T w_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
  return v;
}

template <typename T>
__device__ __forceinline__ T w_excl(T v, T& tot) {  // exclusive scan over the wave's lanes
  const int lane = lane_id();
  T inc = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const T y = __shfl_up(inc, o, kWave);
    if (lane >= o) inc += y;
  }
  tot = __shfl(inc, kWave - 1, kWave);
  return inc - v;
}

__device__ __forceinline__ void w_minmax(uint32_t& kmin, uint32_t& kmax) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = __shfl_xor(kmin, o, kWave), y = __shfl_xor(kmax, o, kWave);
    kmin = x < kmin ? x : kmin;
    kmax = y > kmax ? y : kmax;
  }
}

__device__ __forceinline__ int w_shift(uint32_t span) {
  const int sbits = span ? 32 - __builtin_clz(span) : 0;
  return sbits > kWSubBits ? sbits - kWSubBits : 0;
}

__device__ __forceinline__ void w_zero(WaveLds& W) {
  const int lane = lane_id();
#pragma unroll
  for (int i = 0; i < kWSPer; ++i) {
    W.c[lane * kWSPer + i] = 0u;
    W.m[lane * kWSPer + i] = 0.0;
  }
  wsync();
}

// counts / masses in W.c / W.m -> exclusive offsets, cursors, and the pushed (oversized,
// multi-key) sub-bins appended to the stack; returns the new stack top
__device__ __forceinline__ int w_scan_push(WaveLds& W, BkItem* stack, int top, int shift, uint32_t s, double tpa) {
  const int lane = lane_id(), s0 = lane * kWSPer;
  uint32_t c[kWSPer], csum = 0, np = 0;
  double m[kWSPer], msum = 0.0;
#pragma unroll
  for (int i = 0; i < kWSPer; ++i) {
    c[i] = W.c[s0 + i];
    m[i] = W.m[s0 + i];
    csum += c[i];
    msum += m[i];
    np += (c[i] > static_cast<uint32_t>(kLeaf) && shift > 0) ? 1u : 0u;
  }
  uint32_t ctot, ptot;
  double mtot;
  uint32_t cex = w_excl<uint32_t>(csum, ctot);
  double mex = w_excl<double>(msum, mtot);
  uint32_t pidx = w_excl<uint32_t>(np, ptot);
#pragma unroll
  for (int i = 0; i < kWSPer; ++i) {
    W.o[s0 + i] = cex;
    W.c[s0 + i] = cex;  // cursor
    W.m[s0 + i] = mex;
    if (c[i] > static_cast<uint32_t>(kLeaf) && shift > 0) stack[top + static_cast<int>(pidx++)] = {s + cex, c[i], tpa + mex};
    cex += c[i];
    mex += m[i];
  }
  if (lane == kWave - 1) {
    W.o[kWSub] = cex;
    W.m[kWSub] = mex;
  }
  wsync();
  return top + static_cast<int>(ptot);
}

__device__ __forceinline__ bool w_pushed(const WaveLds& W, uint32_t sub, int shift) {
  return shift > 0 && W.o[sub + 1] - W.o[sub] > static_cast<uint32_t>(kLeaf);
}

// (U, AP) terms of one sample in sub-bin `sub` of a range sorted by sub-bin; the sub-bin's
// samples are W.k / W.t [j - base] for j in [o[sub], o[sub + 1])
__device__ __forceinline__ void w_leaf(Acc& acc, uint32_t k, float t, uint32_t sub, int shift, const WaveLds& W,
                                       uint32_t base, double tpr, double cab, double tpa_in, double FPa) {
  const uint32_t j0 = W.o[sub], j1 = W.o[sub + 1];
  const uint32_t sc = j1 - j0;
  if (sc > static_cast<uint32_t>(kLeaf) && shift > 0) return;  // a pushed range covers it
  const double p0 = W.m[sub];
  double lt_t = 0.0, eq_t;
  int lt_c = 0, eq_c;
  if (shift == 0) {  // one key per sub-bin
    eq_t = W.m[sub + 1] - p0;
    eq_c = static_cast<int>(sc);
  } else {
    float lt = 0.f, eq = 0.f;
    int ec = 0;
    for (uint32_t j = j0 - base; j < j1 - base; ++j) {
      const uint32_t kj = W.k[j];
      const float tj = W.t[j];
      lt += kj < k ? tj : 0.f;
      lt_c += kj < k;
      eq += kj == k ? tj : 0.f;
      ec += kj == k;
    }
    lt_t = lt;
    eq_t = eq;
    eq_c = ec;
  }
  const double tp_in = p0 + lt_t;                                                 // above, inside the range
  const double c_in = cab + static_cast<double>(j0) + static_cast<double>(lt_c);  // above, inside the bin
  const double tp_strict = tpr + tp_in;
  const double tp_ge = tp_strict + eq_t;
  const double fp_ge = FPa + (c_in - (tpa_in + tp_in)) + (static_cast<double>(eq_c) - eq_t);
  acc.u += (1.0 - static_cast<double>(t)) * (tp_strict + 0.5 * eq_t);
  if (t != 0.f) acc.ap += static_cast<double>(t) * tp_ge / (tp_ge + fp_ge);
}

// a range of c <= kWCap samples of the bin slice (k0, t0): registers -> LDS counting sort by
// sub-bin -> pair loops; pushed sub-bins go back to the range's (consumed) global slice
__device__ __forceinline__ int w_range_regs(Acc& acc, uint32_t* k0, float* t0, const BkItem& it, double TPa,
                                            double FPa, WaveLds& W, BkItem* stack, int top) {
  const int lane = lane_id(), c = static_cast<int>(it.c);
  const uint32_t* gk = k0 + it.s;
  const float* gt = t0 + it.s;
  uint32_t kr[kWPer];
  float tr[kWPer];
#pragma unroll
  for (int q = 0; q < kWPer; ++q) {
    const int i = q * kWave + lane;
    const int ic = i < c ? i : c - 1;
    kr[q] = gk[ic];
    tr[q] = gt[ic];
  }
  uint32_t kmin = 0xffffffffu, kmax = 0u;
#pragma unroll
  for (int q = 0; q < kWPer; ++q) {  // clamped duplicates leave min / max unchanged
    kmin = kr[q] < kmin ? kr[q] : kmin;
    kmax = kr[q] > kmax ? kr[q] : kmax;
  }
  w_minmax(kmin, kmax);
  BK_STAMPW(blockIdx.x * kLW + (threadIdx.x >> 6), 4);
  const uint32_t lo = kmin;
  const int shift = w_shift(kmax - kmin);
  w_zero(W);
#pragma unroll
  for (int q = 0; q < kWPer; ++q) {
    if (q * kWave + lane < c) {
      const uint32_t sub = (kr[q] - lo) >> shift;
      atomicAdd(&W.c[sub], 1u);
      if (tr[q] != 0.f) atomicAdd(&W.m[sub], static_cast<double>(tr[q]));
    }
  }
  wsync();
  BK_STAMPW(blockIdx.x * kLW + (threadIdx.x >> 6), 5);
  const int ntop = w_scan_push(W, stack, top, shift, it.s, it.tpa);
  BK_STAMPW(blockIdx.x * kLW + (threadIdx.x >> 6), 6);
#pragma unroll
  for (int q = 0; q < kWPer; ++q) {
    if (q * kWave + lane < c) {
      const uint32_t r = atomicAdd(&W.c[(kr[q] - lo) >> shift], 1u);
      W.k[r] = kr[q];
      W.t[r] = tr[q];
    }
  }
  wsync();
  BK_STAMPW(blockIdx.x * kLW + (threadIdx.x >> 6), 7);
  const double tpr = TPa + it.tpa, cab = static_cast<double>(it.s);
  uint32_t* wk = k0 + it.s;
  float* wt = t0 + it.s;
  const bool pushed_any = ntop > top;
  if (pushed_any) {
    for (int i = lane; i < c; i += kWave) {  // pushed ranges were consumed: their items live there again
      const uint32_t k = W.k[i];
      if (w_pushed(W, (k - lo) >> shift, shift)) {
        wk[i] = k;
        wt[i] = W.t[i];
      }
    }
  }
  // 4 samples per lane in flight: the per-sample chains (sub-bin bounds, pair loop, division)
  // overlap instead of running back to back
  for (int i0 = 0; i0 < c; i0 += 4 * kWave) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * kWave + lane;
      if (i < c) {
        const uint32_t k = W.k[i];
        w_leaf(acc, k, W.t[i], (k - lo) >> shift, shift, W, 0u, tpr, cab, it.tpa, FPa);
      }
    }
  }
  return ntop;
}

// largest sub-bin whose offset is <= p (p < range size): the non-empty sub-bin holding p
__device__ __forceinline__ uint32_t w_sub_at(const WaveLds& W, uint32_t p) {
  uint32_t idx = 0;
#pragma unroll
  for (int step = kWSub >> 1; step > 0; step >>= 1) idx += W.o[idx + step] <= p ? static_cast<uint32_t>(step) : 0u;
  return idx;
}

// a range of c > kWCap samples: chunked passes over global memory (scatter through k1 and back),
// then leaf sub-bins staged through LDS in chunks cut at sub-bin starts
__device__ __forceinline__ int w_range_big(Acc& acc, uint32_t* k0, float* t0, uint32_t* k1, float* t1, BkItem it,
                                        double TPa, double FPa, WaveLds& W, BkItem* stack, int top) {
  const int lane = lane_id(), c = static_cast<int>(it.c);
  constexpr int U8 = 8;
  uint32_t* gk = k0 + it.s;
  float* gt = t0 + it.s;
  uint32_t* dk = k1 + it.s;
  float* dt = t1 + it.s;
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  for (int c0 = 0; c0 < c; c0 += kWave * U8) {
    uint32_t kk[U8];
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      const int i = c0 + q * kWave + lane;
      kk[q] = gk[i < c ? i : c - 1];
    }
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      kmin = kk[q] < kmin ? kk[q] : kmin;
      kmax = kk[q] > kmax ? kk[q] : kmax;
    }
  }
  w_minmax(kmin, kmax);
  const uint32_t lo = kmin;
  const int shift = w_shift(kmax - kmin);
  w_zero(W);
  for (int c0 = 0; c0 < c; c0 += kWave * U8) {
    uint32_t kk[U8];
    float tt[U8];
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      const int i = c0 + q * kWave + lane;
      const int ic = i < c ? i : c - 1;
      kk[q] = gk[ic];
      tt[q] = gt[ic];
    }
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      if (c0 + q * kWave + lane < c) {
        const uint32_t sub = (kk[q] - lo) >> shift;
        atomicAdd(&W.c[sub], 1u);
        if (tt[q] != 0.f) atomicAdd(&W.m[sub], static_cast<double>(tt[q]));
      }
    }
  }
  wsync();
  const int ntop = w_scan_push(W, stack, top, shift, it.s, it.tpa);
  for (int c0 = 0; c0 < c; c0 += kWave * U8) {
    uint32_t kk[U8];
    float tt[U8];
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      const int i = c0 + q * kWave + lane;
      const int ic = i < c ? i : c - 1;
      kk[q] = gk[ic];
      tt[q] = gt[ic];
    }
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      if (c0 + q * kWave + lane < c) {
        const uint32_t r = atomicAdd(&W.c[(kk[q] - lo) >> shift], 1u);
        dk[r] = kk[q];
        dt[r] = tt[q];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (int c0 = 0; c0 < c; c0 += kWave * U8) {  // back into the range's slice: pushed items live there
    uint32_t kk[U8];
    float tt[U8];
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      const int i = c0 + q * kWave + lane;
      const int ic = i < c ? i : c - 1;
      kk[q] = dk[ic];
      tt[q] = dt[ic];
    }
#pragma unroll
    for (int q = 0; q < U8; ++q) {
      const int i = c0 + q * kWave + lane;
      if (i < c) {
        gk[i] = kk[q];
        gt[i] = tt[q];
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  const double tpr = TPa + it.tpa, cab = static_cast<double>(it.s);
  if (shift == 0) {  // one key per sub-bin: closed forms, no pair loops
    for (int i = lane; i < c; i += kWave) {
      const uint32_t k = gk[i];
      w_leaf(acc, k, gt[i], k - lo, 0, W, 0u, tpr, cab, it.tpa, FPa);
    }
    return ntop;
  }
  uint32_t c0 = 0;
  const uint32_t cu = static_cast<uint32_t>(c);
  while (c0 < cu) {  // uniform: every lane walks the same chunk boundaries
    const uint32_t sb0 = w_sub_at(W, c0);
    if (w_pushed(W, sb0, shift)) {
      c0 = W.o[sb0 + 1];
      continue;
    }
    uint32_t c1 = cu;
    if (c0 + kWCap < cu) c1 = W.o[w_sub_at(W, c0 + kWCap)];  // > c0: the sub-bin at c0 has <= kLeaf samples
    const int len = static_cast<int>(c1 - c0);
    for (int i = lane; i < len; i += kWave) {
      W.k[i] = gk[c0 + i];
      W.t[i] = gt[c0 + i];
    }
    wsync();
    for (int i = lane; i < len; i += kWave) {
      const uint32_t k = W.k[i];
      w_leaf(acc, k, W.t[i], (k - lo) >> shift, shift, W, c0, tpr, cab, it.tpa, FPa);
    }
    wsync();
    c0 = c1;
  }
  return ntop;
}

// special bin: singleton groups in source order, one wave scan of (t, 1 - t) per 64 samples
__device__ __forceinline__ void w_special_bin(Acc& acc, const float* gt, int m, double TPa, double FPa) {
  const int lane = lane_id();
  double run_t = 0.0, run_n = 0.0;
  for (int c0 = 0; c0 < m; c0 += kWave) {
    const int i = c0 + lane;
    const double t = i < m ? static_cast<double>(gt[i]) : 0.0;
    const double nn = i < m ? 1.0 - t : 0.0;
    double tt, tn;
    const double et = w_excl<double>(t, tt);
    const double en = w_excl<double>(nn, tn);
    if (i < m) {
      const double tpb = TPa + run_t + et, fpb = FPa + run_n + en;
      acc.u += nn * (tpb + 0.5 * t);
      if (t != 0.0) acc.ap += t * (tpb + t) / (tpb + t + fpb + nn);
    }
    run_t += tt;
    run_n += tn;
  }
}

// (count, positive mass) of bins [0, upto), all loads in flight together
__device__ __forceinline__ void w_prefix(const BucketAucArgs& a, int upto, uint32_t& cnt, double& pm) {
  constexpr int kQ = (kMaxBins + kWave - 1) / kWave;
  double p[kQ];
  uint32_t c[kQ];
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    const int j = q * kWave + lane_id();
    const bool ok = j < upto;
    p[q] = ok ? a.posmass[j] : 0.0;
    c[q] = ok ? a.cursor[j] : 0u;
  }
  double ps = 0.0;
  uint32_t cs = 0;
#pragma unroll
  for (int q = 0; q < kQ; ++q) {
    ps += p[q];
    cs += c[q];
  }
  pm = w_sum<double>(ps);
  cnt = w_sum<uint32_t>(cs);
}

__global__ __launch_bounds__(kLT) void bk_local_kernel(BucketAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int unit = blockIdx.x * kLW + w;  // splitter index; unit 0 also scans the special bins
  const int nunits = a.B;
  if (unit >= nunits) return;
  BK_STAMPW(unit, 0);
  WaveLds& W = reinterpret_cast<WaveLds*>(smem)[w];
  Acc acc;
  {
    const int bb = 2 + 2 * unit;  // between bin; bb + 1 its equal bin (none for the last splitter)
    uint32_t start;
    double TPa;
    w_prefix(a, bb, start, TPa);
    const double FPa = static_cast<double>(start) - TPa;
    const int m = static_cast<int>(a.cursor[bb]);
    const double Pb = a.posmass[bb];
    const int me = unit < a.B - 1 ? static_cast<int>(a.cursor[bb + 1]) : 0;
    const double Pe = unit < a.B - 1 ? a.posmass[bb + 1] : 0.0;
    BK_STAMPW(unit, 1);
    if (m > 0) {
      uint32_t* k0 = a.keys_out + start;
      float* t0 = a.t_out + start;
      // ranges above kWCap keep their pending ranges in global scratch (disjoint per unit)
      BkItem* stack = m > kWCap ? static_cast<BkItem*>(a.stack) + start / kLeaf + 2 * unit : W.stack;
      int top;
      if (m <= kWCap) {
        top = w_range_regs(acc, k0, t0, BkItem{0u, static_cast<uint32_t>(m), 0.0}, TPa, FPa, W, stack, 0);
      } else {
        top = w_range_big(acc, k0, t0, a.keys_tmp + start, a.t_tmp + start, BkItem{0u, static_cast<uint32_t>(m), 0.0},
                          TPa, FPa, W, stack, 0);
      }
      while (top > 0) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        wsync();
        const BkItem it = stack[top - 1];
        --top;
        if (it.c <= static_cast<uint32_t>(kWCap)) top = w_range_regs(acc, k0, t0, it, TPa, FPa, W, stack, top);
        else top = w_range_big(acc, k0, t0, a.keys_tmp + start, a.t_tmp + start, it, TPa, FPa, W, stack, top);
      }
    }
    if (me > 0 && lane == 0) {  // equal bin: one tie group right below the between bin
      const double TPe = TPa + Pb, FPe = FPa + (static_cast<double>(m) - Pb);
      const double Ne = static_cast<double>(me) - Pe;
      acc.u += Ne * (TPe + 0.5 * Pe);
      if (Pe != 0.0) acc.ap += Pe * (TPe + Pe) / (TPe + Pe + FPe + Ne);
    }
  }
  if (unit == 0) {  // special bins: NaN (0), +inf (1), -inf (nbins - 1)
    uint32_t start_last;
    double tp_last;
    w_prefix(a, a.nbins - 1, start_last, tp_last);
    const uint32_t m0 = a.cursor[0], m1 = a.cursor[1], m2 = a.cursor[a.nbins - 1];
    const double p0 = a.posmass[0];
    BK_STAMPW(unit, 1);
    if (m0) w_special_bin(acc, a.t_out, static_cast<int>(m0), 0.0, 0.0);
    if (m1) w_special_bin(acc, a.t_out + m0, static_cast<int>(m1), p0, static_cast<double>(m0) - p0);
    if (m2)
      w_special_bin(acc, a.t_out + start_last, static_cast<int>(m2), tp_last, static_cast<double>(start_last) - tp_last);
  }
  BK_STAMPW(unit, 2);
  const double u = w_sum<double>(acc.u);
  const double ap = w_sum<double>(acc.ap);
  bool last = false;
  if (lane == 0) {
    a.slots[2 * unit] = u;
    a.slots[2 * unit + 1] = ap;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned prev = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == static_cast<unsigned>(nunits - 1);
  }
  last = __shfl(last ? 1 : 0, 0, kWave) != 0;
  BK_STAMPW(unit, 3);
  if (!last) return;
  // the last wave: every slot is published; fold them in unit order
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  double su = 0.0, sa = 0.0, sp = 0.0;
  for (int j = lane; j < nunits; j += kWave) {
    su += __hip_atomic_load(a.slots + 2 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sa += __hip_atomic_load(a.slots + 2 * j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int j = lane; j < a.nbins; j += kWave) sp += __hip_atomic_load(a.posmass + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  su = w_sum<double>(su);
  sa = w_sum<double>(sa);
  sp = w_sum<double>(sp);
  // self-cleaning for the next call (every other wave has finished reading these)
  for (int j = lane; j < a.nbins; j += kWave) {
    a.cursor[j] = 0u;
    a.posmass[j] = 0.0;
  }
  if (lane == 0) {
    *a.done = 0u;
    const double P = sp, N = static_cast<double>(a.n) - sp;
    if (a.out_roc) a.out_roc[0] = (P * N == 0.0) ? 0.5 : su / (P * N);
    if (a.out_pr) a.out_pr[0] = P == 0.0 ? 0.0 : sa / P;
  }
}

constexpr size_t kLdsLocal = sizeof(WaveLds) * kLW;
static_assert(kLdsLocal <= 160 * 1024, "local pass LDS");
static_assert(kTileN <= 4096 && kMaxBins < 4096, "(bin, rank) packs into 12 + 12 bits");
static_assert(kMaxBins * 12 + kMaxB * 4 <= 65536, "hist / scatter LDS at B = kMaxB");
static_assert(kWSub == kWave * kWSPer && kWCap == kWave * kWPer, "local tiling");
static_assert(sizeof(BkItem) == 16, "stack item");

template <typename PT>
int launch_typed(const BucketAucArgs& a, hipStream_t stream, unsigned tiles, size_t lds_hist, size_t lds_scat) {
  hipLaunchKernelGGL(bk_hist_kernel<PT>, dim3(tiles), dim3(kHT), lds_hist, stream, a);
  hipLaunchKernelGGL(bk_scatter_kernel<PT>, dim3(tiles), dim3(kHT), lds_scat, stream, a);
  hipLaunchKernelGGL(bk_local_kernel, dim3(static_cast<unsigned>((a.B + kLW - 1) / kLW)), dim3(kLT), kLdsLocal,
                     stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace

int bucket_auc_buckets(int64_t n) {  // mean bin ~1024 samples: kCap is 4x the mean
  int64_t b = 16;
  while (b < kMaxB && b * 1024 < n) b *= 2;
  return static_cast<int>(b);
}

bool bucket_auc_supported(int64_t n) { return n >= (int64_t{1} << 15) && n <= (int64_t{1} << 21); }

int64_t bucket_auc_tiles(int64_t n) { return (n + kTileN - 1) / kTileN; }

int64_t bucket_auc_stack_items(int64_t n) { return n / kLeaf + 2 * kMaxB + 4; }

int launch_bucket_auc(const BucketAucArgs& a, hipStream_t stream) {
  if (!bucket_auc_supported(a.n) || a.B != bucket_auc_buckets(a.n) || a.S != 4 * a.B || a.nbins != 2 * a.B + 2 ||
      a.S > kSP * kSampleT || a.binrank == nullptr || a.spc == nullptr || a.tileoff == nullptr || a.done == nullptr || a.stack == nullptr)
    return -2;
  const unsigned tiles = static_cast<unsigned>(bucket_auc_tiles(a.n));
  const size_t lds_hist = static_cast<size_t>(a.nbins) * 12 + static_cast<size_t>(a.B) * 4;
  const size_t lds_scat = static_cast<size_t>(a.nbins) * 4;
  static const bool lds_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&bk_local_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 static_cast<int>(kLdsLocal)) == hipSuccess;
  if (!lds_ok) return -3;
  hipLaunchKernelGGL(bk_sample_kernel, dim3(1), dim3(kSampleT), 0, stream, a);
  switch (a.t_dt) {
    case DType::f32: return launch_typed<float>(a, stream, tiles, lds_hist, lds_scat);
    case DType::i64: return launch_typed<int64_t>(a, stream, tiles, lds_hist, lds_scat);
    case DType::i32: return launch_typed<int32_t>(a, stream, tiles, lds_hist, lds_scat);
    case DType::u8:
    case DType::b8: return launch_typed<uint8_t>(a, stream, tiles, lds_hist, lds_scat);
    default: return -2;
  }
}

}  // namespace tea
