// K3s: sample-sort binary AUROC (one row, 32K..2M samples, unweighted).
//
// The K3a + K3 pipeline sorts the whole row with 4 radix passes (an upsweep and a downsweep
// launch each: ~72 us at 1M) and then runs the tie-aware scan (~27 us).  AUROC needs the
// sorted order only INSIDE groups of nearby scores: with the row cut into value buckets,
//   roc = sum_b [ W_b + N_b * TP_above_b ]
// where TP_above_b is the positive mass of all higher-score buckets, N_b the negative mass of
// bucket b, and W_b the Mann-Whitney term of b's own samples (tie groups never straddle a
// bucket, since a sample's bucket is a function of its score).  Five launches:
//   1. ss_sample : one block draws a stratified sample (4 per bucket), radix-sorts it in LDS
//                  and writes B-1 splitters.  Bucket ids: 2*lb for scores strictly between
//                  splitters lb-1 and lb, 2*lb+1 for scores EQUAL to splitter lb - so a
//                  heavily repeated score lands in an "equal" bucket that needs no sort;
//   2. ss_hist   : per 4096-sample tile, bucket ids by an interleaved branch-free binary
//                  search over the LDS splitters, LDS histogram, one global atomic per bin;
//   3. ss_scatter: per tile, LDS-atomic ranks, one global cursor atomic per (tile, bin), the
//                  tile staged in bucket order in LDS and written out in runs;
//   4. ss_local  : one block per bucket: an equal bucket sums its targets; a between bucket
//                  is radix-sorted over only the key bits its splitters leave free (in LDS up
//                  to kSsCap samples, in global scratch beyond), then a chunked tie scan gives
//                  W_b = sum_groups n_g * (TP before the group in b + p_g / 2);
//   5. ss_final  : one block: bucket-order prefix of P_b, roc / (P * N) (0.5 if degenerate),
//                  and the per-bin counters zeroed for the next call (self-cleaning).
// Within a bucket the scatter order is arbitrary; only tie-group tails contribute and their
// prefix sums are order independent (exact for integer targets: FP64 accumulation).
// Status (profiles/rocprof_k3s_samplesort_1m_r2.csv, 1M samples): correct (26 GPU parity tests)
// but slower than K3a + K3 (~97 us): ss_local 136 us, ss_scatter 30, ss_sample 20, ss_hist 17,
// ss_final 6.  Opt-in only (TORCHEVAL_AMD_K3S=1) until the local and scatter kernels are fixed.
// (Measured: buckets of a 1M uniform row are <= 6.2K samples with ~30-sample sub-bins, so the
// local kernel is not an oversized-bucket or sub-bin-skew problem; batching its loads cut it
// from 154 to 136 us only.  SQ counters (profiles/pmc_k3s_samplesort_1m_r2.csv): its 4104 waves
// live ~5.5K cycles each, 22.7M wave-cycles over a 136 us dispatch = ~70 waves resident on
// average, so one long block (or a dispatch limit) sets the time, not the per-bucket work.  The
// hist kernel's LDS binary search takes ~9 bank conflicts per LDS instruction.)
// Reference semantics: torcheval/metrics/functional/classification/auroc.py:115-152.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kSsSampleT = 1024;
constexpr int kSsT = 256;
constexpr int kSsPer = 8;
constexpr int kSsTile = kSsT * kSsPer;
constexpr int kSsL = 256;
constexpr int kSsCap = 8192;

__device__ __forceinline__ uint32_t ss_key(float f) {  // ascending key = descending score
  uint32_t u = __float_as_uint(f);
  if (f != f) u = 0x7fc00000u;  // canonical NaN (first, as torch.sort)
  if (u == 0x80000000u) u = 0u;  // -0 ties +0
  const uint32_t asc = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ~asc;
}

template <typename PT>
__device__ __forceinline__ float ss_target(const void* t, int64_t i) {
  if constexpr (sizeof(PT) == 8) return static_cast<float>(static_cast<const int32_t*>(t)[2 * i]);  // low dword
  else return static_cast<float>(static_cast<const PT*>(t)[i]);
}

__device__ __forceinline__ uint64_t ss_match(uint32_t d, uint64_t active) {
  uint64_t peers = active;
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t ones = __ballot((d >> b) & 1u);
    peers &= ((d >> b) & 1u) ? ones : ~ones;
  }
  return peers;
}

// inclusive block scan (NT threads); `total` = the block's total in every thread.  lds: NT/64.
template <int NT, typename T, typename Op>
__device__ __forceinline__ T ss_scan(T v, T* lds, Op op, T ident, T& total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const T y = __shfl_up(v, o, kWave);
    if (lane >= o) v = op(v, y);
  }
  if (lane == kWave - 1) lds[w] = v;
  __syncthreads();
  T pre = ident, tot = ident;
#pragma unroll
  for (int q = 0; q < NT / kWave; ++q) {
    const T x = lds[q];
    if (q < w) pre = op(pre, x);
    tot = op(tot, x);
  }
  __syncthreads();
  total = tot;
  return op(pre, v);
}

struct SsAdd {
  template <typename T> __device__ T operator()(T a, T b) const { return a + b; }
};
struct SsMax {
  __device__ int operator()(int a, int b) const { return a > b ? a : b; }
};

// Exclusive scan of len <= NT * 8 u32 values in LDS, in place.
template <int NT>
__device__ __forceinline__ void ss_excl_scan_lds(uint32_t* v, int len, uint32_t* lds) {
  const int per = (len + NT - 1) / NT;
  const int j0 = threadIdx.x * per;
  uint32_t s = 0;
  for (int q = 0; q < per; ++q)
    if (j0 + q < len) s += v[j0 + q];
  uint32_t tot;
  uint32_t run = ss_scan<NT>(s, lds, SsAdd{}, 0u, tot) - s;
  for (int q = 0; q < per; ++q)
    if (j0 + q < len) {
      const uint32_t x = v[j0 + q];
      v[j0 + q] = run;
      run += x;
    }
  __syncthreads();
}

// Strided loops whose body waits on a global load (or a returning atomic) compile to one memory
// round trip per iteration; these helpers issue U loads per thread before using any of them.
template <int NT, int U = 8>
__device__ __forceinline__ void ss_copy_lds(uint32_t* dst, const uint32_t* src, int len) {
  for (int c0 = 0; c0 < len; c0 += NT * U) {
    uint32_t v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * NT + static_cast<int>(threadIdx.x);
      v[q] = src[i < len ? i : len - 1];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * NT + static_cast<int>(threadIdx.x);
      if (i < len) dst[i] = v[q];
    }
  }
}

template <int NT, int U = 8>
__device__ __forceinline__ uint32_t ss_sum_prefix(const uint32_t* src, int len) {  // this thread's share of sum src[0, len)
  uint32_t s = 0;
  for (int c0 = 0; c0 < len; c0 += NT * U) {
    uint32_t v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * NT + static_cast<int>(threadIdx.x);
      v[q] = src[i < len ? i : 0];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) s += c0 + q * NT + static_cast<int>(threadIdx.x) < len ? v[q] : 0u;
  }
  return s;
}

// Stable LSD radix sort of m keys (+ optional f32 values) by `passes` 8-bit digits from bit 0,
// ping-ponging a <-> b (the result is in a for an even pass count, b for odd).  The segment
// may live in LDS or in global memory (the same code; the compiler infers the address space).
// Chunks of NT keys in order; within a chunk, wave-ballot digit matches give stable ranks.
template <int NT, bool VALS>
__device__ void ss_block_lsd(uint32_t* ka, float* va, uint32_t* kb, float* vb, int m, int passes,
                             uint32_t (*cnt)[256], uint32_t* base, uint32_t* tot, uint32_t* slds) {
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint64_t below = lane ? (~0ull >> (kWave - lane)) : 0ull;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    for (int d = tid; d < 256; d += NT) base[d] = 0u;
    __syncthreads();
    // digit histogram (wave-aggregated: one LDS atomic per distinct digit per wave)
    for (int c0 = 0; c0 < m; c0 += NT) {
      const int i = c0 + tid;
      const bool valid = i < m;
      const uint32_t d = ((valid ? ka[i] : 0u) >> shift) & 255u;
      const uint64_t peers = ss_match(d, __ballot(valid));
      if (valid && (__ffsll(static_cast<long long>(peers)) - 1) == lane)
        atomicAdd(&base[d], static_cast<uint32_t>(__popcll(peers)));
    }
    __syncthreads();
    {
      const uint32_t c = tid < 256 ? base[tid] : 0u;
      uint32_t t_;
      const uint32_t inc = ss_scan<NT>(c, slds, SsAdd{}, 0u, t_);
      if (tid < 256) base[tid] = inc - c;
    }
    for (int c0 = 0; c0 < m; c0 += NT) {
      const int i = c0 + tid;
      const bool valid = i < m;
      const uint32_t k = valid ? ka[i] : 0u;
      float v = 0.f;
      if constexpr (VALS) v = valid ? va[i] : 0.f;
      const uint32_t d = (k >> shift) & 255u;
      const uint64_t peers = ss_match(d, __ballot(valid));
      const uint32_t r = static_cast<uint32_t>(__popcll(peers & below));
      for (int q = tid; q < (NT / kWave) * 256; q += NT) (&cnt[0][0])[q] = 0u;
      __syncthreads();
      if (valid && (__ffsll(static_cast<long long>(peers)) - 1) == lane) cnt[w][d] = static_cast<uint32_t>(__popcll(peers));
      __syncthreads();
      if (tid < 256) {
        uint32_t acc = 0;
#pragma unroll
        for (int q = 0; q < NT / kWave; ++q) {
          const uint32_t x = cnt[q][tid];
          cnt[q][tid] = acc;
          acc += x;
        }
        tot[tid] = acc;
      }
      __syncthreads();
      if (valid) {
        const uint32_t pos = base[d] + cnt[w][d] + r;
        kb[pos] = k;
        if constexpr (VALS) vb[pos] = v;
      }
      __syncthreads();
      if (tid < 256) base[tid] += tot[tid];
    }
    __syncthreads();
    uint32_t* tk = ka; ka = kb; kb = tk;
    float* tv = va; va = vb; vb = tv;
  }
}

// Bins in ascending key (= descending score) order: 0 NaN, 1 +inf, then the 2B - 1 regular
// buckets, last -inf.  The reference ends a tie group wherever `diff != 0`, and for NaN and
// +-inf neighbours that difference is NaN: every such sample is a group of its own, taken in
// sort (= source index) order.  Their bins therefore keep source order (ordered ranks in the
// scatter, per-tile counts instead of cursor atomics) and are scanned as singletons.
constexpr uint32_t kKeyNan = 0x003fffffu, kKeyPinf = 0x007fffffu, kKeyNinf = 0xff800000u;

__device__ __forceinline__ int ss_special(uint32_t k) {  // 0 NaN, 1 +inf, 2 -inf, -1 finite
  return k == kKeyNan ? 0 : k == kKeyPinf ? 1 : k == kKeyNinf ? 2 : -1;
}

// Interleaved branch-free lower_bound of kSsPer keys over sp[0, B) (sp[B-1] = sentinel):
// regular bucket = 2 * lb + (key == sp[lb]); bin = 2 + bucket, or the special bins.
__device__ __forceinline__ void ss_buckets(const uint32_t* sp, int B, int nbins, const uint32_t (&k)[kSsPer],
                                           uint32_t (&bid)[kSsPer]) {
  uint32_t idx[kSsPer];
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) idx[r] = 0;
  for (int step = B >> 1; step > 0; step >>= 1) {
#pragma unroll
    for (int r = 0; r < kSsPer; ++r) idx[r] += sp[idx[r] + step - 1] < k[r] ? static_cast<uint32_t>(step) : 0u;
  }
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const int c = ss_special(k[r]);
    const uint32_t reg = 2u + 2u * idx[r] + ((static_cast<int>(idx[r]) < B - 1 && sp[idx[r]] == k[r]) ? 1u : 0u);
    bid[r] = c < 0 ? reg : c == 2 ? static_cast<uint32_t>(nbins - 1) : static_cast<uint32_t>(c);
  }
}

__global__ __launch_bounds__(kSsSampleT) void ss_sample_kernel(SampleSortAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t* ka = sh;
  uint32_t* kb = ka + a.S;
  uint32_t(*cnt)[256] = reinterpret_cast<uint32_t(*)[256]>(kb + a.S);
  uint32_t* base = kb + a.S + (kSsSampleT / kWave) * 256;
  uint32_t* tot = base + 256;
  uint32_t* slds = tot + 256;
  const int64_t q = a.n / a.S;  // stratum length (>= 4)
  for (int s = threadIdx.x; s < a.S; s += kSsSampleT) {
    uint32_t h = static_cast<uint32_t>(s) * 2654435761u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    const int64_t pos = static_cast<int64_t>(s) * q + static_cast<int64_t>(h % static_cast<uint32_t>(q));
    ka[s] = ss_key(a.x[pos]);
  }
  __syncthreads();
  ss_block_lsd<kSsSampleT, false>(ka, nullptr, kb, nullptr, a.S, 4, cnt, base, tot, slds);
  const int per = a.S / a.B;
  for (int j = threadIdx.x; j < a.B; j += kSsSampleT) a.sp[j] = j < a.B - 1 ? ka[(j + 1) * per] : 0xffffffffu;
}

__global__ __launch_bounds__(kSsT) void ss_hist_kernel(SampleSortAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t* sp = sh;
  uint32_t* hist = sh + a.B;
  ss_copy_lds<kSsT>(sp, a.sp, a.B);
  for (int j = threadIdx.x; j < a.nbins; j += kSsT) hist[j] = 0u;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kSsTile + threadIdx.x;
  uint32_t k[kSsPer], bid[kSsPer];
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const int64_t i = t0 + r * kSsT;
    k[r] = ss_key(a.x[i < a.n ? i : a.n - 1]);
  }
  __syncthreads();
  ss_buckets(sp, a.B, a.nbins, k, bid);
#pragma unroll
  for (int r = 0; r < kSsPer; ++r)
    if (t0 + r * kSsT < a.n) atomicAdd(&hist[bid[r]], 1u);
  __syncthreads();
  for (int j = threadIdx.x; j < a.nbins; j += kSsT) {
    const uint32_t c = hist[j];
    if (c) atomicAdd(&a.counts[j], c);
  }
  // this tile's special-bin counts (the scatter places those bins in source order)
  if (threadIdx.x < 3) {
    const int j = threadIdx.x == 2 ? a.nbins - 1 : threadIdx.x;
    a.spc[3 * blockIdx.x + threadIdx.x] = hist[j];
  }
}

template <typename PT>
__global__ __launch_bounds__(kSsT) void ss_scatter_kernel(SampleSortAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t* sp = sh;
  uint32_t* lcnt = sp + a.B;         // tile counts -> (after the rank pass) tile starts
  uint32_t* gbase = lcnt + a.nbins;  // global bucket starts -> this tile's run bases
  uint32_t* skey = gbase + a.nbins;
  float* stgt = reinterpret_cast<float*>(skey + kSsTile);
  uint32_t* sbid = reinterpret_cast<uint32_t*>(stgt + kSsTile);
  uint32_t* slds = sbid + kSsTile;
  uint32_t* sord = slds + 16;        // [kSsPer][4 waves][3 classes] ballot counts, then prefixes
  uint32_t* sprev = sord + kSsPer * 12;  // [3] special samples of the tiles before this one
  ss_copy_lds<kSsT>(sp, a.sp, a.B);
  ss_copy_lds<kSsT>(gbase, a.counts, a.nbins);
  for (int j = threadIdx.x; j < a.nbins; j += kSsT) lcnt[j] = 0u;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kSsTile + threadIdx.x;
  uint32_t k[kSsPer], bid[kSsPer], rk[kSsPer];
  float tv[kSsPer];
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const int64_t i = t0 + r * kSsT;
    const int64_t ic = i < a.n ? i : a.n - 1;
    k[r] = ss_key(a.x[ic]);
    tv[r] = ss_target<PT>(a.t, ic);
  }
  {  // special samples of earlier tiles (per class)
    uint32_t c[3] = {0u, 0u, 0u};
    const int nprev = static_cast<int>(blockIdx.x);
    for (int u0 = 0; u0 < nprev; u0 += kSsT * 4) {
      uint32_t v[4][3];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = u0 + q * kSsT + static_cast<int>(threadIdx.x);
        const int uc = u < nprev ? u : 0;
        v[q][0] = a.spc[3 * uc];
        v[q][1] = a.spc[3 * uc + 1];
        v[q][2] = a.spc[3 * uc + 2];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const bool ok = u0 + q * kSsT + static_cast<int>(threadIdx.x) < nprev;
        c[0] += ok ? v[q][0] : 0u;
        c[1] += ok ? v[q][1] : 0u;
        c[2] += ok ? v[q][2] : 0u;
      }
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      uint32_t tot;
      ss_scan<kSsT>(c[q], slds, SsAdd{}, 0u, tot);
      if (threadIdx.x == 0) sprev[q] = tot;
    }
  }
  __syncthreads();
  ss_excl_scan_lds<kSsT>(gbase, a.nbins, slds);  // global bucket starts
  ss_buckets(sp, a.B, a.nbins, k, bid);
  // special samples: ranks in source order (round, wave, lane); others: LDS-atomic ranks
  const bool any_special = (a.spc[3 * blockIdx.x] | a.spc[3 * blockIdx.x + 1] | a.spc[3 * blockIdx.x + 2]) != 0u;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint64_t below = lane ? (~0ull >> (kWave - lane)) : 0ull;
  uint64_t spm[kSsPer];
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    const bool valid = t0 + r * kSsT < a.n;
    const int c = valid && any_special ? ss_special(k[r]) : -1;
    const uint64_t m0 = __ballot(c == 0), m1 = __ballot(c == 1), m2 = __ballot(c == 2);
    if (lane == 0) {
      sord[(r * 4 + w) * 3] = static_cast<uint32_t>(__popcll(m0));
      sord[(r * 4 + w) * 3 + 1] = static_cast<uint32_t>(__popcll(m1));
      sord[(r * 4 + w) * 3 + 2] = static_cast<uint32_t>(__popcll(m2));
    }
    spm[r] = c == 0 ? m0 : c == 1 ? m1 : c == 2 ? m2 : 0ull;
    rk[r] = (valid && c < 0) ? atomicAdd(&lcnt[bid[r]], 1u) : 0u;
  }
  __syncthreads();
  if (threadIdx.x < 3) {  // exclusive prefix over (round, wave) per class
    uint32_t acc = 0;
    for (int q = 0; q < kSsPer * 4; ++q) {
      const uint32_t x = sord[q * 3 + threadIdx.x];
      sord[q * 3 + threadIdx.x] = acc;
      acc += x;
    }
    const int j = threadIdx.x == 2 ? a.nbins - 1 : threadIdx.x;
    lcnt[j] = acc;
    gbase[j] += sprev[threadIdx.x];
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    if (spm[r]) {
      const int c = ss_special(k[r]);
      rk[r] = sord[(r * 4 + w) * 3 + c] + static_cast<uint32_t>(__popcll(spm[r] & below));
    }
  }
  for (int j0 = 2; j0 < a.nbins - 1; j0 += kSsT * 8) {  // all of this thread's cursor atomics in flight
    uint32_t r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = j0 + q * kSsT + static_cast<int>(threadIdx.x);
      const uint32_t c = j < a.nbins - 1 ? lcnt[j] : 0u;
      r[q] = c ? atomicAdd(&a.cursor[j], c) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = j0 + q * kSsT + static_cast<int>(threadIdx.x);
      if (j < a.nbins - 1) gbase[j] += r[q];
    }
  }
  ss_excl_scan_lds<kSsT>(lcnt, a.nbins, slds);  // tile starts (has a trailing barrier)
#pragma unroll
  for (int r = 0; r < kSsPer; ++r) {
    if (t0 + r * kSsT < a.n) {
      const uint32_t p = lcnt[bid[r]] + rk[r];
      skey[p] = k[r];
      stgt[p] = tv[r];
      sbid[p] = bid[r];
    }
  }
  __syncthreads();
  const int64_t rem = a.n - static_cast<int64_t>(blockIdx.x) * kSsTile;
  const int tn = static_cast<int>(rem < kSsTile ? rem : kSsTile);
  for (int p = threadIdx.x; p < tn; p += kSsT) {
    const uint32_t j = sbid[p];
    const uint32_t pos = gbase[j] + (static_cast<uint32_t>(p) - lcnt[j]);
    a.keys_out[pos] = skey[p];
    a.t_out[pos] = stgt[p];
  }
}

// Tie scan of a sorted segment: W = sum over tie groups of n_g * (TP before g + p_g / 2), and
// the segment's positive mass P.  Chunks of kSsL; the group open at a chunk's end carries over.
__device__ void ss_tie_scan(const uint32_t* sk, const float* sv, int m, bool singletons, double* s_e, double* dl,
                            int* il, double* s_cd, int* s_ci, double& W, double& P) {
  const int tid = threadIdx.x;
  double run = 0.0, wsum = 0.0, carry_e = 0.0;
  int carry_h = 0;
  for (int c0 = 0; c0 < m; c0 += kSsL) {
    const int i = c0 + tid;
    const bool valid = i < m;
    const uint32_t k = valid ? sk[i] : 0u;
    const double t = valid ? static_cast<double>(sv[i]) : 0.0;
    const bool head = valid && (singletons || i == 0 || sk[i - 1] != k);
    const bool tail = valid && (singletons || i == m - 1 || sk[i + 1] != k);
    double ctot;
    const double I = run + ss_scan<kSsL>(t, dl, SsAdd{}, 0.0, ctot);
    s_e[tid] = I - t;
    int h_;
    const int H = ss_scan<kSsL>(head ? i : -1, il, SsMax{}, -1, h_);  // barriers: s_e visible
    const int hidx = H >= c0 ? H : carry_h;
    const double eh = H >= c0 ? s_e[H - c0] : carry_e;
    if (tail) {
      const double pg = I - eh;
      const double ng = static_cast<double>(i - hidx + 1) - pg;
      wsum += ng * (eh + 0.5 * pg);
    }
    const int last = (m - c0 < kSsL ? m - c0 : kSsL) - 1;
    if (tid == last) {
      *s_ci = hidx;
      *s_cd = eh;
    }
    __syncthreads();
    carry_h = *s_ci;
    carry_e = *s_cd;
    run += ctot;
    __syncthreads();
  }
  double tot;
  ss_scan<kSsL>(wsum, dl, SsAdd{}, 0.0, tot);
  W = tot;
  P = run;
}

// W and P of a between bucket without sorting it: its samples are counted into 256 sub-bins by
// the top 8 free key bits (LDS atomics), placed sub-bin-contiguous (any order inside), and every
// negative-weight sample adds (1 - t) * (TP of lower sub-bins + TP of smaller keys in its own
// sub-bin + half the TP of equal keys, itself included) - a pair loop over its sub-bin only
// (~m / 256 samples for a quantile bucket).  The copy lives in LDS, or in global scratch for an
// oversized bucket (same code, pointers of either address space).
__device__ __forceinline__ void ss_subbin_area(const uint32_t* gk, const float* gt, int m, uint32_t* sk, float* st,
                                               uint32_t* cnt, uint32_t* cur, uint32_t* off, double* tsum, double* dl,
                                               uint32_t* slds, double& W, double& P) {
  const int tid = threadIdx.x;
  // the sub-bin width from the bucket's actual key range (a splitter-bounded range can be far
  // wider than its samples - the end buckets are unbounded - and put every sample in one sub-bin)
  constexpr int U = 8;  // loads in flight per thread in each sweep
  uint32_t kmin = 0xffffffffu, kmax = 0u;
  for (int c0 = 0; c0 < m; c0 += kSsL * U) {
    uint32_t kk[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * kSsL + tid;
      kk[q] = gk[i < m ? i : m - 1];  // the clamped duplicate leaves min / max unchanged
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      kmin = kk[q] < kmin ? kk[q] : kmin;
      kmax = kk[q] > kmax ? kk[q] : kmax;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t x = __shfl_xor(kmin, o, kWave), y = __shfl_xor(kmax, o, kWave);
    kmin = x < kmin ? x : kmin;
    kmax = y > kmax ? y : kmax;
  }
  if (lane_id() == 0) {
    cnt[tid >> 6] = kmin;
    cur[tid >> 6] = kmax;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kSsL / kWave; ++q) {
    kmin = cnt[q] < kmin ? cnt[q] : kmin;
    kmax = cur[q] > kmax ? cur[q] : kmax;
  }
  const uint32_t lo = kmin, span = kmax - kmin;
  const int sbits = span ? 32 - __clz(static_cast<int>(span)) : 0;
  const int shift = sbits > 8 ? sbits - 8 : 0;
  __syncthreads();
  cnt[tid] = 0u;
  tsum[tid] = 0.0;
  __syncthreads();
  for (int c0 = 0; c0 < m; c0 += kSsL * U) {
    uint32_t kk[U];
    float tt[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * kSsL + tid;
      const int ic = i < m ? i : m - 1;
      kk[q] = gk[ic];
      tt[q] = gt[ic];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (c0 + q * kSsL + tid < m) {
        const uint32_t sub = (kk[q] - lo) >> shift;
        atomicAdd(&cnt[sub], 1u);
        atomicAdd(&tsum[sub], static_cast<double>(tt[q]));
      }
    }
  }
  __syncthreads();
  const uint32_t c = cnt[tid];
  const double ts = tsum[tid];
  uint32_t ctot;
  const uint32_t cinc = ss_scan<kSsL>(c, slds, SsAdd{}, 0u, ctot);
  double ttot;
  const double tinc = ss_scan<kSsL>(ts, dl, SsAdd{}, 0.0, ttot);
  off[tid] = cinc - c;
  cur[tid] = cinc - c;
  tsum[tid] = tinc - ts;  // TP of the lower sub-bins
  __syncthreads();
  for (int c0 = 0; c0 < m; c0 += kSsL * U) {
    uint32_t kk[U];
    float tt[U];
#pragma unroll
    for (int q = 0; q < U; ++q) {
      const int i = c0 + q * kSsL + tid;
      const int ic = i < m ? i : m - 1;
      kk[q] = gk[ic];
      tt[q] = gt[ic];
    }
#pragma unroll
    for (int q = 0; q < U; ++q) {
      if (c0 + q * kSsL + tid < m) {
        const uint32_t r = atomicAdd(&cur[(kk[q] - lo) >> shift], 1u);
        sk[r] = kk[q];
        st[r] = tt[q];
      }
    }
  }
  __syncthreads();
  double w = 0.0;
  for (int i = tid; i < m; i += kSsL) {
    const float t = st[i];
    if (t != 1.f) {
      const uint32_t k = sk[i];
      const uint32_t sub = (k - lo) >> shift;
      const int j0 = static_cast<int>(off[sub]), j1 = j0 + static_cast<int>(cnt[sub]);
      float lt = 0.f, eq = 0.f;
      for (int j = j0; j < j1; ++j) {
        const uint32_t kj = sk[j];
        const float tj = st[j];
        lt += kj < k ? tj : 0.f;
        eq += kj == k ? tj : 0.f;
      }
      w += (1.0 - static_cast<double>(t)) * (tsum[sub] + static_cast<double>(lt) + 0.5 * static_cast<double>(eq));
    }
  }
  double wt;
  ss_scan<kSsL>(w, dl, SsAdd{}, 0.0, wt);
  W = wt;
  P = ttot;
}

__global__ __launch_bounds__(kSsL) void ss_local_kernel(SampleSortAucArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sh[];
  uint32_t* sk = sh;
  float* st = reinterpret_cast<float*>(sk + kSsCap);
  uint32_t* cnt = reinterpret_cast<uint32_t*>(st + kSsCap);
  uint32_t* cur = cnt + 256;
  uint32_t* off = cur + 256;
  uint32_t* slds = off + 256;
  double* tsum = reinterpret_cast<double*>(slds + 16);
  double* s_e = tsum + 256;
  double* dl = s_e + kSsL;
  int* il = reinterpret_cast<int*>(dl + 16);
  double* s_cd = reinterpret_cast<double*>(il + 16);
  int* s_ci = reinterpret_cast<int*>(s_cd + 1);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t part = ss_sum_prefix<kSsL>(a.counts, b);
  uint32_t start;
  ss_scan<kSsL>(part, slds, SsAdd{}, 0u, start);
  const int m = static_cast<int>(a.counts[b]);
  double W = 0.0, P = 0.0;
  if (m > 0) {
    uint32_t* gk = a.keys_out + start;
    float* gt = a.t_out + start;
    if (b < 2 || b == a.nbins - 1) {  // NaN / +inf / -inf: singletons in source order
      ss_tie_scan(gk, gt, m, true, s_e, dl, il, s_cd, s_ci, W, P);
    } else {
      const int rb = b - 2;
      const int lb = rb >> 1;
      const uint32_t lo = lb > 0 ? a.sp[lb - 1] + 1u : 0u;
      const uint32_t hi = lb < a.B - 1 ? a.sp[lb] - 1u : 0xffffffffu;
      const int bits = (rb & 1) || lo == hi ? 0 : 32 - __clz(static_cast<int>(lo ^ hi));
      if (bits == 0) {  // one score: a single tie group, W = N * P / 2
        double sum = 0.0;
        for (int c0 = 0; c0 < m; c0 += kSsL * 8) {
          float tt[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int i = c0 + q * kSsL + tid;
            tt[q] = gt[i < m ? i : m - 1];
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) sum += c0 + q * kSsL + tid < m ? tt[q] : 0.f;
        }
        ss_scan<kSsL>(sum, dl, SsAdd{}, 0.0, P);
        W = 0.5 * (static_cast<double>(m) - P) * P;
      } else {
        if (m <= kSsCap)
          ss_subbin_area(gk, gt, m, sk, st, cnt, cur, off, tsum, dl, slds, W, P);
        else  // oversized bucket: the sub-bin copy in global scratch (L2-resident)
          ss_subbin_area(gk, gt, m, a.keys_tmp + start, a.t_tmp + start, cnt, cur, off, tsum, dl, slds, W, P);
      }
    }
  }
  if (tid == 0) {
    a.rec[3 * b] = P;
    a.rec[3 * b + 1] = static_cast<double>(m) - P;
    a.rec[3 * b + 2] = W;
  }
}

__global__ __launch_bounds__(1024) void ss_final_kernel(SampleSortAucArgs a) {
  __shared__ double dl[16];
  double run = 0.0, area = 0.0, neg = 0.0;
  for (int c0 = 0; c0 < a.nbins; c0 += 1024) {
    const int j = c0 + threadIdx.x;
    const bool ok = j < a.nbins;
    const double p = ok ? a.rec[3 * j] : 0.0;
    const double nb = ok ? a.rec[3 * j + 1] : 0.0;
    const double w = ok ? a.rec[3 * j + 2] : 0.0;
    double ctot;
    const double excl = run + ss_scan<1024>(p, dl, SsAdd{}, 0.0, ctot) - p;
    area += w + nb * excl;
    neg += nb;
    run += ctot;
    if (ok) {  // self-cleaning counters for the next call
      a.counts[j] = 0u;
      a.cursor[j] = 0u;
    }
  }
  double ta, tn;
  ss_scan<1024>(area, dl, SsAdd{}, 0.0, ta);
  ss_scan<1024>(neg, dl, SsAdd{}, 0.0, tn);
  if (threadIdx.x == 0) {
    const double f = run * tn;
    a.out[0] = f == 0.0 ? 0.5 : ta / f;
  }
}

}  // namespace

int samplesort_auc_buckets(int64_t n) {
  int64_t b = 16;
  while (b < 1024 && b * 2048 < n) b *= 2;
  return static_cast<int>(b);
}

bool samplesort_auc_supported(int64_t n) { return n >= (int64_t{1} << 15) && n <= (int64_t{1} << 21); }

int launch_samplesort_auc(const SampleSortAucArgs& a, hipStream_t stream) {
  if (!samplesort_auc_supported(a.n) || a.B != samplesort_auc_buckets(a.n) || a.S != 4 * a.B ||
      a.nbins != 2 * a.B + 2 || a.spc == nullptr)
    return -2;
  const unsigned tiles = static_cast<unsigned>((a.n + kSsTile - 1) / kSsTile);
  const size_t lds_sample = (2 * static_cast<size_t>(a.S) + (kSsSampleT / kWave) * 256 + 512 + 16) * 4;
  const size_t lds_hist = (static_cast<size_t>(a.B) + a.nbins) * 4;
  const size_t lds_scatter = (static_cast<size_t>(a.B) + 2 * a.nbins + 3 * kSsTile + 16 + kSsPer * 12 + 4) * 4;
  const size_t lds_local = (2 * static_cast<size_t>(kSsCap) + 3 * 256 + 16) * 4 + (256 + kSsL + 16) * 8 + 16 * 4 + 16;
  // dynamic LDS beyond 64 KB needs the per-kernel opt-in
  static const bool lds_ok = [] {
    constexpr int kMax = 160 * 1024;
    bool ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_sample_kernel),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_local_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_hist_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_scatter_kernel<float>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_scatter_kernel<int64_t>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_scatter_kernel<int32_t>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    ok = ok && hipFuncSetAttribute(reinterpret_cast<const void*>(&ss_scatter_kernel<uint8_t>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kMax) == hipSuccess;
    return ok;
  }();
  if (!lds_ok) return -3;
  hipLaunchKernelGGL(ss_sample_kernel, dim3(1), dim3(kSsSampleT), lds_sample, stream, a);
  hipLaunchKernelGGL(ss_hist_kernel, dim3(tiles), dim3(kSsT), lds_hist, stream, a);
  switch (a.t_dt) {
    case DType::f32: hipLaunchKernelGGL(ss_scatter_kernel<float>, dim3(tiles), dim3(kSsT), lds_scatter, stream, a); break;
    case DType::i64: hipLaunchKernelGGL(ss_scatter_kernel<int64_t>, dim3(tiles), dim3(kSsT), lds_scatter, stream, a); break;
    case DType::i32: hipLaunchKernelGGL(ss_scatter_kernel<int32_t>, dim3(tiles), dim3(kSsT), lds_scatter, stream, a); break;
    case DType::u8: case DType::b8: hipLaunchKernelGGL(ss_scatter_kernel<uint8_t>, dim3(tiles), dim3(kSsT), lds_scatter, stream, a); break;
    default: return -2;
  }
  hipLaunchKernelGGL(ss_local_kernel, dim3(static_cast<unsigned>(a.nbins)), dim3(kSsL), lds_local, stream, a);
  hipLaunchKernelGGL(ss_final_kernel, dim3(1), dim3(1024), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
