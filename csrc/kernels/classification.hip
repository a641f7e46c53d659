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
// Design (gfx950, measured with csrc/bench/k1_variants.hip at N=8192, C=1000, fp32):
//  * "wide" kernel (C > 32): one wave64 per row.  Every lane issues ALL its 16-B loads of the
//    row chunk (4 x float4 = 1024 f32 columns, or 4 x 8 x bf16 = 2048 columns) before any
//    compare, and the grid is sized so every wave owns ~one row (2048 blocks x 4 waves for
//    N=8192): the whole 32.8 MB read is in flight at once -> 4.5 TB/s.
//  * two-phase argmax per lane: v_maximum3_f32 (NaN-propagating max) over the lane's values,
//    then the first column equal to that max; the cross-lane step is a max-reduce followed by
//    a min-reduce of candidate indices.  ~2.5 VALU per element instead of the ~12 of a
//    (value, index) compare chain (10.5 -> 7.3 us).  Rows containing NaN take a wave-uniform
//    slow path with exact torch.argmax semantics (NaN is the max, first index wins).
//  * micro counts are folded with tea_fold.h (sharded 64-bit {arrivals, count} cells): one
//    same-address float atomic per block costs +23 us at 2048 blocks, the fold +0.5 us.
//  * "narrow" kernel (C <= 32): one thread per row, LDS-privatised class histograms.
//  * invalid targets / predictions never fault: they are skipped and flagged in ``err``
//    (bit 0: target out of range, bit 1: predicted label out of range).
#include <algorithm>
#include <cstdlib>

#include "tea_common.h"
#include "tea_fold.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kChunkLoads = 4;  // 16-B loads per lane per row chunk
constexpr int kNarrowMaxC = 32;

__device__ __forceinline__ float fmaximum(float a, float b) {
  return __builtin_elementwise_maximum(a, b);
}

template <int KIND>
__device__ __forceinline__ float h16(uint16_t b) {
  return KIND == 1 ? bf16_to_f32(b) : f16_to_f32(b);
}

// KIND 0: f32 (VEC 4 or 1); KIND 1: bf16, KIND 2: f16 (VEC 8 or 1)
template <int KIND, int VEC>
__device__ __forceinline__ void load_vec(const void* row, int col, float (&v)[VEC]) {
  if constexpr (KIND == 0 && VEC == 4) {
    // plain loads: __builtin_nontemporal_load here measured 116-117k vs 122-124k updates/s
    const float4 x = *reinterpret_cast<const float4*>(static_cast<const float*>(row) + col);
    v[0] = x.x;
    v[1] = x.y;
    v[2] = x.z;
    v[3] = x.w;
  } else if constexpr (KIND == 0) {
    v[0] = static_cast<const float*>(row)[col];
  } else if constexpr (VEC == 8) {
    const uint4 x = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(row) + col);
    const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = h16<KIND>(static_cast<uint16_t>(w[e] & 0xffffu));
      v[2 * e + 1] = h16<KIND>(static_cast<uint16_t>(w[e] >> 16));
    }
  } else {
    v[0] = h16<KIND>(static_cast<const uint16_t*>(row)[col]);
  }
}

// UNAL rows (f32, any width >= 4, any 4-B alignment): 16-B loads at 4-B-aligned addresses
// (tea_common.h load_f4u).  Loads only compute an address (no use of the loaded registers, so
// every load of a row stays in flight together); the lane whose 4 columns straddle the row end
// (C % 4 != 0) loads the row's LAST 4 columns, and unal_fix_tail - run after all of a chunk's
// loads are issued, on the one wave-load that holds the row end (a wave-uniform test) -
// rotates them into place, so element e holds nominal column col + e and the columns past C
// read -inf: every consumer below (max, target select, tie / rank counts, argmax indices) is
// unchanged.  Lanes wholly past C keep the aligned paths' convention (clamped copies of
// columns 0..3, masked where the consumer needs it).
template <int KIND, int VEC, bool UNAL>
__device__ __forceinline__ void load_row_vec(const void* row, int col, int C, float (&v)[VEC]) {
  if constexpr (UNAL) {
    static_assert(KIND == 0 && VEC == 4, "UNAL rows are f32");
    const int lc = col + 4 <= C ? col : (col < C ? C - 4 : 0);
    const float4 q = load_f4u(static_cast<const float*>(row) + lc);
    v[0] = q.x;
    v[1] = q.y;
    v[2] = q.z;
    v[3] = q.w;
  } else {
    load_vec<KIND, VEC>(row, col < C ? col : 0, v);
  }
}

// `n` wave-loads starting at column `base` (wave-load u covers base + u * 256 ...): rotate the
// straddling lane's values of the wave-load holding column C & ~3 (only when C % 4 != 0)
template <int N>
__device__ __forceinline__ void unal_fix_tail(float (&v)[N][4], int base, int C, int lane) {
  if ((C & 3) == 0) return;
  const int cv = C & ~3, sh = 4 - (C & 3);
  constexpr int STEP = kWave * 4;
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const int ub = base + u * STEP;
    if (cv >= ub && cv < ub + STEP) {  // wave-uniform
      const bool me = lane == (cv - ub) / 4;
      const float ninf = -__builtin_huge_valf();
      float r[4];  // r[e] = v[e + sh] (past the row end: -inf), selects on the uniform sh
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float s1 = e + 1 < 4 ? v[u][e + 1 < 4 ? e + 1 : 3] : ninf;
        const float s2 = e + 2 < 4 ? v[u][e + 2 < 4 ? e + 2 : 3] : ninf;
        const float s3 = e + 3 < 4 ? v[u][e + 3 < 4 ? e + 3 : 3] : ninf;
        r[e] = sh == 1 ? s1 : sh == 2 ? s2 : s3;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[u][e] = me ? r[e] : v[u][e];
    }
  }
}

template <int KIND>
__device__ __forceinline__ float load_one(const void* row, int64_t col) {
  if constexpr (KIND == 0) return static_cast<const float*>(row)[col];
  return h16<KIND>(static_cast<const uint16_t*>(row)[col]);
}

__device__ __forceinline__ int64_t load_target(const void* tgt, DType dt, int64_t i) {
  return dt == DType::i64 ? static_cast<const int64_t*>(tgt)[i] : load_as_i64(tgt, dt, i);
}

// Per-row bookkeeping (one lane / thread per row).  Histogram atomics go to ``hist`` which
// is either global memory or an LDS privatisation (narrow kernel).
struct Hist {
  float* cls_correct;
  float* cls_label;
  float* cls_pred;
  float* cls_fp;
  float* confusion;
};

__device__ __forceinline__ void row_hist(const Hist& h, int64_t C, int64_t t, int64_t pred,
                                         bool correct, int* err, int check_target, int* err_max) {
  const bool t_ok = t >= 0 && t < C;
  const bool p_ok = pred >= 0 && pred < C;
  if (err) {
    const bool bad_t = !t_ok && (h.cls_label || h.cls_correct || h.confusion || check_target);
    const bool bad_p = !p_ok && (h.cls_pred || h.confusion || (h.cls_fp && !correct));
    if (bad_t) atomicOr(err, 1);
    if (bad_p) atomicOr(err, 2);
    // the largest offending label / prediction: the reference's message prints torch.max of
    // the batch, which is that value whenever one is >= C (its check)
    if (err_max && bad_t && t >= C) atomicMax(err_max, static_cast<int>(t < 2147483647 ? t : 2147483647));
    if (err_max && bad_p && pred >= C) atomicMax(err_max + 1, static_cast<int>(pred < 2147483647 ? pred : 2147483647));
  }
  if (t_ok) {
    if (h.cls_correct && correct) atomicAdd(h.cls_correct + t, 1.f);
    if (h.cls_label) atomicAdd(h.cls_label + t, 1.f);
  }
  if (p_ok && h.cls_pred) atomicAdd(h.cls_pred + pred, 1.f);
  if (p_ok && h.cls_fp && !correct) atomicAdd(h.cls_fp + pred, 1.f);
  if (t_ok && p_ok && h.confusion) atomicAdd(h.confusion + t * C + pred, 1.f);
}

// Block epilogue for the micro counters: LDS reduce, then the sharded fold.
__device__ __forceinline__ void fold_or_add(unsigned long long* ws, uint32_t v, float* dst) {
  if (ws) {
    fold_count(ws, v, dst);
  } else if (v) {
    atomicAdd(dst, static_cast<float>(v));
  }
}

// ``my_rows`` = rows this thread/lane accounted for; incorrect = rows - correct.
__device__ __forceinline__ void block_micro(const ClsCountsArgs& a, uint32_t my_correct,
                                            uint32_t my_rows) {
  __shared__ uint32_t lds[2][kWavesPerBlock];
  const uint32_t w = static_cast<uint32_t>(wave_sum(static_cast<int>(my_correct)));
  const uint32_t r = static_cast<uint32_t>(wave_sum(static_cast<int>(my_rows)));
  if (lane_id() == 0) {
    lds[0][threadIdx.x >> 6] = w;
    lds[1][threadIdx.x >> 6] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0, rows = 0;
#pragma unroll
    for (int k = 0; k < kWavesPerBlock; ++k) {
      s += lds[0][k];
      rows += lds[1][k];
    }
    if (a.micro_correct) fold_or_add(a.fold_ws, s, a.micro_correct);
    if (a.micro_incorrect)
      fold_or_add(a.fold_ws ? a.fold_ws + kFoldCells : nullptr, rows - s, a.micro_incorrect);
    if (blockIdx.x == 0) {
      if (a.micro_total) atomicAdd(a.micro_total, static_cast<float>(a.n));
      if (a.micro_total2) atomicAdd(a.micro_total2, static_cast<float>(a.n));
    }
  }
}

// Exact torch.argmax over one row (slow path, NaN-aware compare chain).
template <int KIND>
__device__ __noinline__ int row_argmax_exact(const void* rp, int C, int lane) {
  float bv = -__builtin_huge_valf();
  int bi = 0x7fffffff;
  for (int col = lane; col < C; col += kWave) {
    const float v = load_one<KIND>(rp, col);
    if (argmax_better(v, col, bv, bi)) {
      bv = v;
      bi = col;
    }
  }
  wave_argmax(bv, bi);
  return bi;
}

// one chunk of a row (kChunkLoads wave-loads from column `base`): unconditional clamped loads
// only (a guarded load compiles to a branch and a vmcnt(0) per load, and any use of a loaded
// register here would wait for it - serialising the next chunk's prefetch behind this one)
template <int KIND, int VEC, bool UNAL>
__device__ __forceinline__ void load_chunk(const void* rp, int base, int C, int lane, float (&v)[kChunkLoads][VEC]) {
  constexpr int STEP = kWave * VEC;
#pragma unroll
  for (int u = 0; u < kChunkLoads; ++u) load_row_vec<KIND, VEC, UNAL>(rp, base + u * STEP + lane * VEC, C, v[u]);
}

// ... and when the chunk is consumed: the UNAL tail rotation, columns past C -> -inf
template <int VEC, bool UNAL>
__device__ __forceinline__ void finish_chunk(float (&v)[kChunkLoads][VEC], int base, int C, int lane) {
  constexpr int STEP = kWave * VEC;
  if constexpr (UNAL) unal_fix_tail<kChunkLoads>(v, base, C, lane);
#pragma unroll
  for (int u = 0; u < kChunkLoads; ++u) {
    const bool in = base + u * STEP + lane * VEC < C;
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[u][e] = in ? v[u][e] : -__builtin_huge_valf();
  }
}

// PRED = false: the caller needs only "was the prediction correct" (micro / macro accuracy:
// no predicted-label histograms) and the row fits one chunk (C <= 1024 f32 / 2048 16-bit).
// Then the wave compares the row max with the target's own score first: a row whose target is
// not the max is incorrect without locating the argmax (the v2 index pass + min-reduce is only
// run when they are equal, to apply torch.argmax's first-index rule to ties).
template <int KIND, int VEC, bool TOPK, bool PRED = true, bool UNAL = false>
__device__ __forceinline__ void cls_wide_body(const ClsCountsArgs& a) {
  const int lane = lane_id();
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  constexpr int STEP = kWave * VEC;             // columns per wave-load
  constexpr int CHUNK = STEP * kChunkLoads;     // columns per chunk
  const int C = static_cast<int>(a.c);
  const Hist h{a.cls_correct, a.cls_label, a.cls_pred, a.cls_fp, a.confusion};
  uint32_t correct_acc = 0, rows_acc = 0;

  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wave_id(); row < a.n;
       row += nwaves) {
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELSIZE;
    bool correct;
    int64_t pred = -1;
    int64_t t;
    if constexpr (!TOPK && !PRED) {
      // the whole row (C <= CHUNK) is loaded before the target: the loads do not depend on it, so
      // its round trip overlaps theirs (v2 loaded the target first and waited for it, then the
      // row and then the target's own score - two dependent round trips per row).  Clamped
      // unconditional loads, masked to -inf afterwards.
      float v[kChunkLoads][VEC];
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u) load_row_vec<KIND, VEC, UNAL>(rp, u * STEP + lane * VEC, C, v[u]);
      t = load_target(a.target, a.tg_dt, row);
      if constexpr (UNAL) unal_fix_tail<kChunkLoads>(v, 0, C, lane);
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u) {
        const bool in = u * STEP + lane * VEC < C;
#pragma unroll
        for (int e = 0; e < VEC; ++e) v[u][e] = in ? v[u][e] : -__builtin_huge_valf();
      }
      const bool t_ok = t >= 0 && t < C;
      // the target's score from the registers: t is wave-uniform (one row per wave)
      const int tu = __builtin_amdgcn_readfirstlane(static_cast<int>(t_ok ? t : 0));
      const int ut = tu / STEP, et = tu % VEC, owner = (tu % STEP) / VEC;
      float sel = 0.f;
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) sel = (u == ut && e == et) ? v[u][e] : sel;
      const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), owner));
      float m = v[0][0];
#pragma unroll
      for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
        for (int e = 0; e < VEC; ++e) m = fmaximum(m, v[u][e]);
      float wm = m;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wm = fmaximum(wm, __shfl_xor(wm, o, kWave));
      if (__builtin_expect(wm != wm, 0)) {  // NaN in the row: exact torch.argmax semantics
        correct = row_argmax_exact<KIND>(rp, C, lane) == t;
      } else if (!t_ok || xt != wm) {
        correct = false;
      } else {  // the target holds the max: correct iff no earlier column ties it
        int idx = 0x7fffffff;
#pragma unroll
        for (int u = kChunkLoads - 1; u >= 0; --u)
#pragma unroll
          for (int e = VEC - 1; e >= 0; --e)
            idx = (v[u][e] == wm) ? (u * STEP + lane * VEC + e) : idx;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) idx = min(idx, __shfl_xor(idx, o, kWave));
        correct = idx == t;
      }
    } else if constexpr (!TOPK) {
      t = load_target(a.target, a.tg_dt, row);
      float bv = -__builtin_huge_valf();
      int bi = 0x7fffffff;
      bool saw_nan = false;
      // rows longer than one chunk: the next chunk's loads are issued before this chunk is
      // reduced (two chunks in flight; v1 waited one full round trip per chunk)
      float nx[kChunkLoads][VEC];
      load_chunk<KIND, VEC, UNAL>(rp, 0, C, lane, nx);
      for (int base = 0; base < C; base += CHUNK) {
        float v[kChunkLoads][VEC];
#pragma unroll
        for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[u][e] = nx[u][e];
        if (base + CHUNK < C) load_chunk<KIND, VEC, UNAL>(rp, base + CHUNK, C, lane, nx);
        finish_chunk<VEC, UNAL>(v, base, C, lane);
        // phase 1: NaN-propagating lane max; phase 2: first column holding it
        float m = v[0][0];
#pragma unroll
        for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
          for (int e = 0; e < VEC; ++e) m = fmaximum(m, v[u][e]);
        int idx = 0x7fffffff;
#pragma unroll
        for (int u = kChunkLoads - 1; u >= 0; --u)
#pragma unroll
          for (int e = VEC - 1; e >= 0; --e)
            idx = (v[u][e] == m) ? (base + u * STEP + lane * VEC + e) : idx;
        saw_nan |= (m != m);
        // columns of this chunk are all larger than earlier chunks': strict > keeps the first
        if (m > bv || bi == 0x7fffffff) {
          bv = m;
          bi = idx;
        }
      }
      // cross-lane: max value, then smallest index among the lanes holding it
      float wm = bv;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) wm = fmaximum(wm, __shfl_xor(wm, o, kWave));
      int widx = (bv == wm) ? bi : 0x7fffffff;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) widx = min(widx, __shfl_xor(widx, o, kWave));
      if (__builtin_expect(__any(saw_nan), 0)) widx = row_argmax_exact<KIND>(rp, C, lane);
      pred = widx;
      correct = pred == t;
    } else {
      t = load_target(a.target, a.tg_dt, row);
      const bool t_ok = t >= 0 && t < C;
      const float xt = t_ok ? load_one<KIND>(rp, t) : __builtin_nanf("");
      int cnt = 0;
      float nx[kChunkLoads][VEC];
      load_chunk<KIND, VEC, UNAL>(rp, 0, C, lane, nx);
      for (int base = 0; base < C; base += CHUNK) {
        float v[kChunkLoads][VEC];
#pragma unroll
        for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
          for (int e = 0; e < VEC; ++e) v[u][e] = nx[u][e];
        if (base + CHUNK < C) load_chunk<KIND, VEC, UNAL>(rp, base + CHUNK, C, lane, nx);
        finish_chunk<VEC, UNAL>(v, base, C, lane);
#pragma unroll
        for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
          for (int e = 0; e < VEC; ++e) cnt += v[u][e] > xt;
      }
      cnt = wave_sum(cnt);
      correct = t_ok && cnt < a.k;
    }
    if (lane == 0) {
      correct_acc += correct;
      rows_acc += 1;
      row_hist(h, a.num_classes, t, pred, correct, a.err, a.check_target, a.err_max);
    }
  }
  block_micro(a, correct_acc, rows_acc);
}


// ---------------------------------------------------------------- micro accuracy (k = 1)
// The north-star update (MulticlassAccuracy micro, bs 8192 x C 1000): one wave per row, the
// row's 4 x 16-B loads per lane and the target's scalar load all in flight together.  What the
// A/B harness showed (csrc/bench/k1_v3.hip, profiles/k1_v3_ab_r3.md): the per-row work runs
// after the row's LAST load lands, and the loads of all 8192 waves land near the end of the
// stream, so every VALU instruction per row sits on the kernel's tail.  This body keeps it to
// ~40: a v_maximum3 tree over the lane's values, a DPP wave max (quad perms + half/full row
// mirrors, 4 readlanes) in place of six ds_bpermute round trips, and the target's own score
// by ONE uniform register-indexed move (s_set_gpr_idx_on + v_mov from the owner lane's
// register, then a readlane) in place of a select per element.  Only rows whose target holds
// the max count the other columns equal to it (ballots + scalar popcounts); a second holder
// or a NaN row takes the exact torch.argmax path.  Lanes past C re-read the row's first
// columns (clamped addresses), which cannot change the max and are masked out of the count.
// Replaces reference accuracy.py:260-278 (argmax -> eq -> long -> sum, plus a host tensor).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}

__device__ __forceinline__ float wave_max_dpp(float x) {  // NaN-propagating, wave-uniform
  x = fmaximum(x, dpp_f32<0xB1>(x));   // quad_perm [1,0,3,2]
  x = fmaximum(x, dpp_f32<0x4E>(x));   // quad_perm [2,3,0,1]
  x = fmaximum(x, dpp_f32<0x141>(x));  // row_half_mirror
  x = fmaximum(x, dpp_f32<0x140>(x));  // row_mirror: every lane holds its 16-lane row max
  const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 0));
  const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 16));
  const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 32));
  const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 48));
  return fmaximum(fmaximum(r0, r1), fmaximum(r2, r3));
}

template <int NV>
struct RowVals;
template <>
struct RowVals<16> {
  typedef float type __attribute__((ext_vector_type(16)));
};
template <>
struct RowVals<32> {
  typedef float type __attribute__((ext_vector_type(32)));
};

// The micro rows of one wave (grid-stride over rows): correct / row counts on lane 0.
// KIND 0: f32 (4 floats per 16-B load), 1: bf16, 2: f16 (8 per load); TGT: int64_t / int32_t
template <int KIND, typename TGT, bool UNAL = false>
__device__ __forceinline__ void micro_rows(const void* __restrict__ input, const TGT* __restrict__ target, int64_t n,
                                           int C, int64_t row_stride, uint32_t& correct_acc, uint32_t& rows_acc) {
  constexpr int VEC = KIND == 0 ? 4 : 8;
  constexpr int NV = kChunkLoads * VEC;  // values per lane
  constexpr int STEP = kWave * VEC;      // columns per wave-load
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  typedef typename RowVals<NV>::type vec_t;
  const int lane = lane_id();
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerBlock;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWavesPerBlock + wave_id(); row < n; row += nwaves) {
    const char* rp = static_cast<const char*>(input) + row * row_stride * ELSIZE;
    float f[kChunkLoads][VEC];
#pragma unroll
    for (int u = 0; u < kChunkLoads; ++u) load_row_vec<KIND, VEC, UNAL>(rp, u * STEP + lane * VEC, C, f[u]);
    const int64_t t = target[row];
    if constexpr (UNAL) unal_fix_tail<kChunkLoads>(f, 0, C, lane);
    vec_t v;
#pragma unroll
    for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
      for (int e = 0; e < VEC; ++e) v[u * VEC + e] = f[u][e];
    float m = fmaximum(v[0], v[1]);
#pragma unroll
    for (int e = 2; e < NV; ++e) m = fmaximum(m, v[e]);
    const float wm = wave_max_dpp(m);
    bool correct = false;
    if (__builtin_expect(wm != wm, 0)) {  // NaN in the row: exact torch.argmax semantics
      correct = row_argmax_exact<KIND>(rp, C, lane) == t;
    } else if (t >= 0 && t < C) {
      const int tu = static_cast<int>(t);
      const float sel = v[(tu / STEP) * VEC + (tu % VEC)];  // uniform index: one indexed move
      const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), (tu % STEP) / VEC));
      if (xt == wm) {  // the target holds the max: correct iff it is the only column that does
        int cnt = 0;
#pragma unroll
        for (int u = 0; u < kChunkLoads; ++u) {
          const int valid = min(max((C - u * STEP + VEC - 1) / VEC, 0), kWave);
          const uint64_t lanes = valid >= kWave ? ~0ull : ((1ull << valid) - 1);
#pragma unroll
          for (int e = 0; e < VEC; ++e) cnt += __builtin_popcountll(__ballot(v[u * VEC + e] == wm) & lanes);
        }
        correct = cnt == 1 || row_argmax_exact<KIND>(rp, C, lane) == t;
      }
    }
    if (lane == 0) {
      correct_acc += correct;
      rows_acc += 1;
    }
  }
}

template <int KIND, typename TGT, bool UNAL>
__global__ __launch_bounds__(kBlock) void cls_micro_kernel(ClsCountsArgs a) {
  uint32_t correct_acc = 0, rows_acc = 0;
  micro_rows<KIND, TGT, UNAL>(a.input, static_cast<const TGT*>(a.target), a.n, static_cast<int>(a.c), a.row_stride,
                        correct_acc, rows_acc);
  block_micro(a, correct_acc, rows_acc);
}

// The north-star launch: pending-cell epilogue and a compact kernel-argument block.  Each
// wave's first instructions wait on its kernel arguments, and with ClsCountsArgs (~200 B) and
// in-kernel lane-mask arithmetic the generated code issued the kernarg loads in two dependent
// rounds and ~60 scalar instructions before the first row load.  Here everything the row
// loads need sits in one 56-byte block (one scalar round trip) and the row test needs no lane
// masks (profiles/k1_floor_r4*.txt).
struct MicroPendArgs {
  const void* input;
  const void* target;
  unsigned long long* pend;
  float* total;
  int64_t n;
  int64_t row_stride;
  int32_t c;
  int32_t pad;
};

template <int KIND, typename TGT, bool UNAL>
__device__ __forceinline__ bool micro_row(const MicroPendArgs& a, const char* __restrict__ rp, int64_t t, int lane) {
  constexpr int VEC = KIND == 0 ? 4 : 8;
  constexpr int NV = kChunkLoads * VEC;
  constexpr int STEP = kWave * VEC;
  typedef typename RowVals<NV>::type vec_t;
  const int C = a.c;
  float f[kChunkLoads][VEC];
#pragma unroll
  for (int u = 0; u < kChunkLoads; ++u) load_row_vec<KIND, VEC, UNAL>(rp, u * STEP + lane * VEC, C, f[u]);
  if constexpr (UNAL) unal_fix_tail<kChunkLoads>(f, 0, C, lane);
  vec_t v;
#pragma unroll
  for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
    for (int e = 0; e < VEC; ++e) v[u * VEC + e] = f[u][e];
  // compare-only: no wave-wide max.  A column beats the target under torch.argmax's order if
  // it is larger, or equal at a lower index (NaN rows take the exact path).  Lanes past C hold
  // clamped copies of columns 0..VEC-1: real values of the row, so they cannot create a larger
  // value, and their nominal column (>= C > t) keeps them out of the tie test.
  float m = fmaximum(v[0], v[1]);
#pragma unroll
  for (int e = 2; e < NV; ++e) m = fmaximum(m, v[e]);
  if (__builtin_expect(__ballot(m != m) != 0, 0)) return row_argmax_exact<KIND>(rp, C, lane) == t;  // NaN
  if (!(t >= 0 && t < C)) return false;
  const int tu = static_cast<int>(t);
  const float sel = v[(tu / STEP) * VEC + (tu % VEC)];  // uniform index: one indexed move
  const float xt = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sel), (tu % STEP) / VEC));
  if (__ballot(m > xt) != 0) return false;  // a larger column somewhere: the common incorrect row
  // the target holds the row max: correct iff no column before it ties it (first index wins)
  bool tie = false;
#pragma unroll
  for (int u = 0; u < kChunkLoads; ++u)
#pragma unroll
    for (int e = 0; e < VEC; ++e) tie |= (v[u * VEC + e] == xt) & (u * STEP + lane * VEC + e < tu);  // no branches
  return __ballot(tie) == 0;
}

template <int KIND, typename TGT, int WPB, bool UNAL>
__global__ __launch_bounds__(WPB * kWave) void cls_micro_pend_kernel(MicroPendArgs a) {
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  const int lane = lane_id();
  const int64_t nwaves = static_cast<int64_t>(gridDim.x) * WPB;
  // the wave's first row is loaded unconditionally (clamped to the last row), so nothing
  // branches on `n` before the loads and every kernel argument arrives in one scalar round trip
  const int64_t row0 = static_cast<int64_t>(blockIdx.x) * WPB + wave_id();
  const int64_t r0 = row0 < a.n ? row0 : a.n - 1;  // the launcher guarantees n >= 1
  const bool c0 = micro_row<KIND, TGT, UNAL>(a, static_cast<const char*>(a.input) + r0 * a.row_stride * ELSIZE,
                                       static_cast<const TGT*>(a.target)[r0], lane);
  uint32_t correct_acc = (row0 < a.n && c0) ? 1u : 0u;
  for (int64_t row = row0 + nwaves; row < a.n; row += nwaves) {
    const char* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELSIZE;
    correct_acc += micro_row<KIND, TGT, UNAL>(a, rp, static_cast<const TGT*>(a.target)[row], lane);
  }
  // deferred fold: one no-return atomic per wave into one of 64 pending cells, no LDS, no
  // block barrier, no returning atomic on the kernel's tail (the fold's ~0.6 us + the block
  // reduction's ~0.45 us in the A/B harness); the metric folds the cells at compute / sync
  if (lane == 0 && correct_acc)
    atomicAdd(a.pend + ((blockIdx.x * WPB + wave_id()) % kPendCells) * kPendStride,
              static_cast<unsigned long long>(correct_acc));
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.total) atomicAdd(a.total, static_cast<float>(a.n));
}

__global__ __launch_bounds__(kWave) void micro_finish_kernel(unsigned long long* pend, float* correct,
                                                             const float* total, float* out) {
  unsigned long long* cell = pend + threadIdx.x * kPendStride;
  const unsigned long long s = wave_sum(*cell);
  *cell = 0ull;
  if (threadIdx.x == 0) {
    const float c = correct[0] + static_cast<float>(s);
    correct[0] = c;
    if (out) out[0] = c / total[0];
  }
}

template <int KIND, int VEC, bool TOPK, bool PRED = true, bool UNAL = false>
__global__ __launch_bounds__(kBlock) void cls_wide_kernel(ClsCountsArgs a) {
  // (amdgpu_waves_per_eu(8, 8) on the f32 kernels - 64 VGPRs, every row of an 8192-row batch
  // resident at once - measured slower: 8.9 vs 7.8 us per 8192 x 1000 update)
  cls_wide_body<KIND, VEC, TOPK, PRED, UNAL>(a);
}

// Narrow rows (C <= 32): one thread per row, class histograms privatised in LDS.
template <int KIND, bool TOPK>
__global__ __launch_bounds__(kBlock) void cls_narrow_kernel(ClsCountsArgs a) {
  constexpr int ELSIZE = KIND == 0 ? 4 : 2;
  __shared__ float s_correct[kNarrowMaxC], s_label[kNarrowMaxC], s_pred[kNarrowMaxC];
  __shared__ float s_fp[kNarrowMaxC];
  __shared__ float s_conf[kNarrowMaxC * kNarrowMaxC];
  const int C = static_cast<int>(a.c);
  for (int i = threadIdx.x; i < C * C; i += kBlock) s_conf[i] = 0.f;
  if (threadIdx.x < kNarrowMaxC) {
    s_correct[threadIdx.x] = 0.f;
    s_label[threadIdx.x] = 0.f;
    s_pred[threadIdx.x] = 0.f;
    s_fp[threadIdx.x] = 0.f;
  }
  __syncthreads();
  const Hist lh{a.cls_correct ? s_correct : nullptr, a.cls_label ? s_label : nullptr,
                a.cls_pred ? s_pred : nullptr, a.cls_fp ? s_fp : nullptr,
                a.confusion ? s_conf : nullptr};
  uint32_t correct_acc = 0, rows_acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; row < a.n;
       row += stride) {
    const void* rp = static_cast<const char*>(a.input) + row * a.row_stride * ELSIZE;
    const int64_t t = load_target(a.target, a.tg_dt, row);
    bool correct;
    int64_t pred = -1;
    if constexpr (!TOPK) {
      float bv = -__builtin_huge_valf();
      int bi = 0x7fffffff;
      for (int c = 0; c < C; ++c) {
        const float v = load_one<KIND>(rp, c);
        if (argmax_better(v, c, bv, bi)) {
          bv = v;
          bi = c;
        }
      }
      pred = bi;
      correct = pred == t;
    } else {
      const bool t_ok = t >= 0 && t < C;
      const float xt = t_ok ? load_one<KIND>(rp, t) : __builtin_nanf("");
      int cnt = 0;
      for (int c = 0; c < C; ++c) cnt += load_one<KIND>(rp, c) > xt;
      correct = t_ok && cnt < a.k;
    }
    correct_acc += correct;
    rows_acc += 1;
    row_hist(lh, C, t, pred, correct, a.err, a.check_target, a.err_max);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C; i += kBlock) {
    if (a.cls_correct && s_correct[i] != 0.f) atomicAdd(a.cls_correct + i, s_correct[i]);
    if (a.cls_label && s_label[i] != 0.f) atomicAdd(a.cls_label + i, s_label[i]);
    if (a.cls_pred && s_pred[i] != 0.f) atomicAdd(a.cls_pred + i, s_pred[i]);
    if (a.cls_fp && s_fp[i] != 0.f) atomicAdd(a.cls_fp + i, s_fp[i]);
  }
  if (a.confusion)
    for (int i = threadIdx.x; i < C * C; i += kBlock)
      if (s_conf[i] != 0.f) atomicAdd(a.confusion + i, s_conf[i]);
  block_micro(a, correct_acc, rows_acc);
}

// 1-D integer label predictions: elementwise compare + histograms.
__global__ __launch_bounds__(kBlock) void cls_labels_kernel(ClsCountsArgs a) {
  const Hist h{a.cls_correct, a.cls_label, a.cls_pred, a.cls_fp, a.confusion};
  uint32_t correct_acc = 0, rows_acc = 0;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride) {
    const int64_t p = load_as_i64(a.input, a.in_dt, i);
    const int64_t t = load_target(a.target, a.tg_dt, i);
    const bool correct = p == t;
    correct_acc += correct;
    rows_acc += 1;
    row_hist(h, a.num_classes, t, p, correct, a.err, a.check_target, a.err_max);
  }
  block_micro(a, correct_acc, rows_acc);
}

// Binary: thresholded scores vs targets -> [tp, fp, tn, fn] (+ optional weights).
__global__ __launch_bounds__(kBlock) void binary_counts_kernel(BinaryCountsArgs a) {
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBlock;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < a.n; i += stride) {
    const float x = load_as_f32(a.input, a.in_dt, i);
    const double t = load_as_f64(a.target, a.tg_dt, i);
    const float w = a.weight ? load_as_f32(a.weight, a.w_dt, i) : 1.f;
    const bool pos = !(x < a.threshold);
    const bool t1 = t == 1.0, t0 = t == 0.0;
    const float other = a.strict_binary ? 0.f : w;
    if (pos) {
      acc[0] += t1 ? w : 0.f;
      acc[1] += t0 ? w : (t1 ? 0.f : other);
    } else {
      acc[2] += t0 ? w : 0.f;
      acc[3] += t1 ? w : (t0 ? 0.f : other);
    }
  }
  __shared__ float lds[4][kWavesPerBlock];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float s = wave_sum(acc[j]);
    if (lane_id() == 0) lds[j][threadIdx.x >> 6] = s;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kWavesPerBlock; ++w) s += lds[threadIdx.x][w];
    float* dst = a.out[threadIdx.x];
    if (dst && s != 0.f) atomicAdd(dst, s);
    float* dst2 = a.out2[threadIdx.x];
    if (dst2 && s != 0.f) atomicAdd(dst2, s);
  }
  if (threadIdx.x == 0 && blockIdx.x == 0 && a.total) atomicAdd(a.total, static_cast<float>(a.n));
}

template <int KIND, int VEC, bool UNAL = false>
void launch_wide(const ClsCountsArgs& a, int grid, hipStream_t s) {
  constexpr int kChunkCols = kWave * VEC * kChunkLoads;
  const bool pred_free = a.cls_pred == nullptr && a.cls_fp == nullptr && a.confusion == nullptr &&
                         a.c <= kChunkCols;
  // pure micro counts (no class histograms, no label validation) with 64/32-bit targets
  // (TORCHEVAL_AMD_K1_MICRO=0 keeps the general kernel: A/B switch for profiling)
  static const bool micro_on = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K1_MICRO");
    return e == nullptr || std::atoi(e) != 0;
  }();
  const bool micro_only = micro_on && pred_free && VEC > 1 && a.k == 1 && a.cls_correct == nullptr &&
                          a.cls_label == nullptr && a.err == nullptr && a.err_max == nullptr && !a.check_target;
  if (micro_only && a.pend && (a.tg_dt == DType::i64 || a.tg_dt == DType::i32)) {
    const MicroPendArgs m{a.input, a.target, a.pend, a.micro_total, a.n, a.row_stride, static_cast<int32_t>(a.c), 0};
    // 512-thread workgroups (8 waves, still one wave per row, 1024 blocks): the driver command
    // 144.9k vs 142.7k updates/s with 4-wave workgroups, interleaved on one box, and the floor
    // harness 6.23 vs 6.30 us per launch (profiles/k1_wpb_ab_r4.txt).  TORCHEVAL_AMD_K1_WPB=4
    // selects the 256-thread form.
    static const int wpb = [] {
      const char* e = std::getenv("TORCHEVAL_AMD_K1_WPB");
      return (e && std::atoi(e) == 4) ? 4 : 8;
    }();
    if (wpb == 8) {
      const int g8 = stream_grid(a.n, 8, a.max_blocks > 0 ? (a.max_blocks + 1) / 2 : 1024);
      if (a.tg_dt == DType::i64)
        hipLaunchKernelGGL((cls_micro_pend_kernel<KIND, int64_t, 8, UNAL>), dim3(g8), dim3(8 * kWave), 0, s, m);
      else
        hipLaunchKernelGGL((cls_micro_pend_kernel<KIND, int32_t, 8, UNAL>), dim3(g8), dim3(8 * kWave), 0, s, m);
      return;
    }
    if (a.tg_dt == DType::i64)
      hipLaunchKernelGGL((cls_micro_pend_kernel<KIND, int64_t, kWavesPerBlock, UNAL>), dim3(grid), dim3(kBlock), 0, s, m);
    else
      hipLaunchKernelGGL((cls_micro_pend_kernel<KIND, int32_t, kWavesPerBlock, UNAL>), dim3(grid), dim3(kBlock), 0, s, m);
    return;
  }
  if (micro_only && a.tg_dt == DType::i64) {
    hipLaunchKernelGGL((cls_micro_kernel<KIND, int64_t, UNAL>), dim3(grid), dim3(kBlock), 0, s, a);
    return;
  }
  if (micro_only && a.tg_dt == DType::i32) {
    hipLaunchKernelGGL((cls_micro_kernel<KIND, int32_t, UNAL>), dim3(grid), dim3(kBlock), 0, s, a);
    return;
  }
  if (a.k > 1)
    hipLaunchKernelGGL((cls_wide_kernel<KIND, VEC, true, true, UNAL>), dim3(grid), dim3(kBlock), 0, s, a);
  else if (pred_free)
    hipLaunchKernelGGL((cls_wide_kernel<KIND, VEC, false, false, UNAL>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((cls_wide_kernel<KIND, VEC, false, true, UNAL>), dim3(grid), dim3(kBlock), 0, s, a);
}

template <int KIND>
void launch_narrow(const ClsCountsArgs& a, int grid, hipStream_t s) {
  if (a.k > 1)
    hipLaunchKernelGGL((cls_narrow_kernel<KIND, true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((cls_narrow_kernel<KIND, false>), dim3(grid), dim3(kBlock), 0, s, a);
}

}  // namespace

int launch_cls_counts(const ClsCountsArgs& a, hipStream_t stream) {
  if (a.n <= 0) return 0;
  if (a.c > 0) {
    const uintptr_t base = reinterpret_cast<uintptr_t>(a.input);
    const int kind = a.in_dt == DType::f32 ? 0 : a.in_dt == DType::bf16 ? 1 : a.in_dt == DType::f16 ? 2 : -1;
    if (kind < 0) return -1;
    if (a.c <= kNarrowMaxC) {
      const int cap = a.max_blocks > 0 ? a.max_blocks : 512;
      const int grid = stream_grid(a.n, kBlock, cap);
      if (kind == 0) launch_narrow<0>(a, grid, stream);
      else if (kind == 1) launch_narrow<1>(a, grid, stream);
      else launch_narrow<2>(a, grid, stream);
    } else {
      // one wave per row up to 8 waves/SIMD residency (2048 blocks of 4 waves)
      const int cap = a.max_blocks > 0 ? a.max_blocks : 2048;
      const int grid = stream_grid(a.n, kWavesPerBlock, cap);
      const int vw = kind == 0 ? 4 : 8;
      const bool vec = (a.c % vw == 0) && (a.row_stride % vw == 0) && (base % 16 == 0);
      // f32 rows of any width / alignment keep 16-B loads (UNAL); 16-bit rows that are not
      // 16-B aligned take the scalar form
      if (kind == 0) vec ? launch_wide<0, 4>(a, grid, stream) : launch_wide<0, 4, true>(a, grid, stream);
      else if (kind == 1) vec ? launch_wide<1, 8>(a, grid, stream) : launch_wide<1, 1>(a, grid, stream);
      else vec ? launch_wide<2, 8>(a, grid, stream) : launch_wide<2, 1>(a, grid, stream);
    }
  } else {
    const int cap = a.max_blocks > 0 ? a.max_blocks : 1024;
    const int grid = stream_grid(a.n, kBlock, cap);
    hipLaunchKernelGGL(cls_labels_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  }
  return static_cast<int>(hipGetLastError());
}

int launch_micro_finish(unsigned long long* pend, float* correct, const float* total, float* out,
                        hipStream_t stream) {
  hipLaunchKernelGGL(micro_finish_kernel, dim3(1), dim3(kPendCells), 0, stream, pend, correct, total, out);
  return static_cast<int>(hipGetLastError());
}

int launch_binary_counts(const BinaryCountsArgs& a, hipStream_t stream) {
  if (a.n <= 0) return 0;
  const int cap = a.max_blocks > 0 ? a.max_blocks : 256;
  const int grid = stream_grid(a.n, kBlock * 4, cap);
  hipLaunchKernelGGL(binary_counts_kernel, dim3(grid), dim3(kBlock), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
