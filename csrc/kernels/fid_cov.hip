// K8: FID covariance update C += A^T A, s += colsum(A) on FP32 MFMA.
//
// Replaces fid.py:120-127 (a full D x D x B SGEMM plus a separate column sum) with one
// symmetric rank-k update that computes only the upper-triangle tiles (half the FLOPs),
// mirrors them, and fuses the column sums into the diagonal tiles.
//
// gfx950 mapping, v5.  Round-1's v2 (64 x 64 tiles, 4 waves each owning one 32 x 32 block)
// ran 82 us at 1000 x 2048 with SQ_VALU_MFMA_BUSY ~33 %: one 32 x 32 accumulator per wave
// means two LDS operand reads per MFMA, and D = 2048 gives 528 tiles for 256 CUs (16 CUs run a
// third tile).  v5 (profiles/k8_fid_cov_r2.md has the measured ladder):
//  * 96 x 96 output tiles: D = 2048 -> T = 22 tile rows -> 253 upper-triangle tiles, one
//    workgroup per CU in a single wave of blocks (no quantisation tail).
//  * 8 waves = 2 per SIMD: wave w owns the 48 x 48 quadrant w & 3 as 3 x 3 blocks of
//    v_mfma_f32_16x16x4_f32 (exact FP32 products, 9 independent 4-register accumulators), and
//    the k-steps of parity w >> 2 (in-block 2-way split of K, summed through LDS at the end).
//    Per 4-k step a wave reads 3 A + 3 B operands (one ds_read_b32 each) for 9 MFMAs - 3x the
//    operand reuse of v2 - with the next step's reads pinned ahead of this step's MFMAs
//    (sched_group_barrier), and the SIMD's second wave covers what LDS latency is left.
//  * staging by LDS-DMA (global_load_lds_dwordx4): 64 rows of ``act`` per stage, three LDS
//    stages (144 KB), two stages in flight, counted vmcnt + raw s_barrier.  The operand image
//    is lane-linear with each row's columns rotated by 0/16/32/48 floats (rotation applied to
//    the per-lane source address), so the 4 rows one ds_read_b32 touches hit 4 disjoint
//    16-bank groups.  Rows past the K range / columns past the width read a zero line.
//  * diagonal tiles: quadrant (1, 0) is quadrant (0, 1) transposed, so its two waves sum the
//    tile's columns (the fused colsum) instead of running MFMAs, and the epilogue mirrors it -
//    the diagonal blocks do no more MFMA-pipe work than the others (a colsum pass on top of
//    the MFMAs made them the grid's critical path: 112 vs 139 TF/s in the no-load A/B).
//  * XCD-aware block order: the grid is padded to a multiple of 8 and block b is remapped to
//    item (b % 8) * (nb / 8) + b / 8, so each XCD owns a contiguous run of row-major tiles
//    that share their row panel in that XCD's L2.
//  * split-K for small D or huge N (items = tiles x split): each item accumulates a K-range
//    and writes its raw 96 x 96 partial (plus diagonal column-sum partials) to a workspace;
//    ``fid_fixup_kernel`` sums the partials in a fixed order and does the read-modify-write
//    of C (and the mirror), so the result is deterministic for a given split.  With one item
//    per tile (split = 1, the D = 2048 case) the epilogue RMWs C directly from LDS.
//  * the epilogue stages the tile in LDS (96 x 97, conflict-free transposed read) and updates
//    C[I, J] and the mirrored C[J, I] with coalesced rows; one block owns each output tile, so
//    no atomics anywhere.
// v6 (round 3): the products run on bf16 MFMA (v_mfma_f32_16x16x32_bf16, 16x the FP32 MFMA
// rate) through an exact three-way bf16 split of each FP32 operand (split3, six products per
// pair), each 64-row stage summed into fresh accumulators that are added to the running ones
// on the VALU - more accurate than the FP32-MFMA form (max error vs fp64 at 50000 x 2048:
// 1.0e-6 vs 7.5e-6 of max |C|).  The block splits every staged element once (kMode 2): each
// thread loads 8-row column pieces of the next stage with raw buffer loads (out-of-range
// offsets read 0), splits them while this stage's MFMAs issue (one basic block per stage,
// sched_group_barrier interleave) and stores the planes in fragment order, so a fragment is
// one ds_read_b128.  Measured and dropped: a second register stage (loads two stages ahead)
// was 0-5 % slower; the loop is then bound by the per-CU load rate (48 KB per stage per CU,
// ~10 B/cycle/CU; without the loads the loop runs 24 % faster).  1000 x 2048: 44 us (FP32 form 54 us, hipBLASLt GEMM 76 us); 8192 x 2048:
// 250 us (326, GEMM 481) - profiles/k8_split_bf16_sweep_r3.json.  The per-wave split (kMode 1,
// each element split by two waves, VALU-bound) and the FP32 form (kMode 0) stay selectable.
// Rejected in v2 (kept for the record, MI355X, 1000 x 2048): in-block split-K with 2 x 2
// register blocking of 32 x 32 MFMAs (118 us, 176 VGPRs), BK = 64 (104 us), 8 x 8 super-tile
// enumeration (86 us), 2-4 stage register prefetch (83-84 us), k-contiguous LDS operands
// with ds_read_b128 (89.6 us).
#include <algorithm>
#include <cstdlib>

#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

#ifndef TEA_K8_SCHED
#define TEA_K8_SCHED 1
#endif

constexpr int kT = 96;         // output tile
constexpr int kBK = 64;        // rows of act per stage
constexpr int kThreads = 512;  // 8 waves
constexpr int kFixThreads = 256;
constexpr int kStage = kBK * kT;          // floats per operand per stage (lane-linear image)
constexpr int kSegs = kT / 4;             // float4 slots per image row (24)
constexpr int kGlds = kStage / 4 / kThreads;  // global_load_lds_dwordx4 per thread per operand (3)
constexpr int kCPad = kT + 1;
constexpr int kBufs = 3;                    // LDS stages: two LDS-DMA stages in flight
constexpr int kSmemBytes = 2 * kBufs * kStage * 4;  // 144 KB: one block per CU
static_assert(kStage % (4 * kThreads) == 0, "stage must split evenly into wave-wide LDS-DMA pieces");
static_assert(kT * kCPad + 8 * kT <= 2 * kBufs * kStage, "epilogue tile + column sums must fit");

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// Exact three-way bf16 split of 8 FP32 values into the packed fragments of a
// v_mfma_f32_16x16x32_bf16 operand: x = x1 + x2 + x3 with x1 = x truncated to its top 8
// significand bits, x2 = the next 8 of x - x1, x3 = x - x1 - x2 (<= 8 bits, so exact in bf16).
// Both differences are exact (the subtrahend shares the minuend's leading bits).  Element 2q of
// a fragment is the low half of dword q, 2q + 1 the high half (v_perm_b32 of the two upper halves).
__device__ __forceinline__ void split3(const float (&v)[8], u32x4& p1, u32x4& p2, u32x4& p3) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned u0 = __float_as_uint(v[2 * q]), u1 = __float_as_uint(v[2 * q + 1]);
    const float r0 = v[2 * q] - __uint_as_float(u0 & 0xffff0000u);
    const float r1 = v[2 * q + 1] - __uint_as_float(u1 & 0xffff0000u);
    const unsigned w0 = __float_as_uint(r0), w1 = __float_as_uint(r1);
    const float s0 = r0 - __uint_as_float(w0 & 0xffff0000u);
    const float s1 = r1 - __uint_as_float(w1 & 0xffff0000u);
    p1[q] = __builtin_amdgcn_perm(u1, u0, 0x07060302u);
    p2[q] = __builtin_amdgcn_perm(w1, w0, 0x07060302u);
    p3[q] = __builtin_amdgcn_perm(__float_as_uint(s1), __float_as_uint(s0), 0x07060302u);
  }
}

__device__ __forceinline__ f32x4 mfma_bf16(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Operand image of one stage: LDS row r (= sample b0 + r) holds the tile's 96 columns rotated
// by rot(r) floats.  The four rows one ds_read_b32 touches (r = 4q + lk) then start at banks
// {0, 48, 32, 16} + col (mod 64) - distinct mod 32 within each half-wave too (a rotation of
// 16 on odd row pairs only gave {0, 32, 16, 48}: 3.8 bank-conflict cycles per LDS instruction
// measured, as lanes 0-31 then share banks mod 32) - and the image stays lane-linear for
// global_load_lds (whose LDS destination is base + lane x 16 B): the rotation is applied to
// the per-lane SOURCE address instead.
__device__ __forceinline__ int rot(int r) { return (r & 1) * 16 + ((r >> 1) & 1) * 32; }

__device__ __forceinline__ void tile_coords(int t, int T, int& ti, int& tj) {
  // t enumerates the upper triangle (ti <= tj) row by row
  int row = 0, rem = t;
  while (rem >= T - row) {
    rem -= T - row;
    ++row;
  }
  ti = row;
  tj = row + rem;
}

// kMode 1 and 2: the products run on bf16 MFMA through the exact three-way split (split3) - six
// products per operand pair (x1y1, x1y2, x2y1, x2y2, x1y3, x3y1; the dropped x2y3, x3y2, x3y3
// are below 2^-23 |xy|), i.e. FP32-level products at 6/16 of the FP32 MFMA pipe time.
//  * kMode 2 (default): the block splits each staged element once.  Every thread loads whole
//    8-row column pieces of the next stage into registers (global loads, one stage ahead),
//    splits them and writes the three bf16 planes to LDS in MFMA fragment order (k-contiguous:
//    plane[k / 8][column][k % 8]), so a fragment is one ds_read_b128 and the split's VALU is
//    spread over all 8 waves with no duplication.
//  * kMode 1: LDS-DMA fp32 staging as in kMode 0; each wave splits the operands it reads
//    (every element is split by two waves: the VALU is the limit).
//  * kMode 0: exact FP32 products on v_mfma_f32_16x16x4_f32.
template <int kMode>
__global__ __launch_bounds__(kThreads) void fid_syrk_kernel(FidCovArgs a, int T, int tiles, int items, int64_t chunk) {
  const int nb = gridDim.x;
  int item = blockIdx.x;
  if (nb % 8 == 0) item = (item % 8) * (nb / 8) + item / 8;
  if (item >= items) return;  // grid padding (whole block: no barrier is skipped halfway)
  const int ks = item / tiles, tile = item % tiles;
  int ti, tj;
  tile_coords(tile, T, ti, tj);
  const int64_t I0 = static_cast<int64_t>(ti) * kT, J0 = static_cast<int64_t>(tj) * kT;
  const bool diag = ti == tj;
  const int64_t k0 = ks * chunk;
  const int64_t k1 = min(a.n, k0 + chunk);

  extern __shared__ __attribute__((aligned(16))) float smem[];  // kSmemBytes, the only LDS object
  float* sI = smem;                   // [kBufs][kBK][kT] rotated images
  float* sJ = smem + kBufs * kStage;  // [kBufs][kBK][kT]
  const float* sJr = diag ? sI : sJ;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int quad = w & 3, par = w >> 2;  // output quadrant, k-step parity
  const int wr = quad >> 1, wc = quad & 1;
  const int li = lane & 15, lk = lane >> 4;

  f32x4 acc[3][3];
#pragma unroll
  for (int m = 0; m < 3; ++m)
#pragma unroll
    for (int n = 0; n < 3; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- staging: wave w's piece q covers image slots [(3w + q) * 64, +64), lane = slot
  int prow[kGlds];
  const float* srcI[kGlds];
  const float* srcJ[kGlds];
  bool okI[kGlds], okJ[kGlds];
#pragma unroll
  for (int q = 0; q < kGlds; ++q) {
    const int p = (w * kGlds + q) * 64 + lane;
    const int r = p / kSegs;
    const int c = (4 * (p % kSegs) - rot(r) + kT) % kT;  // source column of this slot
    prow[q] = r;
    okI[q] = I0 + c < a.ld;
    okJ[q] = J0 + c < a.ld;
    srcI[q] = a.act + static_cast<int64_t>(r) * a.row_stride + I0 + c;
    srcJ[q] = a.act + static_cast<int64_t>(r) * a.row_stride + J0 + c;
  }
  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  // rows past the K range and columns past the (4-padded) width read a zero line instead
  auto issue = [&](int buf, int64_t b0) {
    const int64_t shift = b0 * a.row_stride;
    const int64_t rows_left = k1 - b0;
#pragma unroll
    for (int q = 0; q < kGlds; ++q) {
      const bool vr = prow[q] < rows_left;
      const float* gi = vr && okI[q] ? srcI[q] + shift : a.zeros;
      __builtin_amdgcn_global_load_lds((gptr_t)(gi),
                                       (lptr_t)(sI + buf * kStage + (w * kGlds + q) * 256), 16, 0, 0);
      if (!diag) {
        const float* gj = vr && okJ[q] ? srcJ[q] + shift : a.zeros;
        __builtin_amdgcn_global_load_lds((gptr_t)(gj),
                                         (lptr_t)(sJ + buf * kStage + (w * kGlds + q) * 256), 16, 0, 0);
      }
    }
  };

  // ---- operand reads: row r = 8j + 4 par + lk (r % 4 = lk), column c + rot(lk) (mod 96)
  const int rl = rot(lk);
  int offA[3], offB[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    offA[m] = (4 * par + lk) * kT + (wr * 48 + 16 * m + li + rl) % kT;
    offB[m] = (4 * par + lk) * kT + (wc * 48 + 16 * m + li + rl) % kT;
  }
  // bf16 split path: wave parity par takes the stage's rows [32 par, 32 par + 32); fragment
  // element j of lane group lk is row 32 par + 4 j + lk (the k order inside an MFMA only has to
  // agree between the two operands), so the four rows one ds_read_b32 touches are consecutive
  // and carry the four distinct rotations, as in the FP32 path
  int offA3[3], offB3[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    offA3[m] = (32 * par + lk) * kT + (wr * 48 + 16 * m + li + rl) % kT;
    offB3[m] = (32 * par + lk) * kT + (wc * 48 + 16 * m + li + rl) % kT;
  }
  auto mma_stage_x3 = [&](int buf) {
    const float* cI = sI + buf * kStage;
    const float* cJ = sJr + buf * kStage;
    float av[3][8], bv[3][8];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        av[m][j] = cI[offA3[m] + 4 * j * kT];
        bv[m][j] = cJ[offB3[m] + 4 * j * kT];
      }
    u32x4 a1[3], a2[3], a3[3], b1[3], b2[3], b3[3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      split3(av[m], a1[m], a2[m], a3[m]);
      split3(bv[m], b1[m], b2[m], b3[m]);
    }
    // term-major order: nine independent accumulators between two dependent MFMAs.  The stage
    // sums into fresh accumulators that are added to the running ones on the VALU (one RNE
    // rounding per stage): chaining all six split products of every row into the running sum
    // would round each small term against the whole-K magnitude (measured: 4x the FP32 path's
    // error at K = 50000; per-stage partials put it below that path)
    f32x4 sacc[3][3];
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a3[m], b1[n], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a1[m], b3[n], sacc[m][n]);
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a2[m], b2[n], sacc[m][n]);
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a2[m], b1[n], sacc[m][n]);
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a1[m], b2[n], sacc[m][n]);
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n) acc[m][n] += mfma_bf16(a1[m], b1[n], sacc[m][n]);
  };
  auto mma_stage = [&](int buf) {
    const float* cI = sI + buf * kStage;
    const float* cJ = sJr + buf * kStage;
    float av[2][3], bv[2][3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      av[0][m] = cI[offA[m]];
      bv[0][m] = cJ[offB[m]];
    }
#pragma unroll
    for (int j = 0; j < kBK / 8; ++j) {  // this wave's k-steps
      const int cur = j & 1;
      if (j + 1 < kBK / 8) {
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          av[cur ^ 1][m] = cI[(j + 1) * 8 * kT + offA[m]];
          bv[cur ^ 1][m] = cJ[(j + 1) * 8 * kT + offB[m]];
        }
      }
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[cur][m], bv[cur][n], acc[m][n], 0, 0, 0);
    }
#if TEA_K8_SCHED
    // pin the software pipeline: the first step's operand reads, then per step the next
    // step's reads issued ahead of this step's 9 MFMAs (the default schedule re-reads into
    // registers that are still feeding MFMAs and waits lgkmcnt(0) right before the next group)
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int j = 0; j < kBK / 8; ++j) {
      if (j + 1 < kBK / 8) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 9, 0);
    }
#endif
  };

  // ---- diagonal tiles: quadrant (1, 0) is the transpose of quadrant (0, 1), so its two waves
  // (both on one SIMD) skip their MFMAs and sum the tile's columns instead (wave par: rows of
  // parity par; lane: columns lane and 64 + lane); the epilogue mirrors (0, 1) into (1, 0).
  // The diagonal blocks then carry no more MFMA-pipe work than the others, which they would
  // otherwise add to the kernel's critical path.
  const bool col_wave = diag && quad == 2;
  float colsum0 = 0.f, colsum1 = 0.f;
  auto col_stage = [&](int buf) {
    const float* img = sI + buf * kStage;
#pragma unroll 8
    for (int r = par; r < kBK; r += 2) {
      colsum0 += img[r * kT + (lane + rot(r)) % kT];
      if (lane < kT - 64) colsum1 += img[r * kT + (64 + lane + rot(r)) % kT];
    }
  };

  // ---- the C tile (and its mirror) this block read-modify-writes at the end: loaded into
  // registers now, so the epilogue's reads are not a serial HBM round trip after the loop
  // C is read as float4 rows when d % 4 == 0 (every 4-column group then lies wholly inside or
  // outside [0, d)): 96 x 24 float4 per tile, <= 5 per thread, clamped addresses + selects so
  // the loads issue back to back (a guarded load per element compiled to a branch + wait each)
  constexpr int kSeg4 = kT / 4;                                     // 24
  constexpr int kPer4 = (kT * kSeg4 + kThreads - 1) / kThreads;     // 5
  const bool vec4 = a.d % 4 == 0;
  float4 cpre[kPer4], mpre[kPer4];
  auto prefetch_c = [&]() {
    if (!(a.split == 1 && vec4)) return;
#pragma unroll
    for (int q = 0; q < kPer4; ++q) {
      const int e = threadIdx.x + kThreads * q;
      const int row = (e < kT * kSeg4 ? e : 0) / kSeg4, c4 = ((e < kT * kSeg4 ? e : 0) % kSeg4) * 4;
      const bool in = e < kT * kSeg4 && I0 + row < a.d && J0 + c4 < a.d;
      const bool min_ = e < kT * kSeg4 && !diag && J0 + row < a.d && I0 + c4 < a.d;
      const float4 x = *reinterpret_cast<const float4*>(a.cov + (in ? (I0 + row) * a.d + J0 + c4 : 0));
      const float4 y = *reinterpret_cast<const float4*>(a.cov + (min_ ? (J0 + row) * a.d + I0 + c4 : 0));
      // per-component selects (a whole-float4 select is lowered through a stack slot)
      cpre[q] = make_float4(in ? x.x : 0.f, in ? x.y : 0.f, in ? x.z : 0.f, in ? x.w : 0.f);
      mpre[q] = make_float4(min_ ? y.x : 0.f, min_ ? y.y : 0.f, min_ ? y.z : 0.f, min_ ? y.w : 0.f);
    }
  };
  // kMode 2 keeps its next stage in registers during the loop: its C reads go after the loop
  if constexpr (kMode != 2) prefetch_c();

  // ---- K loop: three LDS stages, two LDS-DMA stages in flight behind the MFMAs.  The end of
  // stage s waits only for stage s + 1's pieces (a counted vmcnt leaves stage s + 2's in
  // flight) and meets at a raw s_barrier - __syncthreads() would drain vmcnt to 0.  The buffer
  // refilled at stage s + 1 is the one stage s read, so that barrier also retires its reads.
  auto wait_next = [&](bool keep_one) {
    if (keep_one) {
      if (diag) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");  // kGlds pieces per stage
      else asm volatile("s_waitcnt vmcnt(6)" ::: "memory");       // 2 x kGlds
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
  };
  static_assert(kGlds == 3, "the counted waits above assume 3 pieces per operand per stage");

  // ---- kMode 2: register-staged columns, split once per element into LDS bf16 planes
  constexpr int kPlaneB = 8 * kT * 16;  // one plane of one operand: [8 k-groups][96 columns] x 16 B
  constexpr int kOpB = 3 * kPlaneB;      // 36 KB
  constexpr int kBufB = 2 * kOpB;        // 72 KB per stage, two stages = kSmemBytes
  static_assert(2 * kBufB <= kSmemBytes, "two plane stages must fit the LDS allocation");
  constexpr int kUnits = 3;              // (operand, k-group, column) units per thread
  static_assert(kUnits * kThreads == 2 * 8 * kT, "units must cover both operands' 8 x 96 pieces");
  float cs2[kUnits] = {0.f, 0.f, 0.f};   // diagonal tiles: per-unit column sums (operand I)
  if constexpr (kMode == 2) {
    char* lds = reinterpret_cast<char*>(smem);
    // raw buffer loads over this item's K range: a byte offset at or past num_records reads 0,
    // which masks the rows past the range; an invalid unit (a column past the width, or the
    // J operand of a diagonal tile) starts at 2^31 (the launcher keeps the range below 2^31 B)
    // (a split-K item past the end has an empty range: num_records 0, every load reads 0)
    const uint32_t rs4 = static_cast<uint32_t>(a.row_stride) * 4u;
    const int64_t krows = k1 > k0 ? k1 - k0 : 0;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.act + (krows ? k0 * a.row_stride : 0)), 0, static_cast<int>(krows * rs4), 0x00020000);
    uint32_t uvo[kUnits];
    int uoff[kUnits];
    bool ucs[kUnits];
#pragma unroll
    for (int q = 0; q < kUnits; ++q) {
      const int u = (w * kUnits + q) * 64 + lane;
      const int op = u / (8 * kT), g = (u / kT) % 8, col = u % kT;
      const int64_t x0 = op ? J0 : I0;
      const bool ok = x0 + col < a.ld && !(diag && op == 1);
      uvo[q] = ok ? static_cast<uint32_t>(8 * g) * rs4 + static_cast<uint32_t>(x0 + col) * 4u : 0x80000000u;
      uoff[q] = op * kOpB + (g * kT + col) * 16;
      ucs[q] = diag && op == 0;
    }
    float v[kUnits][8];
    auto load = [&](int64_t b0) {
      const uint32_t st = static_cast<uint32_t>(b0 - k0) * rs4;
#pragma unroll
      for (int q = 0; q < kUnits; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[q][j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, uvo[q] + st + j * rs4, 0, 0));
    };
    auto split_store = [&](int b) {
#pragma unroll
      for (int q = 0; q < kUnits; ++q) {
        float t = 0.f;  // (branch-free: a divergent branch would split the stage's block)
#pragma unroll
        for (int j = 0; j < 8; ++j) t += v[q][j];
        cs2[q] += ucs[q] ? t : 0.f;
        u32x4 p1, p2, p3;
        split3(v[q], p1, p2, p3);
        char* dst = lds + b * kBufB + uoff[q];
        *reinterpret_cast<u32x4*>(dst) = p1;
        *reinterpret_cast<u32x4*>(dst + kPlaneB) = p2;
        *reinterpret_cast<u32x4*>(dst + 2 * kPlaneB) = p3;
      }
    };
    // fragment reads: block column c, k-group 4 par + lk -> one ds_read_b128 per plane
    const int fa = ((4 * par + lk) * kT + wr * 48 + li) * 16;
    const int fb = (diag ? 0 : kOpB) + ((4 * par + lk) * kT + wc * 48 + li) * 16;
    auto mma_planes = [&](int b) {
      const char* base = lds + b * kBufB;
      u32x4 a1[3], a2[3], a3[3], b1[3], b2[3], b3[3];
#pragma unroll
      for (int m = 0; m < 3; ++m) {
        const char* pa = base + fa + m * 16 * 16;
        const char* pb = base + fb + m * 16 * 16;
        a1[m] = *reinterpret_cast<const u32x4*>(pa);
        a2[m] = *reinterpret_cast<const u32x4*>(pa + kPlaneB);
        a3[m] = *reinterpret_cast<const u32x4*>(pa + 2 * kPlaneB);
        b1[m] = *reinterpret_cast<const u32x4*>(pb);
        b2[m] = *reinterpret_cast<const u32x4*>(pb + kPlaneB);
        b3[m] = *reinterpret_cast<const u32x4*>(pb + 2 * kPlaneB);
      }
      f32x4 sacc[3][3];
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a3[m], b1[n], f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a1[m], b3[n], sacc[m][n]);
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a2[m], b2[n], sacc[m][n]);
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a2[m], b1[n], sacc[m][n]);
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) sacc[m][n] = mfma_bf16(a1[m], b2[n], sacc[m][n]);
#pragma unroll
      for (int m = 0; m < 3; ++m)
#pragma unroll
        for (int n = 0; n < 3; ++n) acc[m][n] += mfma_bf16(a1[m], b1[n], sacc[m][n]);
    };
    load(k0);
    split_store(0);
    load(k0 + kBK);
    __syncthreads();
    int b = 0;
    // One basic block per stage, so the next stage's split (VALU), LDS stores and global loads
    // can be interleaved with this stage's MFMAs (in-order issue: VALU placed after 54 MFMAs
    // would wait for all of them to issue).  Past the K range the loads read the zero line and
    // the last stores land in a buffer nobody reads (the loop's final barrier orders them
    // before the epilogue reuses the LDS).  Every wave runs the MFMAs: on a diagonal tile the
    // quadrant (1, 0) result is discarded by the mirror, and the column sums come from the
    // staging units instead.
    for (int64_t b0 = k0; b0 < k1; b0 += kBK) {
      __builtin_amdgcn_sched_barrier(0);
      mma_planes(b);
      split_store(b ^ 1);  // the other stage's readers all passed the previous barrier
#ifndef TEA_K8_NO_STAGE_LOADS  // (csrc/bench/k8_variants.hip: the loop without its global loads)
      load(b0 + 2 * kBK);
#endif
#if TEA_K8_SCHED
      __builtin_amdgcn_sched_group_barrier(0x100, 18, 0);  // fragment reads
#pragma unroll
      for (int i = 0; i < 54; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // three VALU of the next stage's split
      }
      __builtin_amdgcn_sched_group_barrier(0x200, 9, 0);   // plane stores
      __builtin_amdgcn_sched_group_barrier(0x020, 24, 0);  // next loads
#endif
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
      b ^= 1;
    }
    prefetch_c();
  } else {
  issue(0, k0);
  const bool two = k0 + kBK < k1;
  if (two) issue(1, k0 + kBK);
  wait_next(two);
  int buf = 0;
  for (int64_t b0 = k0; b0 < k1; b0 += kBK) {
    const int ahead = buf == 0 ? 2 : buf - 1;  // (buf + 2) % 3
    const bool more = b0 + 2 * kBK < k1;
#ifndef TEA_K8_NO_STAGE_LOADS  // (csrc/bench/k8_variants.hip: the loop without its global loads)
    if (more) issue(ahead, b0 + 2 * kBK);
#endif
    if (col_wave) {
      col_stage(buf);
    } else {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (kMode == 1) mma_stage_x3(buf);
      else mma_stage(buf);
      __builtin_amdgcn_sched_barrier(0);
    }
    wait_next(more);
    buf = buf == 2 ? 0 : buf + 1;
  }
  }  // kMode 0 / 1

  // ---- sum the two k-parity halves of each quadrant in LDS (96 x 97 floats, reusing the
  // operand buffers; the loop's last barrier retired every operand read)
  float* sC = smem;
  float* sCol = smem + kCPad * kT;  // [2][kT] (kMode 2: [8][kT]): the column-sum partials
  auto to_lds = [&](bool add) {
#pragma unroll
    for (int m = 0; m < 3; ++m)
#pragma unroll
      for (int n = 0; n < 3; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int idx = (wr * 48 + m * 16 + 4 * lk + r) * kCPad + wc * 48 + n * 16 + li;
          sC[idx] = add ? sC[idx] + acc[m][n][r] : acc[m][n][r];
        }
  };
  if constexpr (kMode == 2) {
    if (diag) {  // sCol [8 k-groups][kT]: unit (0, g, col) -> sCol[g * kT + col]
#pragma unroll
      for (int q = 0; q < kUnits; ++q) {
        const int u = (w * kUnits + q) * 64 + lane;
        if (u < 8 * kT) sCol[u] = cs2[q];
      }
    }
  } else if (col_wave) {
    sCol[par * kT + lane] = colsum0;
    if (lane < kT - 64) sCol[par * kT + 64 + lane] = colsum1;
  }
  if (par == 1 && !col_wave) to_lds(false);
  __syncthreads();
  if (par == 0 && !col_wave) to_lds(true);
  __syncthreads();
  float colsum = 0.f;
  if (diag) {
    // the lower triangle = the upper transposed: quadrant (1, 0) was never computed, and on the
    // split path the diagonal quadrants' (i, j) and (j, i) sum the same split products in a
    // different order, so the mirror keeps the result exactly symmetric
    for (int e = threadIdx.x; e < kT * kT; e += kThreads) {
      const int r = e / kT, c = e % kT;
      if (r > c) sC[r * kCPad + c] = sC[c * kCPad + r];
    }
    if (threadIdx.x < kT) {
      if constexpr (kMode == 2) {
#pragma unroll
        for (int g = 0; g < 8; ++g) colsum += sCol[g * kT + threadIdx.x];
      } else {
        colsum = sCol[threadIdx.x] + sCol[kT + threadIdx.x];
      }
    }
    __syncthreads();
  }

  if (a.split > 1) {
    // raw partial tile [kT][kT] (row-major) + diagonal column-sum partial for the fix-up pass
    float* part = a.ws + static_cast<int64_t>(item) * kT * kT;
    for (int e = threadIdx.x; e < kT * kT; e += kThreads) part[e] = sC[(e / kT) * kCPad + e % kT];
    if (diag && threadIdx.x < kT)
      a.ws[static_cast<int64_t>(items) * kT * kT + (static_cast<int64_t>(ks) * T + ti) * kT + threadIdx.x] = colsum;
    return;
  }

  // ---- epilogue: C[I, J] += tile and mirrored C[J, I] += tile^T as float4 rows (C read up
  // front); a scalar pass when d % 4 != 0
  if (vec4) {
#pragma unroll
    for (int q = 0; q < kPer4; ++q) {
      const int e = threadIdx.x + kThreads * q;
      if (e >= kT * kSeg4) continue;
      const int row = e / kSeg4, c4 = (e % kSeg4) * 4;
      if (I0 + row < a.d && J0 + c4 < a.d) {
        const float* t = sC + row * kCPad + c4;
        *reinterpret_cast<float4*>(a.cov + (I0 + row) * a.d + J0 + c4) =
            make_float4(cpre[q].x + t[0], cpre[q].y + t[1], cpre[q].z + t[2], cpre[q].w + t[3]);
      }
      if (!diag && J0 + row < a.d && I0 + c4 < a.d) {
        // mirrored: C[J0 + row][I0 + c4 + k] = tile[c4 + k][row]
        const float* t = sC + c4 * kCPad + row;
        *reinterpret_cast<float4*>(a.cov + (J0 + row) * a.d + I0 + c4) =
            make_float4(mpre[q].x + t[0], mpre[q].y + t[kCPad], mpre[q].z + t[2 * kCPad], mpre[q].w + t[3 * kCPad]);
      }
    }
  } else {
    for (int e = threadIdx.x; e < kT * kT; e += kThreads) {
      const int row = e / kT, col = e % kT;
      const int64_t gi = I0 + row, gj = J0 + col;
      if (gi < a.d && gj < a.d) a.cov[gi * a.d + gj] += sC[row * kCPad + col];
      if (!diag) {
        const int64_t mi = J0 + row, mj = I0 + col;
        if (mi < a.d && mj < a.d) a.cov[mi * a.d + mj] += sC[col * kCPad + row];
      }
    }
  }
  if (diag && a.colsum && threadIdx.x < kT && I0 + threadIdx.x < a.d) a.colsum[I0 + threadIdx.x] += colsum;
}

// split-K fix-up: one block per 32 x 32 sub-tile of an upper tile; sums the `split` partials
// in item order, RMWs C and the mirrored C^T sub-tile (LDS transpose), and folds the column
// sums of the diagonal tiles.
__global__ __launch_bounds__(kFixThreads) void fid_fixup_kernel(FidCovArgs a, int T, int tiles) {
  constexpr int kS = 32;
  constexpr int kSub = kT / kS;  // 3
  const int tile = blockIdx.x / (kSub * kSub);
  const int sub = blockIdx.x % (kSub * kSub);
  const int r0 = (sub / kSub) * kS, c0 = (sub % kSub) * kS;
  int ti, tj;
  tile_coords(tile, T, ti, tj);
  const int64_t I0 = static_cast<int64_t>(ti) * kT, J0 = static_cast<int64_t>(tj) * kT;
  const bool diag = ti == tj;
  const int64_t items = static_cast<int64_t>(tiles) * a.split;
  __shared__ float s[kS][kS + 1];
#pragma unroll
  for (int q = 0; q < kS * kS / kFixThreads; ++q) {
    const int e = threadIdx.x + kFixThreads * q;
    const int row = e / kS, col = e % kS;
    float v = 0.f;
    for (int ks = 0; ks < a.split; ++ks)
      v += a.ws[(static_cast<int64_t>(ks) * tiles + tile) * kT * kT + (r0 + row) * kT + c0 + col];
    s[row][col] = v;
    const int64_t gi = I0 + r0 + row, gj = J0 + c0 + col;
    if (gi < a.d && gj < a.d) a.cov[gi * a.d + gj] += v;
  }
  if (!diag) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kS * kS / kFixThreads; ++q) {
      const int e = threadIdx.x + kFixThreads * q;
      const int row = e / kS, col = e % kS;  // mirrored C[J0 + c0 + row][I0 + r0 + col] = sub[col][row]
      const int64_t mi = J0 + c0 + row, mj = I0 + r0 + col;
      if (mi < a.d && mj < a.d) a.cov[mi * a.d + mj] += s[col][row];
    }
  } else if (a.colsum && r0 == 0 && threadIdx.x < kS) {
    const int64_t c = I0 + c0 + threadIdx.x;
    float v = 0.f;
    for (int ks = 0; ks < a.split; ++ks) v += a.ws[items * kT * kT + (static_cast<int64_t>(ks) * T + ti) * kT + c0 + threadIdx.x];
    if (c < a.d) a.colsum[c] += v;
  }
}

int cu_count() {
  static int cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0)
      v = 256;
    return v;
  }();
  return cus;
}

}  // namespace

int fid_cov_mode() {
  const char* e = std::getenv("TORCHEVAL_AMD_K8_EXACT");
  if (e != nullptr && e[0] == '1') return 0;
  const char* m = std::getenv("TORCHEVAL_AMD_K8_MODE");
  if (m != nullptr && (m[0] == '0' || m[0] == '1')) return m[0] - '0';
  return 2;
}

int fid_cov_split(int64_t n, int64_t d) {
  if (const char* e = std::getenv("TORCHEVAL_AMD_K8_SPLIT")) {
    const int s = std::atoi(e);
    if (s >= 1) return s;
  }
  const int64_t T = (d + kT - 1) / kT;
  const int64_t tiles = T * (T + 1) / 2;
  const int64_t cus = cu_count();
  if (tiles * 4 >= cus * 3) return 1;  // the triangle fills >= 3/4 of the CUs already
  const int64_t stages = (n + kBK - 1) / kBK;
  int64_t s = cus / tiles;               // one item per CU
  // keep >= 4 stages (256 rows) per item: at K = 1000, D = 512 / 768 a split of 4 beats the
  // 7-8 that "one item per CU" gives (22.6 vs 24.6 us, 24.4 vs 26.2; profiles/k8_smalld_splits_r3.json)
  s = std::min<int64_t>(s, stages / 4);
  return static_cast<int>(std::max<int64_t>(s, 1));
}

int64_t fid_cov_workspace_bytes(int64_t d, int split) {
  if (split <= 1) return 0;
  const int64_t T = (d + kT - 1) / kT;
  const int64_t tiles = T * (T + 1) / 2;
  return (static_cast<int64_t>(split) * tiles * kT * kT + static_cast<int64_t>(split) * T * kT) * 4;
}

int launch_fid_cov(const FidCovArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.d <= 0) return 0;
  const int T = static_cast<int>((a.d + kT - 1) / kT);
  const int tiles = T * (T + 1) / 2;
  const int split = std::max(1, a.split);
  if (split > 1 && a.ws == nullptr) return -1;
  // K range per item: whole stages
  const int64_t stages = (a.n + kBK - 1) / kBK;
  const int64_t chunk = ((stages + split - 1) / split) * kBK;
  const int items = tiles * split;
  const int grid = (items + 7) / 8 * 8;
  auto opt_in = [](const void* f) {
    return hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kSmemBytes) == hipSuccess;
  };
  static const bool lds_ok = opt_in(reinterpret_cast<const void*>(&fid_syrk_kernel<0>)) &&
                             opt_in(reinterpret_cast<const void*>(&fid_syrk_kernel<1>)) &&
                             opt_in(reinterpret_cast<const void*>(&fid_syrk_kernel<2>));
  if (!lds_ok) return -3;
  if (a.zeros == nullptr || a.ld % 4 != 0 || a.ld < a.d || a.row_stride % 4 != 0) return -1;
  int mode = fid_cov_mode();
  // kMode 2 addresses an item's K range (+ two stages of overrun) with 32-bit buffer offsets
  if (mode == 2 && (chunk + 2 * kBK) * a.row_stride * 4 >= (int64_t{1} << 31)) mode = 1;
  switch (mode) {
    case 0:
      hipLaunchKernelGGL(fid_syrk_kernel<0>, dim3(grid), dim3(kThreads), kSmemBytes, stream, a, T, tiles, items, chunk);
      break;
    case 1:
      hipLaunchKernelGGL(fid_syrk_kernel<1>, dim3(grid), dim3(kThreads), kSmemBytes, stream, a, T, tiles, items, chunk);
      break;
    default:
      hipLaunchKernelGGL(fid_syrk_kernel<2>, dim3(grid), dim3(kThreads), kSmemBytes, stream, a, T, tiles, items, chunk);
  }
  int rc = static_cast<int>(hipGetLastError());
  if (rc || split == 1) return rc;
  hipLaunchKernelGGL(fid_fixup_kernel, dim3(tiles * 9), dim3(kFixThreads), 0, stream, a, T, tiles);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
