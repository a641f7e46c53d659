// K8: FID covariance update C += A^T A, s += colsum(A) on FP32 MFMA.
//
// Replaces fid.py:120-127 (a full D x D x B SGEMM plus a separate column sum) with one
// symmetric rank-k update that computes only the upper-triangle tiles (half the FLOPs),
// mirrors them, and fuses the column sums into the diagonal tiles.
//
// gfx950 mapping, v3.  Round-1's v2 (64 x 64 tiles, 4 waves each owning one 32 x 32 block)
// ran 82 us at 1000 x 2048 with SQ_VALU_MFMA_BUSY ~33 %: one 32 x 32 accumulator per wave
// means two LDS operand reads per MFMA and 16 B/clk/CU of L2 operand traffic per block, and
// D = 2048 gives 528 tiles for 256 CUs (16 CUs run a third tile).  v3 sizes the tile so the
// upper triangle IS the machine:
//  * 96 x 96 output tiles: D = 2048 -> T = 22 tile rows -> 253 upper-triangle tiles, one
//    workgroup per CU in a single wave of blocks (no quantisation tail).
//  * 8 waves = 2 per SIMD: wave w owns the 48 x 48 quadrant w & 3 as 3 x 3 blocks of
//    v_mfma_f32_16x16x4_f32 (exact FP32 products, 9 independent 4-register accumulators), and
//    the k-steps of parity w >> 2 (in-block 2-way split of K, summed through LDS at the end).
//    Per 4-k step a wave reads 3 A + 3 B operands (one ds_read_b32 each) for 9 MFMAs - 3x the
//    operand reuse of v2 - and the next step's operands are read before this step's MFMAs
//    (register double buffer); the SIMD's second wave covers what LDS latency is left.
//    (4 waves with one wave per SIMD, measured: 54 TF at 1000 x 2048, 82 TF at 50k x 2048.)
//  * the K loop streams 64 rows of ``act`` per stage (both operands of sample k are reads of
//    row k), float4 loads, LDS double buffer (112 KB, dynamic) with a register-staged prefetch
//    one stage ahead; the loads are branch-free and their consumers are fenced below the
//    MFMAs with sched_barrier, so the global latency hides behind the matrix work.
//    LDS rows are padded to 112 floats: the four k-rows one ds_read_b32 touches start 48 banks
//    apart (mod 64), so the 16-lane row segments never share a bank.
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

constexpr int kT = 96;        // output tile
constexpr int kBK = 64;       // rows of act per stage
constexpr int kLD = 112;      // padded LDS row (floats)
constexpr int kThreads = 512;  // 8 waves
constexpr int kFixThreads = 256;
constexpr int kStage = kBK * kLD;      // floats per operand per stage
constexpr int kSegs = kT / 4;          // float4 segments per tile row (24)
constexpr int kLoads = kBK * kSegs / kThreads;  // float4 loads per thread per operand (3)
constexpr int kCPad = kT + 1;
static_assert(kBK * kSegs % kThreads == 0, "stage must split evenly over the block");
static_assert(kT * kCPad <= 4 * kStage, "epilogue tile must fit in the operand buffers");
constexpr int kSmemBytes = 4 * kStage * 4;  // 112 KB: one block per CU
static_assert(kCPad * kT + kBK * kT <= 4 * kStage, "epilogue tile + column sums must fit");
static_assert((kCPad * kT) % 4 == 0, "column-sum partials must stay 16-byte aligned");

typedef float f32x4 __attribute__((ext_vector_type(4)));

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

__device__ __forceinline__ float4 load_seg(const float* row, int64_t c, int64_t d) {
  if (c + 3 < d) return *reinterpret_cast<const float4*>(row + c);
  float t[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e = 0; e < 4; ++e)
    if (c + e < d) t[e] = row[c + e];
  return make_float4(t[0], t[1], t[2], t[3]);
}

// kVec: d % 4 == 0, so every float4 segment of a row is wholly inside or wholly outside [0, d)
// and the stage loads are branch-free (clamped address + select): no exec-mask branches and no
// vmcnt waits between the loads of one stage, so all of them overlap the stage's MFMAs.
template <bool kVec>
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

  extern __shared__ __attribute__((aligned(16))) float smem[];  // kSmemBytes
  float* sI = smem;               // [2][kBK][kLD]
  float* sJ = smem + 2 * kStage;  // [2][kBK][kLD]
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
  float colsum = 0.f;

  int srow[kLoads], scol[kLoads];
#pragma unroll
  for (int h = 0; h < kLoads; ++h) {
    const int idx = threadIdx.x + kThreads * h;
    srow[h] = idx / kSegs;
    scol[h] = (idx % kSegs) * 4;
  }
  const float4 zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
  // One stage of global loads in registers.  Two sets: the loads of stage s + 2 are issued
  // at the start of stage s and committed to LDS at the end of stage s + 1, so each load has
  // two stages of MFMA work (~2 x 4.6k cycles) to land.  fetch issues the loads only; the
  // zero-masking of out-of-range rows / columns consumes the values, so it is in commit().
  struct Regs {
    float4 i[kLoads], j[kLoads];
    bool vi[kLoads], vj[kLoads];
  };
  Regs R0, R1;
  auto fetch = [&](Regs& R, int64_t b0) {
#pragma unroll
    for (int h = 0; h < kLoads; ++h) {
      const int64_t b = b0 + srow[h];
      const bool vb = b < k1;
      const float* row = a.act + (vb ? b : k1 - 1) * a.row_stride;  // k1 >= 1: always a real row
      if constexpr (kVec) {
        const int64_t ci = I0 + scol[h], cj = J0 + scol[h];
        R.vi[h] = vb && ci < a.d;
        R.vj[h] = vb && cj < a.d;
        R.i[h] = *reinterpret_cast<const float4*>(row + (ci < a.d ? ci : 0));
        R.j[h] = *reinterpret_cast<const float4*>(row + (cj < a.d ? cj : 0));
      } else {
        R.vi[h] = R.vj[h] = true;
        R.i[h] = vb ? load_seg(row, I0 + scol[h], a.d) : zero4;
        R.j[h] = vb ? load_seg(row, J0 + scol[h], a.d) : zero4;
      }
    }
  };
  // per-component selects: a whole-float4 select gets lowered through a stack slot
  auto masked = [](const float4& x, bool v) {
    return make_float4(v ? x.x : 0.f, v ? x.y : 0.f, v ? x.z : 0.f, v ? x.w : 0.f);
  };
  // diagonal tiles: column sums ride along in registers (each thread always stages the same
  // 4 columns), folded through LDS once at the end - a per-stage LDS pass made the diagonal
  // blocks the slowest blocks of the grid (the no-load loop ran 112 vs 139 TF/s)
  float4 csum[kLoads];
#pragma unroll
  for (int h = 0; h < kLoads; ++h) csum[h] = zero4;
  auto commit = [&](Regs& R, int buf) {
    // branch-free (one basic block with the MFMAs, so the scheduler can interleave them):
    // diagonal tiles also write the unused J buffer, off-diagonal tiles also sum columns
#pragma unroll
    for (int h = 0; h < kLoads; ++h) {
      const int off = buf * kStage + srow[h] * kLD + scol[h];
      const float4 x = masked(R.i[h], R.vi[h]);
#ifndef TEA_K8_NO_LDS_WRITE  // (bench variant: loads consumed by the column sums only)
      *reinterpret_cast<float4*>(sI + off) = x;
      *reinterpret_cast<float4*>(sJ + off) = masked(R.j[h], R.vj[h]);
#else
      csum[h].x += R.j[h].x;
#endif
      csum[h].x += x.x;
      csum[h].y += x.y;
      csum[h].z += x.z;
      csum[h].w += x.w;
    }
  };

  auto mma_stage = [&](int buf) {
    const float* cI = sI + buf * kStage + wr * 48 + li + (4 * par + lk) * kLD;
    const float* cJ = sJr + buf * kStage + wc * 48 + li + (4 * par + lk) * kLD;
    float av[2][3], bv[2][3];
#pragma unroll
    for (int m = 0; m < 3; ++m) {
      av[0][m] = cI[16 * m];
      bv[0][m] = cJ[16 * m];
    }
#pragma unroll
    for (int j = 0; j < kBK / 8; ++j) {  // this wave's k-steps: rows 8j + 4 par + [0, 4)
      const int cur = j & 1;
      if (j + 1 < kBK / 8) {
#pragma unroll
        for (int m = 0; m < 3; ++m) {
          av[cur ^ 1][m] = cI[(j + 1) * 8 * kLD + 16 * m];
          bv[cur ^ 1][m] = cJ[(j + 1) * 8 * kLD + 16 * m];
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
    // registers that are still feeding MFMAs and waits lgkmcnt(0) right before the next
    // group), with the stage's LDS commit, global loads and their address / select VALU work
    // spread over the MFMA gaps instead of forming a serial phase around the barrier
    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
    for (int j = 0; j < kBK / 8; ++j) {
      if (j < 2 * kLoads) {
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x002, 12, 0);
      if (j + 1 < kBK / 8) __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 9, 0);
    }
#endif
  };

  // One K stage, as one basic block: commit stage b0 + BK (loaded during the previous stage,
  // held in C) into the other LDS buffer - free since the last barrier -, issue the loads of
  // stage b0 + 2 BK into F, and run the MFMAs on buffer buf, all interleaved; then the
  // barrier.  Past the end the commits write masked zeros nobody reads and the loads re-read
  // row k1 - 1, so no branch splits the block.
  auto stage = [&](int64_t b0, int buf, Regs& F, Regs& C) {
    __builtin_amdgcn_sched_barrier(0);
#ifndef TEA_K8_NO_STAGE_LOADS  // (csrc/bench/k8_variants.hip: the loop without its global loads)
    commit(C, buf ^ 1);
#ifndef TEA_K8_NO_FETCH
    fetch(F, b0 + 2 * kBK);
#endif
#endif
    mma_stage(buf);
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  };

  fetch(R0, k0);
  commit(R0, 0);
  fetch(R1, k0 + kBK);
  __syncthreads();
  for (int64_t b0 = k0; b0 < k1;) {
    stage(b0, 0, R0, R1);
    b0 += kBK;
    if (b0 >= k1) break;
    stage(b0, 1, R1, R0);
    b0 += kBK;
  }

  // sum the two k-parity halves of each quadrant in LDS (96 x 97 floats, reusing the operand
  // buffers; the loop's last barrier retired every operand read)
  float* sC = smem;
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
  float* sCol = smem + kCPad * kT;  // [kBK][kT] column-sum partials (diagonal tiles)
  if (diag) {
#pragma unroll
    for (int h = 0; h < kLoads; ++h) *reinterpret_cast<float4*>(sCol + srow[h] * kT + scol[h]) = csum[h];
  }
  if (par == 1) to_lds(false);
  __syncthreads();
  if (par == 0) to_lds(true);
  if (diag && threadIdx.x < kT) {
#pragma unroll 8
    for (int r = 0; r < kBK; ++r) colsum += sCol[r * kT + threadIdx.x];
  }
  __syncthreads();

  if (a.split > 1) {
    // raw partial tile [kT][kT] (row-major) + diagonal column-sum partial for the fix-up pass
    float* part = a.ws + static_cast<int64_t>(item) * kT * kT;
    for (int e = threadIdx.x; e < kT * kT; e += kThreads) part[e] = sC[(e / kT) * kCPad + e % kT];
    if (diag && threadIdx.x < kT)
      a.ws[static_cast<int64_t>(items) * kT * kT + (static_cast<int64_t>(ks) * T + ti) * kT + threadIdx.x] = colsum;
    return;
  }

  // epilogue: coalesced RMW of C[I, J] and the mirrored C[J, I] from the LDS tile
  for (int e = threadIdx.x; e < kT * kT; e += kThreads) {
    const int row = e / kT, col = e % kT;
    const int64_t gi = I0 + row, gj = J0 + col;
    if (gi < a.d && gj < a.d) a.cov[gi * a.d + gj] += sC[row * kCPad + col];
    if (!diag) {
      // mirrored tile: C[J0 + row][I0 + col] = tile[col][row]
      const int64_t mi = J0 + row, mj = I0 + col;
      if (mi < a.d && mj < a.d) a.cov[mi * a.d + mj] += sC[col * kCPad + row];
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
  int64_t s = cus / tiles;            // one item per CU
  s = std::min<int64_t>(s, stages / 8);  // keep >= 8 stages per item
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
  static const bool lds_ok = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&fid_syrk_kernel<true>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kSmemBytes) == hipSuccess &&
           hipFuncSetAttribute(reinterpret_cast<const void*>(&fid_syrk_kernel<false>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, kSmemBytes) == hipSuccess;
  }();
  if (!lds_ok) return -3;
  if (a.d % 4 == 0)
    hipLaunchKernelGGL(fid_syrk_kernel<true>, dim3(grid), dim3(kThreads), kSmemBytes, stream, a, T, tiles, items, chunk);
  else
    hipLaunchKernelGGL(fid_syrk_kernel<false>, dim3(grid), dim3(kThreads), kSmemBytes, stream, a, T, tiles, items, chunk);
  int rc = static_cast<int>(hipGetLastError());
  if (rc || split == 1) return rc;
  hipLaunchKernelGGL(fid_fixup_kernel, dim3(tiles * 9), dim3(kFixThreads), 0, stream, a, T, tiles);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
