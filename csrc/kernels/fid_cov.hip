// K8: FID covariance update C += A^T A, s += colsum(A) on FP32 MFMA.
//
// Replaces fid.py:120-127 (a full D x D x B SGEMM plus a separate column sum) with one
// symmetric rank-k update that computes only the upper-triangle tiles (half the FLOPs),
// mirrors them, and fuses the column sums into the diagonal tiles.
//
// gfx950 mapping (v2, after profiling v1's 128 x 128 tiles: 136 blocks for D = 2048 left half
// of the 256 CUs idle and the "prefetch" stalled on its own loads):
//  * 64 x 64 output tiles, 256 threads = 4 waves, each wave one 32 x 32 block accumulated by
//    v_mfma_f32_32x32x2_f32 (exact FP32 products, 16 accumulator VGPRs).  D = 2048 gives 528
//    tiles (> 2 per CU) and ~5 resident blocks per CU by LDS.
//  * the K loop streams rows of ``act``: both MFMA operands of sample k are reads of row k
//    (A-operand lane = act[k][I0 + i], B-operand lane = act[k][J0 + j]), 64 consecutive floats
//    = 256 B per row segment, loaded as float4 (16 threads per row).
//  * BK = 32 rows per stage, LDS double buffer, register-staged prefetch: the next stage's
//    global loads are issued before the current stage's 16 MFMAs and only written to LDS
//    after them, so HBM/L2 latency overlaps the matrix work.
//  * XCD-aware tile order: blocks are dealt round-robin to the 8 XCDs, so block b is remapped
//    to tile (b % 8) * (nb / 8) + b / 8 - each XCD owns a contiguous run of row-panel tiles and
//    reuses the same activation panel from its own L2.
//  * epilogue stages the tile in LDS (64 x 65, conflict-free for the transposed read) and
//    read-modify-writes C[I, J] and the mirrored C[J, I] with coalesced rows; one block owns
//    each output tile, so there are no atomics and the result is deterministic.
//  * measured and rejected (MI355X, 1000 x 2048): in-block split-K with every wave computing
//    the whole tile as 4 MFMA chains (2 x 2 register blocking, half the LDS operand reads):
//    118 us - 176 VGPRs, and the waves still wait ~41% of their cycles on the per-stage
//    operand fetch (SQ_WAIT_INST_ANY), so fewer LDS reads did not help; BK = 64: 104 us;
//    8 x 8 super-tile enumeration (per-XCD runs needing ~16 instead of ~34 panels): 86 us;
//    register prefetch 2 / 3 / 4 stages deep: 83 / 83 / 84 us (so not global latency);
//    k-contiguous [feature][sample] LDS operands (4x4 register transpose at staging) so one
//    ds_read_b128 per operand feeds 4 MFMAs instead of one ds_read_b32 per MFMA: 89.6 vs
//    82.5 us (so not LDS issue either).  What is left is block quantisation: D = 2048 gives
//    528 tiles for 256 CUs, so 16 CUs run 3 tiles while the rest run 2 (~1.45x the mean);
//    only a cross-block split of K (partials + fix-up pass) would even that out.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kTile = 64;
constexpr int kBK = 32;  // rows per stage (64: 104 vs 78 us, 64 KB of LDS halves residency; hoisting the stage's LDS reads ahead of its MFMAs: 87 us)
constexpr int kThreads = 256;
constexpr int kPad = kTile + 1;
constexpr int kStage = kBK * kTile;  // floats per operand per stage

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void tile_coords(int bid, int T, int& ti, int& tj) {
  // bid enumerates the upper triangle (ti <= tj) row by row
  int row = 0, rem = bid;
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

__global__ __launch_bounds__(kThreads) void fid_syrk_kernel(FidCovArgs a) {
  const int T = static_cast<int>((a.d + kTile - 1) / kTile);
  const int nb = gridDim.x;
  int bid = blockIdx.x;
  if (nb % 8 == 0) bid = (bid % 8) * (nb / 8) + bid / 8;
  int ti, tj;
  tile_coords(bid, T, ti, tj);
  const int64_t I0 = static_cast<int64_t>(ti) * kTile, J0 = static_cast<int64_t>(tj) * kTile;
  const bool diag = ti == tj;

  __shared__ __attribute__((aligned(16))) float smem[4 * kStage];  // 32 KB
  float* sI = smem;               // [2][kBK][kTile]
  float* sJ = smem + 2 * kStage;  // [2][kBK][kTile]
  const float* sJr = diag ? sI : sJ;
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int lr = threadIdx.x >> 4;         // 0..15: staged rows lr, lr + 16
  const int lc = (threadIdx.x & 15) * 4;   // 0..60

  // two accumulators on alternating k-steps: consecutive MFMAs are independent, so a wave
  // does not serialise on its own accumulator (2-3 resident waves per SIMD at D = 2048)
  f32x16 acc, acc2;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = acc2[r] = 0.f;
  float colsum = 0.f;

  float4 pI[2], pJ[2];
  auto fetch = [&](int64_t b0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t b = b0 + lr + 16 * h;
      pI[h] = pJ[h] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (b < a.n) {
        const float* row = a.act + b * a.row_stride;
        pI[h] = load_seg(row, I0 + lc, a.d);
        if (!diag) pJ[h] = load_seg(row, J0 + lc, a.d);
      }
    }
  };
  auto commit = [&](int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      *reinterpret_cast<float4*>(sI + buf * kStage + (lr + 16 * h) * kTile + lc) = pI[h];
      if (!diag) *reinterpret_cast<float4*>(sJ + buf * kStage + (lr + 16 * h) * kTile + lc) = pJ[h];
    }
  };

  fetch(0);
  commit(0);
  __syncthreads();
  int buf = 0;
  for (int64_t b0 = 0; b0 < a.n; b0 += kBK) {
    const bool more = b0 + kBK < a.n;
    if (more) fetch(b0 + kBK);  // in flight during this stage's MFMAs
    const float* cI = sI + buf * kStage;
    const float* cJ = sJr + buf * kStage;
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 4) {
      const int k = kk + (lane >> 5);
      const float av = cI[k * kTile + wr * 32 + (lane & 31)];
      const float bv = cJ[k * kTile + wc * 32 + (lane & 31)];
      const float av2 = cI[(k + 2) * kTile + wr * 32 + (lane & 31)];
      const float bv2 = cJ[(k + 2) * kTile + wc * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
      acc2 = __builtin_amdgcn_mfma_f32_32x32x2f32(av2, bv2, acc2, 0, 0, 0);
    }
    if (diag && threadIdx.x < kTile) {
#pragma unroll
      for (int k = 0; k < kBK; ++k) colsum += cI[k * kTile + threadIdx.x];
    }
    if (more) commit(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: tile -> LDS (64 x 65 floats, reusing the operand buffers) -> coalesced RMW
  float* sC = smem;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int col = wc * 32 + (lane & 31);
    sC[row * kPad + col] = acc[r] + acc2[r];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < kTile * kTile; e += kThreads) {
    const int row = e / kTile, col = e % kTile;
    const int64_t gi = I0 + row, gj = J0 + col;
    if (gi < a.d && gj < a.d) a.cov[gi * a.d + gj] += sC[row * kPad + col];
    if (!diag) {
      // mirrored tile: C[J0 + row][I0 + col] = tile[col][row]
      const int64_t mi = J0 + row, mj = I0 + col;
      if (mi < a.d && mj < a.d) a.cov[mi * a.d + mj] += sC[col * kPad + row];
    }
  }
  if (diag && a.colsum && threadIdx.x < kTile && I0 + threadIdx.x < a.d)
    a.colsum[I0 + threadIdx.x] += colsum;
}

}  // namespace

int launch_fid_cov(const FidCovArgs& a, hipStream_t stream) {
  if (a.n <= 0 || a.d <= 0) return 0;
  const int T = static_cast<int>((a.d + kTile - 1) / kTile);
  const int blocks = T * (T + 1) / 2;
  hipLaunchKernelGGL(fid_syrk_kernel, dim3(blocks), dim3(kThreads), 0, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
