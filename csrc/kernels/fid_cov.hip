// K8: FID covariance update C += A^T A, s += colsum(A) on FP32 MFMA.
//
// Replaces fid.py:120-127 (a full D x D x B SGEMM plus a separate column sum) with one
// symmetric rank-k update that computes only the upper-triangle 128 x 128 tiles (half the
// FLOPs) and mirrors them, with the column sums fused into the diagonal tiles.
//
// gfx950 mapping:
//  * v_mfma_f32_32x32x2_f32 (exact FP32 fmaf chains, 64 FLOP/clk/SIMD): the A-operand lane
//    holds A^T[i][k] = act[k][i], the B-operand lane act[k][j] - both are reads of row k of
//    the activation matrix, so the K loop streams rows of ``act`` (128 consecutive floats =
//    512 B per row segment, fully coalesced) into LDS.
//  * 256-thread blocks, 4 waves, each wave a 64 x 64 sub-tile = 2 x 2 MFMA tiles
//    (4 x 16 accumulator registers); LDS double buffer of 2 x (BK x 128) floats per operand.
//  * epilogue stages the 128 x 128 tile in LDS (padded rows) so both C[I,J] and the mirrored
//    C[J,I] are read-modify-written with coalesced rows.  Each output tile is owned by one
//    block, so no atomics.
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

constexpr int kTile = 128;
constexpr int kBK = 16;
constexpr int kThreads = 256;
constexpr int kPad = kTile + 1;

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

__global__ __launch_bounds__(kThreads) void fid_syrk_kernel(FidCovArgs a) {
  const int T = static_cast<int>((a.d + kTile - 1) / kTile);
  int ti, tj;
  tile_coords(blockIdx.x, T, ti, tj);
  const int64_t I0 = static_cast<int64_t>(ti) * kTile, J0 = static_cast<int64_t>(tj) * kTile;
  const bool diag = ti == tj;

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* sI = smem;                         // [2][kBK][kTile]
  float* sJ = smem + 2 * kBK * kTile;       // [2][kBK][kTile]
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int wr = w >> 1, wc = w & 1;

  f32x16 acc[2][2];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[m][n][r] = 0.f;
  float colsum = 0.f;

  // each thread stages 8 floats per operand per stage: rows (tid / 32) and (tid / 32 + 8),
  // columns 4 * (tid % 32) .. +3
  const int lr = threadIdx.x >> 5;          // 0..7
  const int lc = (threadIdx.x & 31) * 4;    // 0..124
  auto stage = [&](int buf, int64_t b0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = lr + 8 * h;
      const int64_t b = b0 + r;
      float4 vi = make_float4(0.f, 0.f, 0.f, 0.f), vj = vi;
      if (b < a.n) {
        const float* row = a.act + b * a.row_stride;
        if (I0 + lc + 3 < a.d) {
          vi = *reinterpret_cast<const float4*>(row + I0 + lc);
        } else {
          float t4[4] = {0.f, 0.f, 0.f, 0.f};
          for (int e = 0; e < 4; ++e)
            if (I0 + lc + e < a.d) t4[e] = row[I0 + lc + e];
          vi = make_float4(t4[0], t4[1], t4[2], t4[3]);
        }
        if (!diag) {
          if (J0 + lc + 3 < a.d) {
            vj = *reinterpret_cast<const float4*>(row + J0 + lc);
          } else {
            float t4[4] = {0.f, 0.f, 0.f, 0.f};
            for (int e = 0; e < 4; ++e)
              if (J0 + lc + e < a.d) t4[e] = row[J0 + lc + e];
            vj = make_float4(t4[0], t4[1], t4[2], t4[3]);
          }
        }
      }
      *reinterpret_cast<float4*>(sI + (buf * kBK + r) * kTile + lc) = vi;
      if (!diag) *reinterpret_cast<float4*>(sJ + (buf * kBK + r) * kTile + lc) = vj;
    }
  };

  const float* sJbase = diag ? sI : sJ;
  int buf = 0;
  stage(0, 0);
  __syncthreads();
  for (int64_t b0 = 0; b0 < a.n; b0 += kBK) {
    if (b0 + kBK < a.n) stage(buf ^ 1, b0 + kBK);  // prefetch next stage into the other buffer
    const float* cI = sI + buf * kBK * kTile;
    const float* cJ = sJbase + buf * kBK * kTile;
    if (diag && threadIdx.x < kTile) {
#pragma unroll
      for (int k = 0; k < kBK; ++k) colsum += cI[k * kTile + threadIdx.x];
    }
#pragma unroll
    for (int kk = 0; kk < kBK; kk += 2) {
      const int k = kk + (lane >> 5);
      float av[2], bv[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) av[m] = cI[k * kTile + wr * 64 + m * 32 + (lane & 31)];
#pragma unroll
      for (int n = 0; n < 2; ++n) bv[n] = cJ[k * kTile + wc * 64 + n * 32 + (lane & 31)];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[m], bv[n], acc[m][n], 0, 0, 0);
    }
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: stage the tile in LDS (reuses the operand buffers: 128 x 129 floats = 66 KB)
  float* sC = smem;
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wr * 64 + m * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int col = wc * 64 + n * 32 + (lane & 31);
        sC[row * kPad + col] = acc[m][n][r];
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
  const size_t smem_ops = 4 * kBK * kTile * sizeof(float);
  const size_t smem_c = static_cast<size_t>(kTile) * kPad * sizeof(float);
  const size_t smem = smem_ops > smem_c ? smem_ops : smem_c;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(fid_syrk_kernel),
                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(smem));
    attr_set = true;
  }
  hipLaunchKernelGGL(fid_syrk_kernel, dim3(blocks), dim3(kThreads), smem, stream, a);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
