// Odd-width probe: do 16-B loads from 4-B-aligned addresses (rows of an odd width start at
// every 4-B phase) stream at the aligned rate on gfx950?  Three read-only kernels over the
// same [N, D] fp32 matrix, one wave per row (K1's geometry), 4 x 16-B loads per lane:
//   aligned   D = 1000 (every row 16-B aligned)
//   unaligned D = 1001, float4 loads at 4-B-aligned addresses (ext_vector_type aligned(4))
//   split     D = 1001, scalar head up to the first 16-B boundary, aligned 16-B body, tail
// and the column-walk geometry of K5 (a thread owns 4 columns and walks rows) at both widths.
// Usage: unaligned_probe.bin [iters=400]; one line per variant, us per launch (events).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

typedef float f4a __attribute__((ext_vector_type(4)));
typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));

namespace {

constexpr int N = 8192;

template <bool UNALIGNED>
__global__ __launch_bounds__(256) void row_read_kernel(const float* __restrict__ x, int d, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* rp = x + row * d;
  float m = 0.f;
  const int dv = d & ~3;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int col = u * 256 + lane * 4;
    const int cc = col < dv ? col : 0;
    f4a q;
    if constexpr (UNALIGNED) {
      const f4u v = *reinterpret_cast<const f4u*>(rp + cc);
      q = f4a{v.x, v.y, v.z, v.w};
    } else {
      q = *reinterpret_cast<const f4a*>(rp + cc);
    }
    m += col < dv ? (q.x + q.y) + (q.z + q.w) : 0.f;
  }
  if (lane < d - dv) m += rp[dv + lane];
  if (m == 12345.678f) sink[row] = m;
}

__global__ __launch_bounds__(256) void row_read_split_kernel(const float* __restrict__ x, int d, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const int64_t off = row * d;
  const int head = static_cast<int>((4 - (off & 3)) & 3);
  const float* bp = x + off + head;  // 16-B aligned
  const int nb = (d - head) >> 2;
  float m = 0.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int v = u * 64 + lane;
    const f4a q = *reinterpret_cast<const f4a*>(bp + 4 * (v < nb ? v : 0));
    m += v < nb ? (q.x + q.y) + (q.z + q.w) : 0.f;
  }
  const int tail = d - head - 4 * nb;
  if (lane < head) m += x[off + lane];
  if (lane < tail) m += bp[4 * nb + lane];
  if (m == 12345.678f) sink[row] = m;
}

// K5 geometry: block = 64 column groups x 4 row lanes, each thread walks 8 rows (U = 8)
template <bool UNALIGNED>
__global__ __launch_bounds__(256) void col_walk_kernel(const float* __restrict__ x, int d, int rows_per_block,
                                                      float* __restrict__ sink) {
  const int cg = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int col = (blockIdx.y * 64 + cg) * 4;
  if (col + 3 >= d) return;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  for (int64_t r = r0 + rl; r < r0 + rows_per_block; r += 32) {
    f4a q[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float* p = x + (r + 4 * u) * d + col;
      if constexpr (UNALIGNED) {
        const f4u v = *reinterpret_cast<const f4u*>(p);
        q[u] = f4a{v.x, v.y, v.z, v.w};
      } else {
        q[u] = *reinterpret_cast<const f4a*>(p);
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a0 += q[u].x;
      a1 += q[u].y;
      a2 += q[u].z;
      a3 += q[u].w;
    }
  }
  if (a0 + a1 + a2 + a3 == 12345.678f) sink[col] = a0;
}

template <typename F>
float time_us(F launch, int iters) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) launch(i);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  return ms * 1e3f / iters;
}

}  // namespace

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 400;
  constexpr int kPool = 8;
  const size_t per = static_cast<size_t>(N) * 1024;
  float* x;
  float* sink;
  CK(hipMalloc(&x, per * kPool * sizeof(float)));
  CK(hipMalloc(&sink, 1 << 20));
  CK(hipMemset(x, 0, per * kPool * sizeof(float)));
  auto buf = [&](int i) { return x + per * (i % kPool); };
  for (int rep = 0; rep < 3; ++rep) {
    for (int d : {1000, 1001, 1002, 1003}) {
      const double mb = static_cast<double>(N) * d * 4 / 1e6;
      const float ta = d % 4 == 0 ? time_us([&](int i) {
        hipLaunchKernelGGL(row_read_kernel<false>, dim3(N / 4), dim3(256), 0, 0, buf(i), d, sink);
      }, iters) : -1.f;
      const float tu = time_us([&](int i) {
        hipLaunchKernelGGL(row_read_kernel<true>, dim3(N / 4), dim3(256), 0, 0, buf(i), d, sink);
      }, iters);
      const float ts = time_us([&](int i) {
        hipLaunchKernelGGL(row_read_split_kernel, dim3(N / 4), dim3(256), 0, 0, buf(i), d, sink);
      }, iters);
      const dim3 cgrid(N / 64, (d / 4 + 63) / 64);
      const float ca = d % 4 == 0 ? time_us([&](int i) {
        hipLaunchKernelGGL(col_walk_kernel<false>, cgrid, dim3(256), 0, 0, buf(i), d, 64, sink);
      }, iters) : -1.f;
      const float cu = time_us([&](int i) {
        hipLaunchKernelGGL(col_walk_kernel<true>, cgrid, dim3(256), 0, 0, buf(i), d, 64, sink);
      }, iters);
      printf("{\"d\": %d, \"MB\": %.1f, \"row_aligned_us\": %.2f, \"row_unaligned_us\": %.2f, \"row_split_us\": %.2f, "
             "\"col_aligned_us\": %.2f, \"col_unaligned_us\": %.2f, \"row_unaligned_TBps\": %.2f, \"col_unaligned_TBps\": %.2f}\n",
             d, mb, ta, tu, ts, ca, cu, mb / tu, mb / cu);
    }
  }
  return 0;
}
