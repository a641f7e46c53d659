// Launch-to-host-observation latency of a tiny kernel on MI355X, three ways:
//   sync    hipLaunchKernel + hipStreamSynchronize (what torch.cuda.synchronize / .item() wait on)
//   memcpy  hipLaunchKernel + 4-byte hipMemcpyAsync D2H + hipStreamSynchronize (== tensor.item())
//   poll    the kernel stores a sequence number into pinned, device-mapped host memory with a
//           system-scope store; the host spins on that word (no HIP call after the launch)
// Each measured idle (device synchronized first) and behind a ~6 us streaming kernel (the
// state of a compute() right after updates).  Median of 300 each, microseconds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ void tiny_kernel(int* dev_word, int v) {
  if (threadIdx.x == 0) dev_word[0] = v;
}

__global__ void poll_kernel(int* host_word, int v) {
  if (threadIdx.x == 0) __hip_atomic_store(host_word, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ~32 MB streaming read (one wave per 1000-float row, 8192 rows) standing in for a K1 update
__global__ __launch_bounds__(256) void stream_kernel(const float* __restrict__ x, float* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const float* rp = x + row * 1000;
  float m = -1e30f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int col = u * 256 + lane * 4;
    const float4 q = *reinterpret_cast<const float4*>(rp + (col < 1000 ? col : 0));
    m = fmaxf(m, fmaxf(fmaxf(q.x, q.y), fmaxf(q.z, q.w)));
  }
  if (m == 12345.f) sink[row] = m;
}

int main() {
  int* dev_word;
  float *x, *sink;
  CK(hipMalloc(&dev_word, 64));
  CK(hipMalloc(&x, 8192ull * 1000 * 4));
  CK(hipMalloc(&sink, 8192 * 4));
  CK(hipMemset(x, 0, 8192ull * 1000 * 4));
  int* host_word = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&host_word), 64, hipHostMallocMapped | hipHostMallocCoherent));
  int* host_word_dev = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&host_word_dev), host_word, 0));
  int* pinned_out = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned_out), 64, 0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  using clk = std::chrono::steady_clock;
  auto us = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  int seq = 0;
  for (int behind = 0; behind < 2; ++behind) {
    std::vector<double> t_sync, t_memcpy, t_poll;
    for (int rep = 0; rep < 330; ++rep) {
      const bool keep = rep >= 30;
      // sync
      CK(hipStreamSynchronize(s));
      auto a = clk::now();
      if (behind) hipLaunchKernelGGL(stream_kernel, dim3(2048), dim3(256), 0, s, x, sink);
      hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s, dev_word, ++seq);
      CK(hipStreamSynchronize(s));
      auto b = clk::now();
      if (keep) t_sync.push_back(us(a, b));
      // memcpy (.item())
      a = clk::now();
      if (behind) hipLaunchKernelGGL(stream_kernel, dim3(2048), dim3(256), 0, s, x, sink);
      hipLaunchKernelGGL(tiny_kernel, dim3(1), dim3(64), 0, s, dev_word, ++seq);
      CK(hipMemcpyAsync(pinned_out, dev_word, 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      b = clk::now();
      if (pinned_out[0] != seq) printf("memcpy mismatch\n");
      if (keep) t_memcpy.push_back(us(a, b));
      // poll
      CK(hipStreamSynchronize(s));
      const int want = ++seq;
      a = clk::now();
      if (behind) hipLaunchKernelGGL(stream_kernel, dim3(2048), dim3(256), 0, s, x, sink);
      hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, s, host_word_dev, want);
      long spins = 0;
      while (__atomic_load_n(host_word, __ATOMIC_ACQUIRE) != want) {
        if (++spins > 2000000000L) {
          printf("poll timeout\n");
          return 1;
        }
      }
      b = clk::now();
      if (keep) t_poll.push_back(us(a, b));
    }
    CK(hipStreamSynchronize(s));
    printf("{\"behind_stream_kernel\": %d, \"sync_us\": %.2f, \"memcpy_item_us\": %.2f, \"poll_us\": %.2f}\n", behind,
           med(t_sync), med(t_memcpy), med(t_poll));
  }
  return 0;
}
