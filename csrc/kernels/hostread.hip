// Low-latency device -> host read of a few int32 words (device error flags read by compute()).
//
// tensor.item() is a D2H copy plus a stream synchronize: ~17 us on an idle MI355X and ~21 us
// right behind an update kernel, most of it the runtime's completion-signal path.  Here one
// lane stores the words into a pinned, device-mapped host slot with system-scope stores and
// then publishes a sequence number with a system-scope release store; the host spins on that
// word with acquire loads (csrc/runtime/hostread.cpp) - 7 us idle, 12.6 us behind a 6 us
// kernel (profiles/host_poll_latency_r4.json, csrc/bench/host_poll_latency.hip).
#include "tea_common.h"
#include "tea_kernels.h"

namespace tea {

namespace {

// words of src, then (optional) words2 of src2 (two tensors in one read, e.g. FID's two counts)
__global__ __launch_bounds__(kWave) void publish_words_kernel(const int32_t* src, int words, const int32_t* src2,
                                                              int words2, int32_t* slot, int32_t seq) {
  if (threadIdx.x != 0) return;
  for (int w = 0; w < words; ++w) __hip_atomic_store(slot + 1 + w, src[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int w = 0; w < words2; ++w)
    __hip_atomic_store(slot + 1 + words + w, src2[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(slot, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

int launch_publish_words(const int32_t* src, int words, int32_t* slot_dev, int32_t seq, hipStream_t stream,
                         const int32_t* src2, int words2) {
  if (!src || !slot_dev || words < 0 || words2 < 0 || words + words2 > kHostReadWords || (words2 && !src2)) return -1;
  hipLaunchKernelGGL(publish_words_kernel, dim3(1), dim3(kWave), 0, stream, src, words, src2, words2, slot_dev, seq);
  return static_cast<int>(hipGetLastError());
}

}  // namespace tea
