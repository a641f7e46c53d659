// Low-latency host read of small int32 device tensors (device error flags; csrc/kernels/hostread.hip).
//
// compute() of a metric whose GPU updates validate labels on the device reads one to three
// int32 flag words.  tensor.item() / tolist() pay a D2H copy plus a stream synchronize; here a
// one-lane kernel publishes the words into a pinned, device-mapped host slot and the host spins
// on the slot's sequence word (bounded: past `spin_us` it falls back to a stream synchronize,
// so a read queued behind long GPU work does not burn a core).  A pool of slots, one fresh
// sequence number per read: concurrent readers never share a slot in flight.
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <atomic>
#include <cstring>
#include <chrono>
#include <mutex>
#include <vector>

#include "tea_kernels.h"
#include "tea_runtime.h"

namespace {

constexpr int kSlots = 256;
constexpr int kSlotInts = 16;  // [seq, up to kHostReadWords words, pad]
static_assert(tea::kHostReadWords + 1 <= kSlotInts, "slot too small");

struct SlotPool {
  int32_t* host = nullptr;  // pinned, mapped, coherent
  int32_t* dev = nullptr;   // the device's address of `host`
};

// process-lifetime (never freed: a read may still be in flight at interpreter exit)
SlotPool& pool() {
  static SlotPool* p = [] {
    auto* s = new SlotPool;
    void* h = nullptr;
    TORCH_CHECK(hipHostMalloc(&h, kSlots * kSlotInts * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) ==
                    hipSuccess,
                "hostread: hipHostMalloc failed");
    std::memset(h, 0, kSlots * kSlotInts * sizeof(int32_t));
    void* d = nullptr;
    TORCH_CHECK(hipHostGetDevicePointer(&d, h, 0) == hipSuccess, "hostread: hipHostGetDevicePointer failed");
    s->host = static_cast<int32_t*>(h);
    s->dev = static_cast<int32_t*>(d);
    return s;
  }();
  return *p;
}

std::atomic<uint32_t> g_seq{0};

// the values of a contiguous int32 CUDA tensor of <= kHostReadWords elements, as of the end of
// the work queued before this call on the device's current stream
std::vector<int64_t> read_words(const at::Tensor& t, const at::Tensor* t2, int64_t spin_us) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() >= 1 &&
                  t.numel() + (t2 ? t2->numel() : 0) <= tea::kHostReadWords,
              "read_small_ints: contiguous int32 device tensors of 1..", tea::kHostReadWords, " elements in all");
  if (t2 != nullptr)
    TORCH_CHECK(t2->is_cuda() && t2->device() == t.device() && t2->scalar_type() == at::kInt && t2->is_contiguous() &&
                    t2->numel() >= 1,
                "read_small_ints_pair: the second tensor must be a contiguous int32 tensor on the same device");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(t.device());
  const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
  SlotPool& p = pool();
  // sequence numbers are never 0 (the slots start zeroed)
  uint32_t seq32 = g_seq.fetch_add(1, std::memory_order_relaxed) + 1;
  if (seq32 == 0 || seq32 > 0x7fffffffu) {
    g_seq.store(1);
    seq32 = 1;
  }
  const int32_t seq = static_cast<int32_t>(seq32);
  const int slot = static_cast<int>(seq32 % kSlots);
  int32_t* hs = p.host + slot * kSlotInts;
  const int words1 = static_cast<int>(t.numel()), words2 = t2 ? static_cast<int>(t2->numel()) : 0;
  const int words = words1 + words2;
  TORCH_CHECK(tea::launch_publish_words(t.data_ptr<int32_t>(), words1, p.dev + slot * kSlotInts, seq, s,
                                        t2 ? t2->data_ptr<int32_t>() : nullptr, words2) == 0,
              "read_small_ints: launch failed");
  const auto t0 = std::chrono::steady_clock::now();
  bool seen = false;
  for (uint32_t it = 0;; ++it) {
    if (__atomic_load_n(hs, __ATOMIC_ACQUIRE) == seq) {
      seen = true;
      break;
    }
    if ((it & 255u) == 255u &&
        std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us))
      break;
  }
  if (!seen) {  // long queue ahead: block like .item() would, then the slot is final
    TORCH_CHECK(hipStreamSynchronize(s) == hipSuccess, "read_small_ints: hipStreamSynchronize failed");
    TORCH_CHECK(__atomic_load_n(hs, __ATOMIC_ACQUIRE) == seq, "read_small_ints: slot not published");
  }
  std::vector<int64_t> out(words);
  for (int w = 0; w < words; ++w) out[w] = __atomic_load_n(hs + 1 + w, __ATOMIC_RELAXED);
  return out;
}

std::vector<int64_t> read_small_ints(const at::Tensor& t, int64_t spin_us) { return read_words(t, nullptr, spin_us); }

// two tensors' words in ONE read (one publish launch, one host wait)
std::vector<int64_t> read_small_ints_pair(const at::Tensor& a, const at::Tensor& b, int64_t spin_us) {
  return read_words(a, &b, spin_us);
}

}  // namespace

void tea_register_hostread(pybind11::module_& m) {
  m.def("read_small_ints_pair", &read_small_ints_pair,
        "values of two small int32 device tensors (a's words, then b's) through one pinned-memory publish",
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("spin_us") = 1000,
        pybind11::call_guard<pybind11::gil_scoped_release>());
  m.def("read_small_ints", &read_small_ints,
        "values of a small int32 device tensor through a pinned-memory publish + host spin (low latency)",
        pybind11::arg("t"), pybind11::arg("spin_us") = 1000, pybind11::call_guard<pybind11::gil_scoped_release>());
}
