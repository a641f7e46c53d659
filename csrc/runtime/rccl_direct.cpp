// Direct RCCL communicators for the metric-state sync.
//
// torch.distributed's collectives cost ~12 us of host time per call on MI355X
// (profiles/rccl_primitive_latency_r3.json: Work objects, stream-sync events, record_stream,
// watchdog bookkeeping), which is most of a small-state sync.  The sync engine's hot path
// (torcheval_amd/parallel/state_buffer.py) instead keeps its own communicator per process
// group: rank 0 draws an ncclUniqueId, the group broadcasts it once through torch.distributed,
// and collectives are enqueued straight onto the caller's current HIP stream.
//
// * Sync plans: a metric's whole sync is ONE grouped call (ncclGroupStart/End, which RCCL
//   launches as one aggregated kernel): every (op, dtype) run of its contiguous state buffer
//   and its device error flag are all-reduced OUT OF PLACE from the live buffer into a result
//   buffer of the same layout.  No snapshot copy, no packing, no host work per state.
// * Failure semantics (c10d-grade, reference toolkit.py:388 runs under the process group's
//   timeout): every enqueue records a completion event that a watchdog thread polls together
//   with ncclCommGetAsyncError.  A collective still pending at its deadline (default: the
//   process group's timeout) or an async error marks the communicator failed and the watchdog
//   aborts it (ncclCommAbort unblocks the kernels).  As in c10d's default async error handling,
//   an unobserved failure then tears the process down (TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0
//   keeps the process and makes the next use of the communicator raise).  A sync with an
//   explicit ``timeout=`` waits for its own completion event on the host and raises
//   TimeoutError at the deadline; the communicator is aborted in the background and rebuilt by
//   the next sync.
//
// The RCCL entry points are resolved at run time from the librccl.so.1 that torch already
// loaded (same library instance, no link-time dependency); if it cannot be found the engine
// keeps using torch.distributed.
//
// Replaces, for the fast sync path, reference torcheval/metrics/toolkit.py:371-391 (pickled
// all_gather_object per sync).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <dlfcn.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>
#include <torch/extension.h>
#include <torch/library.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "tea_kernels.h"
#include "tea_runtime.h"

namespace {

using Clock = std::chrono::steady_clock;

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

const RcclApi& api() {
  static const RcclApi a = [] {
    RcclApi r;
    // the instance torch loaded (matched by soname); load it ourselves only if torch has not
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.comm_abort = reinterpret_cast<decltype(r.comm_abort)>(dlsym(h, "ncclCommAbort"));
    r.async_error = reinterpret_cast<decltype(r.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.all_gather && r.all_reduce && r.comm_destroy && r.comm_abort &&
           r.async_error && r.group_start && r.group_end && r.error_string;
    return r;
  }();
  return a;
}

// ------------------------------------------------------------------ communicator table
enum CommState : int { kOk = 0, kFailed = 1, kAborted = 2, kDestroyed = 3 };

struct Comm {
  ncclComm_t comm = nullptr;
  int device = 0;
  int64_t timeout_ms = 600000;
  std::atomic<int> state{kOk};
  bool observed = false;  // a blocking waiter reported the failure itself (no teardown)
  bool teardown = false;  // decided when the failure is detected (env read then, not at abort)
  std::string reason;
  // completion tracking (under g_mu): one probe event in flight per communicator.  Collectives
  // enqueued while a probe is pending are counted; when the probe retires, the watchdog records
  // a follow-up probe behind them on their stream (hipEventRecord costs ~5 us of host time, so
  // a burst of syncs pays it once, not per sync)
  int probes = 0;
  uint64_t untracked = 0;
  hipStream_t last_stream = nullptr;  // nullptr is a real stream here: the device's null stream
  bool has_last = false;              // a collective was ever enqueued (last_stream is valid)
};

struct Pending {
  hipEvent_t ev;
  int64_t handle;
  Clock::time_point deadline;
  uint64_t seq;  // unique per tracked collective (events are pooled and reused)
};

// Process-lifetime state, never destroyed: a watchdog still running when static destructors
// start (a program that skipped Python's atexit) must not find its mutex or queues gone.
std::mutex& g_mu = *new std::mutex;
std::condition_variable& g_cv = *new std::condition_variable;
std::vector<std::unique_ptr<Comm>>& g_comms = *new std::vector<std::unique_ptr<Comm>>;  // handle = index
std::deque<Pending>& g_pending = *new std::deque<Pending>;
std::vector<hipEvent_t>& g_event_pool = *new std::vector<hipEvent_t>;
std::vector<int64_t>& g_abort_queue = *new std::vector<int64_t>;
uint64_t g_seq = 0;  // under g_mu
std::thread* g_watchdog = nullptr;  // leaked on purpose: joined by rccl_shutdown, never destroyed at exit
bool g_stop = false;

Comm& comm_ref(int64_t handle) {
  TORCH_CHECK(handle >= 0 && handle < static_cast<int64_t>(g_comms.size()) && g_comms[handle],
              "rccl_direct: invalid communicator handle ", handle);
  return *g_comms[handle];
}

ncclComm_t usable_comm(int64_t handle) {
  std::lock_guard<std::mutex> lock(g_mu);
  Comm& c = comm_ref(handle);
  const int s = c.state.load();
  TORCH_CHECK(s == kOk, "rccl_direct: communicator ", handle, " is unusable (",
              s == kDestroyed ? std::string("destroyed") : c.reason, ")");
  return c.comm;
}

void check(ncclResult_t rc, const char* what) {
  TORCH_CHECK(rc == ncclSuccess, "rccl_direct: ", what, " failed: ", api().error_string(rc));
}

bool teardown_on_failure() {
  const char* e = std::getenv("TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING");
  return !(e && std::strcmp(e, "0") == 0);
}

// caller holds g_mu
void mark_failed_locked(int64_t handle, const std::string& why, bool observed) {
  Comm& c = *g_comms[handle];
  int expect = kOk;
  if (!c.state.compare_exchange_strong(expect, kFailed)) return;
  c.reason = why;
  c.observed = observed;
  c.teardown = !observed && teardown_on_failure();
  g_abort_queue.push_back(handle);
  g_cv.notify_all();
}

void abort_comm(int64_t handle) {
  ncclComm_t comm;
  int device;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    comm = g_comms[handle]->comm;
    device = g_comms[handle]->device;
  }
  (void)hipSetDevice(device);
  (void)api().comm_abort(comm);  // unblocks the communicator's kernels, frees its resources
  bool teardown;
  std::string why;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    Comm& c = *g_comms[handle];
    c.state.store(kAborted);
    c.probes = 0;
    c.untracked = 0;
    teardown = c.teardown;
    why = c.reason;
    // the aborted collectives' events complete once the stream drains; drop them unqueried
    for (auto it = g_pending.begin(); it != g_pending.end();) {
      if (it->handle == handle) {
        (void)hipEventDestroy(it->ev);
        it = g_pending.erase(it);
      } else {
        ++it;
      }
    }
    g_cv.notify_all();
  }
  if (teardown) {
    // c10d's default (TORCH_NCCL_ASYNC_ERROR_HANDLING): a collective that failed behind the
    // program's back leaves every later result suspect, so the process goes down loudly
    std::fprintf(stderr,
                 "[torcheval_amd] rccl_direct: communicator %lld failed (%s); aborted it and tearing the process "
                 "down (set TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING=0 to raise on the next sync instead)\n",
                 static_cast<long long>(handle), why.c_str());
    std::fflush(stderr);
    std::abort();
  }
}

bool watchdog_enabled();
void watchdog_loop();

// a probe event from the pool (or a new one); caller does NOT hold g_mu
hipEvent_t take_event() {
  hipEvent_t ev = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    if (!g_event_pool.empty()) {
      ev = g_event_pool.back();
      g_event_pool.pop_back();
    }
  }
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
  return ev;
}

// record a probe for `handle` on `stream` and queue it (caller does NOT hold g_mu and has
// already counted it in c.probes); its sequence number, or 0 when the record failed (count undone)
uint64_t record_probe(int64_t handle, hipStream_t stream) {
  hipEvent_t ev = take_event();
  const bool ok = ev && hipEventRecord(ev, stream) == hipSuccess;
  std::lock_guard<std::mutex> lock(g_mu);
  Comm& c = *g_comms[handle];
  if (!ok) {
    --c.probes;
    if (ev) g_event_pool.push_back(ev);
    return 0;
  }
  const uint64_t seq = ++g_seq;
  g_pending.push_back({ev, handle, Clock::now() + std::chrono::milliseconds(c.timeout_ms), seq});
  if (!g_watchdog) {
    g_stop = false;
    g_watchdog = new std::thread(watchdog_loop);
  }
  g_cv.notify_all();
  return seq;
}

void watchdog_loop() {
  auto last_async_poll = Clock::now();
  struct Probe {
    uint64_t seq;
    hipEvent_t ev;
    int64_t handle;
    Clock::time_point deadline;
    hipError_t q;
  };
  std::vector<Probe> batch;
  std::vector<std::pair<int64_t, hipStream_t>> follow_ups;
  std::unique_lock<std::mutex> lk(g_mu);
  while (!g_stop) {
    if (!g_abort_queue.empty()) {
      const int64_t h = g_abort_queue.back();
      g_abort_queue.pop_back();
      lk.unlock();
      abort_comm(h);
      lk.lock();
      continue;
    }
    if (g_pending.empty()) {
      g_cv.wait_for(lk, std::chrono::milliseconds(200));
      continue;
    }
    // query a snapshot of the oldest probes WITHOUT the lock (hipEventQuery takes the runtime's
    // own locks; holding g_mu here stalled every sync's enqueue behind the scan)
    batch.clear();
    for (const auto& p : g_pending) {
      batch.push_back({p.seq, p.ev, p.handle, p.deadline, hipSuccess});
      if (batch.size() >= 64) break;
    }
    lk.unlock();
    for (auto& b : batch) b.q = hipEventQuery(b.ev);
    const auto now = Clock::now();
    lk.lock();
    follow_ups.clear();
    for (const auto& b : batch) {
      auto it = g_pending.begin();
      while (it != g_pending.end() && it->seq != b.seq) ++it;
      if (it == g_pending.end()) continue;  // retired meanwhile (destroy / abort)
      Comm& c = *g_comms[b.handle];
      if (b.q == hipSuccess) {
        g_event_pool.push_back(it->ev);
        g_pending.erase(it);
        --c.probes;
        if (c.state.load() == kOk && c.probes == 0 && c.untracked > 0 && c.has_last) {
          // collectives enqueued behind the retired probe: probe them now
          c.untracked = 0;
          ++c.probes;
          follow_ups.emplace_back(b.handle, c.last_stream);
        }
        continue;
      }
      if (c.state.load() == kOk) {
        if (b.q != hipErrorNotReady) {
          mark_failed_locked(b.handle, std::string("completion query failed: ") + hipGetErrorString(b.q), false);
        } else if (now > b.deadline) {
          mark_failed_locked(b.handle,
                             "a collective did not complete within " + std::to_string(c.timeout_ms) + " ms", false);
        }
      }
    }
    if (!follow_ups.empty()) {
      lk.unlock();
      for (const auto& fu : follow_ups) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        int dev = 0;
        {
          std::lock_guard<std::mutex> lock(g_mu);
          dev = g_comms[fu.first]->device;
        }
        (void)hipSetDevice(dev);
        // never insert into a stream that is being captured into a graph
        const bool capturing = hipStreamIsCapturing(fu.second, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
        const bool ok = !capturing && record_probe(fu.first, fu.second) != 0;  // a failed record undoes its count
        if (!ok) {
          std::lock_guard<std::mutex> lock(g_mu);
          Comm& c = *g_comms[fu.first];
          if (capturing) --c.probes;
          ++c.untracked;  // probed at the next sync of this communicator
        }
      }
      lk.lock();
    }
    if (now - last_async_poll > std::chrono::milliseconds(10)) {
      last_async_poll = now;
      for (const auto& p : g_pending) {
        Comm& c = *g_comms[p.handle];
        if (c.state.load() != kOk) continue;
        ncclResult_t e = ncclSuccess;
        if (api().async_error(c.comm, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress)
          mark_failed_locked(p.handle, std::string("async error: ") + api().error_string(e), false);
      }
    }
    g_cv.wait_for(lk, std::chrono::microseconds(500));
  }
}

// TORCHEVAL_AMD_RCCL_WATCHDOG=0: no completion events (no deadlines; A/B of the tracking cost)
bool watchdog_enabled() {
  const char* e = std::getenv("TORCHEVAL_AMD_RCCL_WATCHDOG");
  return !(e && std::strcmp(e, "0") == 0);
}

// completion tracking of a collective just enqueued for `handle` on `stream` (caller does NOT
// hold g_mu): a probe event when none is in flight, else counted for the watchdog's follow-up
// probe.  `force`: always record (a host waiter needs a probe behind everything it enqueued:
// the watchdog's follow-up for counted collectives may not be recorded yet).  Returns the
// recorded probe's sequence number (0 = none recorded).
uint64_t track(int64_t handle, hipStream_t stream, bool force = false) {
  if (!watchdog_enabled() && !force) return 0;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    Comm& c = comm_ref(handle);
    c.last_stream = stream;
    c.has_last = true;
    if (c.probes > 0 && !force) {
      ++c.untracked;
      return 0;
    }
    ++c.probes;
    if (force) c.untracked = 0;  // the forced probe covers everything before it on the stream
  }
  const uint64_t seq = record_probe(handle, stream);
  TORCH_CHECK(seq != 0, "rccl_direct: hipEventRecord failed");
  return seq;
}

ncclDataType_t dtype_of(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kLong: return ncclInt64;
    case at::kInt: return ncclInt32;
    case at::kByte:
    case at::kBool: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    default: TORCH_CHECK(false, "rccl_direct: unsupported dtype ", t.scalar_type());
  }
  return ncclUint8;
}

hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

bool rccl_available() { return api().ok; }

// 128-byte ncclUniqueId into a CPU uint8 tensor (rank 0 of the group)
void rccl_unique_id(at::Tensor out) {
  TORCH_CHECK(api().ok, "rccl_direct: librccl.so.1 not available");
  TORCH_CHECK(out.device().is_cpu() && out.scalar_type() == at::kByte && out.is_contiguous() &&
                  out.numel() == NCCL_UNIQUE_ID_BYTES,
              "rccl_direct: unique id buffer must be a contiguous CPU uint8 [128]");
  ncclUniqueId id;
  check(api().get_unique_id(&id), "ncclGetUniqueId");
  std::memcpy(out.data_ptr(), &id, NCCL_UNIQUE_ID_BYTES);
}

// collective over the group (every rank calls it with the same id); returns a handle
int64_t rccl_comm_init(const at::Tensor& id_bytes, int64_t nranks, int64_t rank, int64_t device, int64_t timeout_ms) {
  TORCH_CHECK(api().ok, "rccl_direct: librccl.so.1 not available");
  TORCH_CHECK(id_bytes.device().is_cpu() && id_bytes.scalar_type() == at::kByte && id_bytes.is_contiguous() &&
                  id_bytes.numel() == NCCL_UNIQUE_ID_BYTES,
              "rccl_direct: unique id must be a contiguous CPU uint8 [128]");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rccl_direct: bad rank / nranks");
  TORCH_CHECK(timeout_ms > 0, "rccl_direct: timeout must be positive");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes.data_ptr(), NCCL_UNIQUE_ID_BYTES);
  int prev = 0;
  TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "rccl_direct: hipGetDevice failed");
  TORCH_CHECK(hipSetDevice(static_cast<int>(device)) == hipSuccess, "rccl_direct: hipSetDevice failed");
  ncclComm_t comm = nullptr;
  const ncclResult_t rc = api().comm_init_rank(&comm, static_cast<int>(nranks), id, static_cast<int>(rank));
  (void)hipSetDevice(prev);
  check(rc, "ncclCommInitRank");
  auto c = std::make_unique<Comm>();
  c->comm = comm;
  c->device = static_cast<int>(device);
  c->timeout_ms = timeout_ms;
  std::lock_guard<std::mutex> lock(g_mu);
  g_comms.push_back(std::move(c));
  return static_cast<int64_t>(g_comms.size()) - 1;
}

void rccl_set_timeout(int64_t handle, int64_t timeout_ms) {
  TORCH_CHECK(timeout_ms > 0, "rccl_direct: timeout must be positive");
  std::lock_guard<std::mutex> lock(g_mu);
  comm_ref(handle).timeout_ms = timeout_ms;
}

// 0 ok, 1 failed (abort pending), 2 aborted, 3 destroyed; -1 unknown handle
int64_t rccl_comm_state(int64_t handle) {
  std::lock_guard<std::mutex> lock(g_mu);
  if (handle < 0 || handle >= static_cast<int64_t>(g_comms.size()) || !g_comms[handle]) return -1;
  return g_comms[handle]->state.load();
}

std::string rccl_comm_reason(int64_t handle) {
  std::lock_guard<std::mutex> lock(g_mu);
  return comm_ref(handle).reason;
}

// wait (bounded) until the background abort of a failed communicator has finished
bool rccl_wait_aborted(int64_t handle, int64_t timeout_ms) {
  std::unique_lock<std::mutex> lk(g_mu);
  Comm& c = comm_ref(handle);
  return g_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return c.state.load() >= kAborted; });
}

// Destroy a healthy communicator after its pending work has drained (bounded); a communicator
// whose work does not drain in time is aborted instead.
void rccl_comm_destroy(int64_t handle) {
  ncclComm_t comm;
  int device;
  hipStream_t s_last = nullptr;
  bool has_last = false;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    if (handle >= 0 && handle < static_cast<int64_t>(g_comms.size()) && g_comms[handle] &&
        g_comms[handle]->state.load() == kOk) {
      s_last = g_comms[handle]->last_stream;
      has_last = g_comms[handle]->has_last;
    }
  }
  // a probe behind every collective enqueued so far, tracked or counted (a watchdog follow-up
  // for counted ones may not be recorded yet, so never rely on it here)
  if (has_last) track(handle, s_last, true);
  {
    std::lock_guard<std::mutex> lock(g_mu);
    if (handle < 0 || handle >= static_cast<int64_t>(g_comms.size()) || !g_comms[handle]) return;
    Comm& c = *g_comms[handle];
    if (c.state.load() != kOk) return;  // failed / aborted / destroyed: nothing left to free here
    comm = c.comm;
    device = c.device;
  }
  const auto deadline = Clock::now() + std::chrono::seconds(30);
  for (;;) {
    bool busy = false;
    {
      std::lock_guard<std::mutex> lock(g_mu);
      for (const auto& p : g_pending)
        if (p.handle == handle && hipEventQuery(p.ev) == hipErrorNotReady) busy = true;
    }
    if (!busy) break;
    if (Clock::now() > deadline) {
      std::lock_guard<std::mutex> lock(g_mu);
      mark_failed_locked(handle, "work still pending at destroy", true);
      return;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  {
    std::lock_guard<std::mutex> lock(g_mu);
    g_comms[handle]->state.store(kDestroyed);
    for (auto it = g_pending.begin(); it != g_pending.end();) {
      if (it->handle == handle) {
        g_event_pool.push_back(it->ev);
        it = g_pending.erase(it);
      } else {
        ++it;
      }
    }
  }
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  const ncclResult_t rc = api().comm_destroy(comm);
  (void)hipSetDevice(prev);
  check(rc, "ncclCommDestroy");
}

// Block the host until the newest tracked collective of `handle` completes, at most
// timeout_ms.  false = deadline passed: the communicator is marked failed (observed, so no
// teardown) and aborted in the background.
bool rccl_wait(int64_t handle, int64_t timeout_ms) {
  hipStream_t s_last = nullptr;
  bool has_last = false;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    Comm& c = comm_ref(handle);
    TORCH_CHECK(c.state.load() == kOk, "rccl_direct: communicator ", handle, " is unusable (", c.reason, ")");
    s_last = c.last_stream;
    has_last = c.has_last;
  }
  if (!has_last) return true;  // nothing was ever enqueued
  // our own probe behind the newest collective: "the newest pending entry" is not enough - a
  // counted collective's follow-up probe may still be on its way from the watchdog (that race
  // let a held collective pass as complete)
  const uint64_t seq = track(handle, s_last, true);
  const auto deadline = Clock::now() + std::chrono::milliseconds(timeout_ms);
  for (;;) {
    {
      std::lock_guard<std::mutex> lock(g_mu);
      // still pending? (the watchdog retires completed entries; their events are reused)
      hipEvent_t ev = nullptr;
      for (const auto& p : g_pending)
        if (p.seq == seq) ev = p.ev;
      if (!ev) return g_comms[handle]->state.load() == kOk;
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) return true;
      if (q != hipErrorNotReady || Clock::now() > deadline) {
        mark_failed_locked(handle,
                           q != hipErrorNotReady ? std::string("completion query failed: ") + hipGetErrorString(q)
                                                 : "a collective did not complete within " +
                                                       std::to_string(timeout_ms) + " ms",
                           true);
        return false;
      }
    }
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// stop the watchdog (after draining the abort queue); called from Python's atexit hook so the
// thread never outlives the HIP runtime
void rccl_shutdown() {
  std::thread* t = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    t = g_watchdog;
    g_watchdog = nullptr;
    g_stop = true;
    g_cv.notify_all();
  }
  if (t) {
    t->join();
    delete t;
  }
}

// dst [nranks * src.numel()] <- every rank's src, on the current stream of src's device
void rccl_all_gather(int64_t handle, const at::Tensor& src, at::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous() &&
                  src.scalar_type() == dst.scalar_type() && src.device() == dst.device(),
              "rccl_direct: all_gather needs contiguous device tensors of one dtype");
  TORCH_CHECK(src.numel() > 0 && dst.numel() % src.numel() == 0, "rccl_direct: all_gather size mismatch");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  const hipStream_t s = stream_of(src);
  check(api().all_gather(src.data_ptr(), dst.data_ptr(), static_cast<size_t>(src.numel()), dtype_of(src),
                         usable_comm(handle), s),
        "ncclAllGather");
  track(handle, s);
}

// op 0 sum, 1 max, 2 min; in place, or into `out` (same dtype and size) when given
void rccl_all_reduce(int64_t handle, at::Tensor t, int64_t op, const c10::optional<at::Tensor>& out) {
  TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "rccl_direct: all_reduce needs a contiguous device tensor");
  TORCH_CHECK(op >= 0 && op <= 2, "rccl_direct: op must be 0 (sum), 1 (max) or 2 (min)");
  void* recv = t.data_ptr();
  if (out.has_value()) {
    TORCH_CHECK(out->is_cuda() && out->is_contiguous() && out->scalar_type() == t.scalar_type() &&
                    out->numel() == t.numel() && out->device() == t.device(),
                "rccl_direct: all_reduce out must match the input");
    recv = out->data_ptr();
  }
  if (t.numel() == 0) return;
  const ncclRedOp_t rop = op == 0 ? ncclSum : op == 1 ? ncclMax : ncclMin;
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(t.device());
  const hipStream_t s = stream_of(t);
  check(api().all_reduce(t.data_ptr(), recv, static_cast<size_t>(t.numel()), dtype_of(t), rop, usable_comm(handle),
                         s),
        "ncclAllReduce");
  track(handle, s);
}

// ------------------------------------------------------------------ sync plans
// One entry per RCCL operand of a metric's state buffer: kind 0 = all-reduce of `count`
// elements from src+src_off into dst+dst_off; kind 1 = all-gather of `count` bytes from
// src+src_off into dst+dst_off (nranks * count bytes).  Offsets are bytes.
struct PlanOp {
  int kind;
  int64_t src_off, dst_off, count;
  ncclDataType_t dt;
  ncclRedOp_t op;
  int64_t esize;
};
// A state view of the result buffer (the synced metric's states): dtype, element offset into
// the buffer viewed as that dtype, shape (empty = 0-dim).
struct ViewSpec {
  at::ScalarType dtype;
  int64_t elem_off;
  std::vector<int64_t> shape;
};
struct Plan {
  std::vector<PlanOp> ops;
  int64_t src_end = 0, dst_end_per_rank = 0;
  std::vector<ViewSpec> views;
};
std::deque<Plan>& g_plans = *new std::deque<Plan>;  // under g_mu; immutable, stable addresses

// codes of torcheval_amd.parallel.state_buffer._DT_CODE
bool nccl_dtype(int64_t code, ncclDataType_t* dt, int64_t* es) {
  switch (code) {
    case 0: *dt = ncclFloat32; *es = 4; return true;
    case 1: *dt = ncclFloat16; *es = 2; return true;
    case 2: *dt = ncclBfloat16; *es = 2; return true;
    case 3: *dt = ncclFloat64; *es = 8; return true;
    case 4: *dt = ncclInt64; *es = 8; return true;
    case 5: *dt = ncclInt32; *es = 4; return true;
    case 6: case 7: *dt = ncclUint8; *es = 1; return true;  // bool: or / and through uint8 max / min
    case 8: *dt = ncclInt8; *es = 1; return true;
    default: return false;  // int16: no RCCL type
  }
}

// ops: [kind, src_off, dst_off, count, dtype_code, op_code] each; returns a plan id
int64_t rccl_plan_create(const std::vector<std::vector<int64_t>>& ops) {
  TORCH_CHECK(!ops.empty(), "rccl_plan_create: empty plan");
  Plan p;
  for (const auto& o : ops) {
    TORCH_CHECK(o.size() == 6, "rccl_plan_create: each op is [kind, src_off, dst_off, count, dtype, op]");
    PlanOp q;
    q.kind = static_cast<int>(o[0]);
    q.src_off = o[1];
    q.dst_off = o[2];
    q.count = o[3];
    TORCH_CHECK(q.kind == 0 || q.kind == 1, "rccl_plan_create: kind must be 0 (all-reduce) or 1 (all-gather)");
    TORCH_CHECK(q.src_off >= 0 && q.dst_off >= 0 && q.count > 0, "rccl_plan_create: bad offsets / count");
    if (q.kind == 0) {
      TORCH_CHECK(nccl_dtype(o[4], &q.dt, &q.esize), "rccl_plan_create: dtype code ", o[4], " has no RCCL type");
      TORCH_CHECK(o[5] >= 0 && o[5] <= 2, "rccl_plan_create: op must be 0/1/2");
      q.op = o[5] == 0 ? ncclSum : o[5] == 1 ? ncclMax : ncclMin;
      TORCH_CHECK(q.src_off % q.esize == 0 && q.dst_off % q.esize == 0, "rccl_plan_create: misaligned operand");
      p.dst_end_per_rank = std::max(p.dst_end_per_rank, q.dst_off + q.count * q.esize);
    } else {
      q.dt = ncclUint8;
      q.esize = 1;
      q.op = ncclSum;
    }
    p.src_end = std::max(p.src_end, q.src_off + q.count * q.esize);
    p.ops.push_back(q);
  }
  std::lock_guard<std::mutex> lock(g_mu);
  g_plans.push_back(std::move(p));
  return static_cast<int64_t>(g_plans.size()) - 1;
}

void rccl_group_start() { check(api().group_start(), "ncclGroupStart"); }

// end a group; with track_handle >= 0, record that communicator's completion event on the
// current stream of `device` (the group's kernels are enqueued only here)
void rccl_group_end(int64_t track_handle, int64_t device) {
  check(api().group_end(), "ncclGroupEnd");
  if (track_handle >= 0) track(track_handle, c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device).stream());
}

// Run a plan: src / dst are uint8 buffers on one device; all of the plan's collectives are
// one RCCL group on the current stream.  `grouped`: the caller already opened a group (the
// collection sync); the completion event is then recorded at its rccl_group_end.
void rccl_plan_run(int64_t handle, int64_t plan, const at::Tensor& src, const at::Tensor& dst, int64_t nranks,
                   bool grouped) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.scalar_type() == at::kByte && dst.scalar_type() == at::kByte &&
                  src.is_contiguous() && dst.is_contiguous() && src.device() == dst.device(),
              "rccl_plan_run: contiguous uint8 device buffers on one device expected");
  const Plan* p;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    TORCH_CHECK(plan >= 0 && plan < static_cast<int64_t>(g_plans.size()), "rccl_plan_run: invalid plan ", plan);
    p = &g_plans[plan];
  }
  TORCH_CHECK(src.numel() >= p->src_end, "rccl_plan_run: src smaller than the plan");
  for (const auto& q : p->ops) {
    const int64_t end = q.kind == 0 ? q.dst_off + q.count * q.esize : q.dst_off + nranks * q.count;
    TORCH_CHECK(dst.numel() >= end, "rccl_plan_run: dst smaller than the plan");
  }
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  const hipStream_t s = stream_of(src);
  const ncclComm_t comm = usable_comm(handle);
  const uint8_t* sp = src.data_ptr<uint8_t>();
  uint8_t* dp = dst.data_ptr<uint8_t>();
  // a one-operand plan (e.g. MulticlassAccuracy's counters) needs no group: its ncclGroupEnd
  // launch bookkeeping is pure host cost
  const bool group = p->ops.size() > 1;
  if (group) check(api().group_start(), "ncclGroupStart");
  ncclResult_t rc = ncclSuccess;
  for (const auto& q : p->ops) {
    rc = q.kind == 0 ? api().all_reduce(sp + q.src_off, dp + q.dst_off, static_cast<size_t>(q.count), q.dt, q.op,
                                        comm, s)
                     : api().all_gather(sp + q.src_off, dp + q.dst_off, static_cast<size_t>(q.count), ncclUint8,
                                        comm, s);
    if (rc != ncclSuccess) break;
  }
  const ncclResult_t rc_end = group ? api().group_end() : ncclSuccess;
  check(rc, "sync plan collective");
  check(rc_end, "ncclGroupEnd");
  if (!grouped) track(handle, s);
}

at::ScalarType scalar_of_code(int64_t code) {
  switch (code) {
    case 0: return at::kFloat;
    case 1: return at::kHalf;
    case 2: return at::kBFloat16;
    case 3: return at::kDouble;
    case 4: return at::kLong;
    case 5: return at::kInt;
    case 6: return at::kByte;
    case 7: return at::kBool;
    case 8: return at::kChar;
    case 9: return at::kShort;
    default: TORCH_CHECK(false, "rccl_plan_set_views: bad dtype code ", code);
  }
  return at::kByte;
}

// views: [dtype_code, elem_off, *shape] per state, in the order the caller assigns them
void rccl_plan_set_views(int64_t plan, const std::vector<std::vector<int64_t>>& views) {
  std::vector<ViewSpec> vs;
  for (const auto& v : views) {
    TORCH_CHECK(v.size() >= 2 && v[1] >= 0, "rccl_plan_set_views: each view is [dtype, elem_off, *shape]");
    vs.push_back({scalar_of_code(v[0]), v[1], std::vector<int64_t>(v.begin() + 2, v.end())});
  }
  std::lock_guard<std::mutex> lock(g_mu);
  TORCH_CHECK(plan >= 0 && plan < static_cast<int64_t>(g_plans.size()), "rccl_plan_set_views: invalid plan ", plan);
  g_plans[plan].views = std::move(vs);
}

// The whole direct sync of one metric in one call: a fresh result buffer like `src`, the
// plan's grouped collectives (live buffer -> result, on the current stream), and the synced
// states as views of the result buffer (plan order).  Returns [result, *views].
std::vector<at::Tensor> plan_views(int64_t plan, const at::Tensor& dst);

std::vector<at::Tensor> rccl_plan_sync(int64_t handle, int64_t plan, const at::Tensor& src, int64_t nranks) {
  at::Tensor dst = at::empty_like(src);
  rccl_plan_run(handle, plan, src, dst, nranks, false);
  return plan_views(plan, dst);
}

// [dst, *views]: the plan's state views of a result buffer (no collectives; CPU-testable)
std::vector<at::Tensor> plan_views(int64_t plan, const at::Tensor& dst) {
  TORCH_CHECK(dst.scalar_type() == at::kByte && dst.is_contiguous() && dst.dim() == 1,
              "rccl_plan_views: a contiguous 1-D uint8 buffer expected");
  const Plan* p;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    TORCH_CHECK(plan >= 0 && plan < static_cast<int64_t>(g_plans.size()), "rccl_plan_views: invalid plan ", plan);
    p = &g_plans[plan];
  }
  std::vector<at::Tensor> out;
  out.reserve(p->views.size() + 1);
  out.push_back(dst);
  at::Tensor typed[32];  // one typed view of the result buffer per dtype (ScalarType < 32)
  for (const auto& v : p->views) {
    const int key = static_cast<int>(v.dtype);
    TORCH_CHECK(key >= 0 && key < 32, "rccl_plan_sync: dtype out of range");
    if (!typed[key].defined()) typed[key] = dst.view(v.dtype);
    const at::Tensor& t = typed[key];
    std::vector<int64_t> strides(v.shape.size(), 1);
    int64_t numel = 1;
    for (int64_t d = static_cast<int64_t>(v.shape.size()) - 1; d >= 0; --d) {
      strides[d] = numel;
      numel *= v.shape[d];
    }
    TORCH_CHECK(v.elem_off + numel <= t.numel(), "rccl_plan_views: view outside the buffer");
    out.push_back(t.as_strided(v.shape, strides, v.elem_off));
  }
  return out;
}

// ------------------------------------------------------------------ test support
// A pinned, device-visible host flag and a one-lane kernel that spins on it (bounded by
// max_ms of wall clock): lets a test hold a stream ahead of a collective to exercise the
// deadline path.
int* g_host_flag = nullptr;

int* host_flag() {
  if (!g_host_flag) {
    void* p = nullptr;
    TORCH_CHECK(hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess,
                "test flag: hipHostMalloc failed");
    g_host_flag = static_cast<int*>(p);
    __atomic_store_n(g_host_flag, 1, __ATOMIC_SEQ_CST);
  }
  return g_host_flag;
}

void test_host_flag_set(int64_t v) { __atomic_store_n(host_flag(), static_cast<int>(v), __ATOMIC_SEQ_CST); }

void test_spin_on_host_flag(int64_t device, int64_t max_ms) {
  TORCH_CHECK(max_ms > 0 && max_ms <= 60000, "test_spin_on_host_flag: max_ms in (0, 60000]");
  int* h = host_flag();
  void* d = nullptr;
  TORCH_CHECK(hipHostGetDevicePointer(&d, h, 0) == hipSuccess, "test flag: hipHostGetDevicePointer failed");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device)));
  const hipStream_t s = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device).stream();
  TORCH_CHECK(tea::launch_spin_on_flag(static_cast<const int*>(d), max_ms, s) == 0, "test_spin_on_host_flag: launch");
}

}  // namespace

void tea_register_rccl(pybind11::module_& m) {
  namespace py = pybind11;
  m.def("rccl_available", &rccl_available, "whether librccl.so.1 resolved for the direct communicators");
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId into a CPU uint8 [128]", py::arg("out"));
  m.def("rccl_comm_init", &rccl_comm_init, "ncclCommInitRank (collective over the group) -> handle",
        py::arg("id_bytes"), py::arg("nranks"), py::arg("rank"), py::arg("device"), py::arg("timeout_ms") = 600000);
  m.def("rccl_set_timeout", &rccl_set_timeout, "watchdog deadline of a communicator's collectives",
        py::arg("handle"), py::arg("timeout_ms"));
  m.def("rccl_comm_state", &rccl_comm_state, "0 ok, 1 failed, 2 aborted, 3 destroyed, -1 unknown", py::arg("handle"));
  m.def("rccl_comm_reason", &rccl_comm_reason, "why a communicator failed", py::arg("handle"));
  m.def("rccl_wait_aborted", &rccl_wait_aborted, "wait for the background abort of a failed communicator",
        py::arg("handle"), py::arg("timeout_ms"), py::call_guard<py::gil_scoped_release>());
  m.def("rccl_comm_destroy", &rccl_comm_destroy, "ncclCommDestroy of a handle (after its work drains)",
        py::arg("handle"), py::call_guard<py::gil_scoped_release>());
  m.def("rccl_wait", &rccl_wait, "host wait for the newest collective of a handle; false = deadline passed",
        py::arg("handle"), py::arg("timeout_ms"), py::call_guard<py::gil_scoped_release>());
  m.def("rccl_shutdown", &rccl_shutdown, "stop the watchdog thread", py::call_guard<py::gil_scoped_release>());
  m.def("rccl_all_gather", &rccl_all_gather, "ncclAllGather on the current stream", py::arg("handle"),
        py::arg("src"), py::arg("dst"));
  m.def("rccl_all_reduce", &rccl_all_reduce,
        "ncclAllReduce on the current stream (op 0/1/2 = sum/max/min), in place or into out", py::arg("handle"),
        py::arg("t"), py::arg("op"), py::arg("out") = py::none());
  m.def("rccl_plan_create", &rccl_plan_create, "register a sync plan: [[kind, src_off, dst_off, count, dtype, op]]",
        py::arg("ops"));
  m.def("rccl_plan_run", &rccl_plan_run, "run a sync plan as one RCCL group (src -> dst, out of place)",
        py::arg("handle"), py::arg("plan"), py::arg("src"), py::arg("dst"), py::arg("nranks"),
        py::arg("grouped") = false);
  m.def("rccl_plan_set_views", &rccl_plan_set_views, "register a plan's state views: [[dtype, elem_off, *shape]]",
        py::arg("plan"), py::arg("views"));
  m.def("rccl_plan_sync", &rccl_plan_sync,
        "fresh result buffer + the plan's grouped collectives + the synced state views -> [result, *views]",
        py::arg("handle"), py::arg("plan"), py::arg("src"), py::arg("nranks"));
  m.def("rccl_plan_views", &plan_views, "[buffer, *the plan's state views of it] (no collectives)",
        py::arg("plan"), py::arg("dst"));
  m.def("rccl_group_start", &rccl_group_start, "ncclGroupStart");
  m.def("rccl_group_end", &rccl_group_end, "ncclGroupEnd (+ completion event of track_handle on device's stream)",
        py::arg("track_handle") = -1, py::arg("device") = 0);
  m.def("test_host_flag_set", &test_host_flag_set, "test support: set the pinned host flag", py::arg("value"));
  m.def("test_spin_on_host_flag", &test_spin_on_host_flag,
        "test support: enqueue a kernel spinning until the host flag is nonzero (at most max_ms)", py::arg("device"),
        py::arg("max_ms"));
}

TORCH_LIBRARY_FRAGMENT(torcheval_amd, m) {
  m.def("rccl_all_gather(int handle, Tensor src, Tensor(a!) dst) -> ()");
  m.def("rccl_all_reduce(int handle, Tensor(a!) t, int op, Tensor(b!)? out=None) -> ()");
}

TORCH_LIBRARY_IMPL(torcheval_amd, CUDA, m) {
  m.impl("rccl_all_gather", &rccl_all_gather);
  m.impl("rccl_all_reduce", &rccl_all_reduce);
}
