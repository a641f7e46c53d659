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
#include <map>
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
#include "tea_watchdog.h"

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
// The bookkeeping (communicator states, probe events, the watchdog thread, aborts) lives in
// tea_watchdog.h, driven here by HIP events and RCCL calls; the same template runs under
// ThreadSanitizer with a fake backend (csrc/tests/watchdog_tsan.cpp).

// TORCHEVAL_AMD_RCCL_WATCHDOG=0: no completion events (no deadlines; A/B of the tracking cost)
bool watchdog_enabled() {
  const char* e = std::getenv("TORCHEVAL_AMD_RCCL_WATCHDOG");
  return !(e && std::strcmp(e, "0") == 0);
}

struct HipBackend {
  using Event = hipEvent_t;
  using Stream = hipStream_t;
  using Comm = ncclComm_t;
  Event create_event() {
    hipEvent_t ev = nullptr;
    return hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess ? ev : nullptr;
  }
  bool record(Event ev, Stream s) { return hipEventRecord(ev, s) == hipSuccess; }
  int query(Event ev) {
    const hipError_t q = hipEventQuery(ev);
    return q == hipSuccess ? 0 : q == hipErrorNotReady ? 1 : 2;
  }
  void destroy_event(Event ev) { (void)hipEventDestroy(ev); }
  bool capturing(Stream s) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    return hipStreamIsCapturing(s, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone;
  }
  void set_device(int d) { (void)hipSetDevice(d); }
  void comm_abort(Comm c) { (void)api().comm_abort(c); }
  bool async_error(Comm c, std::string* why) {
    ncclResult_t e = ncclSuccess;
    if (api().async_error(c, &e) == ncclSuccess && e != ncclSuccess && e != ncclInProgress) {
      *why = api().error_string(e);
      return true;
    }
    return false;
  }
  bool tracking_enabled() { return watchdog_enabled(); }
  bool teardown_on_failure() {
    // c10d's default (TORCH_NCCL_ASYNC_ERROR_HANDLING): a collective that failed behind the
    // program's back leaves every later result suspect, so the process goes down loudly
    const char* e = std::getenv("TORCHEVAL_AMD_RCCL_ASYNC_ERROR_HANDLING");
    return !(e && std::strcmp(e, "0") == 0);
  }
  void teardown(const std::string& msg) {
    std::fprintf(stderr, "%s\n", msg.c_str());
    std::fflush(stderr);
    std::abort();
  }
  void fail(const std::string& msg) { throw std::runtime_error(msg); }  // raises to the caller
};

// process-lifetime, never destroyed: a watchdog still running when static destructors start (a
// program that skipped Python's atexit) must not find its state gone
tea_wd::Watchdog<HipBackend>& wd() {
  static HipBackend* b = new HipBackend;
  static tea_wd::Watchdog<HipBackend>* w = new tea_wd::Watchdog<HipBackend>(*b);
  return *w;
}

ncclComm_t usable_comm(int64_t handle) { return wd().usable(handle); }

uint64_t track(int64_t handle, hipStream_t stream, bool force = false) { return wd().track(handle, stream, force); }

void check(ncclResult_t rc, const char* what) {
  TORCH_CHECK(rc == ncclSuccess, "rccl_direct: ", what, " failed: ", api().error_string(rc));
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
  return wd().add(comm, static_cast<int>(device), timeout_ms);
}

void rccl_set_timeout(int64_t handle, int64_t timeout_ms) {
  TORCH_CHECK(timeout_ms > 0, "rccl_direct: timeout must be positive");
  wd().set_timeout(handle, timeout_ms);
}

// 0 ok, 1 failed (abort pending), 2 aborted, 3 destroyed; -1 unknown handle
int64_t rccl_comm_state(int64_t handle) { return wd().state(handle); }

std::string rccl_comm_reason(int64_t handle) { return wd().reason(handle); }

// Abort a communicator this rank still considers healthy because a PEER's failed (the group's
// health vote, parallel/rccl_direct.py agree): marked failed as observed (no teardown) and
// aborted by the watchdog thread like any failure; rccl_wait_aborted waits for it.
void rccl_comm_abort(int64_t handle) { wd().mark_failed(handle, "aborted: another rank's communicator failed", true); }

// wait (bounded) until the background abort of a failed communicator has finished
bool rccl_wait_aborted(int64_t handle, int64_t timeout_ms) { return wd().wait_aborted(handle, timeout_ms); }

// Destroy a healthy communicator after its pending work has drained (bounded); a communicator
// whose work does not drain in time is aborted instead.
void rccl_comm_destroy(int64_t handle) {
  if (!wd().valid(handle)) return;
  if (!wd().drain_for_destroy(handle, std::chrono::seconds(30))) return;  // failed / aborted / pending
  const auto cd = wd().comm_and_device(handle);
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(cd.second);
  const ncclResult_t rc = api().comm_destroy(cd.first);
  (void)hipSetDevice(prev);
  check(rc, "ncclCommDestroy");
}

// Block the host until the newest tracked collective of `handle` completes, at most
// timeout_ms.  false = deadline passed: the communicator is marked failed (observed, so no
// teardown) and aborted in the background.
bool rccl_wait(int64_t handle, int64_t timeout_ms) { return wd().wait(handle, timeout_ms); }

// stop the watchdog (after draining the abort queue); called from Python's atexit hook so the
// thread never outlives the HIP runtime
void rccl_shutdown() { wd().shutdown(); }

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
std::mutex& g_mu = *new std::mutex;  // the plan tables
std::deque<Plan>& g_plans = *new std::deque<Plan>;  // under g_mu; immutable, stable addresses
std::map<int64_t, std::vector<std::vector<int64_t>>>& g_plan_ops =
    *new std::map<int64_t, std::vector<std::vector<int64_t>>>;  // under g_mu: each plan's spec

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

// Plans are immutable and communicator-agnostic, so identical specs share one id (interned by
// ops + views): a metric rebuilt per evaluation epoch (load_state_dict / to() / a new
// instance) finds its layout's plan again instead of growing the table without bound.
std::map<std::vector<int64_t>, int64_t>& g_plan_ids = *new std::map<std::vector<int64_t>, int64_t>;  // under g_mu

std::vector<int64_t> plan_key(const std::vector<std::vector<int64_t>>& ops, const std::vector<std::vector<int64_t>>& views) {
  std::vector<int64_t> k;
  for (const auto& o : ops) {
    k.push_back(static_cast<int64_t>(o.size()));
    k.insert(k.end(), o.begin(), o.end());
  }
  k.push_back(-1);  // ops / views separator
  for (const auto& v : views) {
    k.push_back(static_cast<int64_t>(v.size()));
    k.insert(k.end(), v.begin(), v.end());
  }
  return k;
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

std::vector<ViewSpec> parse_views(const std::vector<std::vector<int64_t>>& views) {
  std::vector<ViewSpec> vs;
  for (const auto& v : views) {
    TORCH_CHECK(v.size() >= 2 && v[1] >= 0, "rccl_plan views: each view is [dtype, elem_off, *shape]");
    vs.push_back({scalar_of_code(v[0]), v[1], std::vector<int64_t>(v.begin() + 2, v.end())});
  }
  return vs;
}

// ops: [kind, src_off, dst_off, count, dtype_code, op_code] each; views: [dtype_code, elem_off,
// *shape] per synced state (may be empty: rccl_plan_set_views once, later); returns a plan id
int64_t rccl_plan_create(const std::vector<std::vector<int64_t>>& ops, const std::vector<std::vector<int64_t>>& views) {
  TORCH_CHECK(!ops.empty(), "rccl_plan_create: empty plan");
  const std::vector<int64_t> key = plan_key(ops, views);
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = g_plan_ids.find(key);
    if (it != g_plan_ids.end()) return it->second;
  }
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
  p.views = parse_views(views);
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_plan_ids.find(key);  // a concurrent caller interned it meanwhile
  if (it != g_plan_ids.end()) return it->second;
  g_plans.push_back(std::move(p));
  const int64_t id = static_cast<int64_t>(g_plans.size()) - 1;
  g_plan_ids.emplace(key, id);
  g_plan_ops.emplace(id, ops);
  return id;
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


// views: [dtype_code, elem_off, *shape] per state, in the order the caller assigns them.  Plans
// are shared (interned): only a plan created without views may receive them (once); setting the
// views it already has is a no-op.
void rccl_plan_set_views(int64_t plan, const std::vector<std::vector<int64_t>>& views) {
  std::vector<ViewSpec> vs = parse_views(views);
  std::lock_guard<std::mutex> lock(g_mu);
  TORCH_CHECK(plan >= 0 && plan < static_cast<int64_t>(g_plans.size()), "rccl_plan_set_views: invalid plan ", plan);
  Plan& p = g_plans[plan];
  auto same = [&]() {
    if (p.views.size() != vs.size()) return false;
    for (size_t i = 0; i < vs.size(); ++i)
      if (p.views[i].dtype != vs[i].dtype || p.views[i].elem_off != vs[i].elem_off || p.views[i].shape != vs[i].shape)
        return false;
    return true;
  };
  if (same()) return;
  TORCH_CHECK(p.views.empty(), "rccl_plan_set_views: plan ", plan, " already has other views (plans are immutable)");
  p.views = std::move(vs);
  // re-key the interned entry: (ops, no views) -> (ops, these views)
  const auto& ops = g_plan_ops.at(plan);
  g_plan_ids.erase(plan_key(ops, {}));
  g_plan_ids.emplace(plan_key(ops, views), plan);
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
  m.def("rccl_comm_abort", &rccl_comm_abort, "abort a healthy communicator whose peer failed (no teardown)",
        py::arg("handle"));
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
  m.def("rccl_plan_create", &rccl_plan_create,
        "register (or find) a sync plan: [[kind, src_off, dst_off, count, dtype, op]] + [[dtype, elem_off, *shape]]",
        py::arg("ops"), py::arg("views") = std::vector<std::vector<int64_t>>{});
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
