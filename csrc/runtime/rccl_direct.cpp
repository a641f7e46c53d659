// Direct RCCL communicators for the metric-state sync.
//
// torch.distributed's all_gather_into_tensor costs ~12 us of host time per call on MI355X
// (profiles/rccl_primitive_latency_r3.json: Work objects, stream-sync events, record_stream,
// watchdog bookkeeping), which is most of a small-state sync.  The sync engine's hot path
// (torcheval_amd/parallel/state_buffer.py) instead keeps its own communicator per process
// group: rank 0 draws an ncclUniqueId, the group broadcasts it once through torch.distributed,
// and ncclAllGather / ncclAllReduce are then enqueued straight onto the caller's current HIP
// stream.  The RCCL entry points are resolved at run time from the librccl.so.1 that torch
// already loaded (same library instance, no second copy, no link-time dependency); if it
// cannot be found the engine keeps using torch.distributed.
//
// Replaces, for the fast sync path, reference torcheval/metrics/toolkit.py:371-391 (pickled
// all_gather_object per sync).
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <dlfcn.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>
#include <torch/extension.h>
#include <torch/library.h>

#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "tea_runtime.h"

namespace {

struct RcclApi {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
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
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.ok = r.get_unique_id && r.comm_init_rank && r.all_gather && r.all_reduce && r.comm_destroy && r.error_string;
    return r;
  }();
  return a;
}

std::mutex g_mu;
std::vector<ncclComm_t> g_comms;  // handle = index; destroyed slots are nullptr

ncclComm_t comm_of(int64_t handle) {
  std::lock_guard<std::mutex> lock(g_mu);
  TORCH_CHECK(handle >= 0 && handle < static_cast<int64_t>(g_comms.size()) && g_comms[handle] != nullptr,
              "rccl_direct: invalid communicator handle ", handle);
  return g_comms[handle];
}

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
int64_t rccl_comm_init(const at::Tensor& id_bytes, int64_t nranks, int64_t rank, int64_t device) {
  TORCH_CHECK(api().ok, "rccl_direct: librccl.so.1 not available");
  TORCH_CHECK(id_bytes.device().is_cpu() && id_bytes.scalar_type() == at::kByte && id_bytes.is_contiguous() &&
                  id_bytes.numel() == NCCL_UNIQUE_ID_BYTES,
              "rccl_direct: unique id must be a contiguous CPU uint8 [128]");
  TORCH_CHECK(nranks >= 1 && rank >= 0 && rank < nranks, "rccl_direct: bad rank / nranks");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes.data_ptr(), NCCL_UNIQUE_ID_BYTES);
  int prev = 0;
  TORCH_CHECK(hipGetDevice(&prev) == hipSuccess, "rccl_direct: hipGetDevice failed");
  TORCH_CHECK(hipSetDevice(static_cast<int>(device)) == hipSuccess, "rccl_direct: hipSetDevice failed");
  ncclComm_t comm = nullptr;
  const ncclResult_t rc = api().comm_init_rank(&comm, static_cast<int>(nranks), id, static_cast<int>(rank));
  (void)hipSetDevice(prev);
  check(rc, "ncclCommInitRank");
  std::lock_guard<std::mutex> lock(g_mu);
  g_comms.push_back(comm);
  return static_cast<int64_t>(g_comms.size()) - 1;
}

void rccl_comm_destroy(int64_t handle) {
  ncclComm_t comm;
  {
    std::lock_guard<std::mutex> lock(g_mu);
    if (handle < 0 || handle >= static_cast<int64_t>(g_comms.size()) || g_comms[handle] == nullptr) return;
    comm = g_comms[handle];
    g_comms[handle] = nullptr;
  }
  check(api().comm_destroy(comm), "ncclCommDestroy");
}

// dst [nranks * src.numel()] <- every rank's src, on the current stream of src's device
void rccl_all_gather(int64_t handle, const at::Tensor& src, at::Tensor dst) {
  TORCH_CHECK(src.is_cuda() && dst.is_cuda() && src.is_contiguous() && dst.is_contiguous() &&
                  src.scalar_type() == dst.scalar_type() && src.device() == dst.device(),
              "rccl_direct: all_gather needs contiguous device tensors of one dtype");
  TORCH_CHECK(src.numel() > 0 && dst.numel() % src.numel() == 0, "rccl_direct: all_gather size mismatch");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  check(api().all_gather(src.data_ptr(), dst.data_ptr(), static_cast<size_t>(src.numel()), dtype_of(src),
                         comm_of(handle), stream_of(src)),
        "ncclAllGather");
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
  check(api().all_reduce(t.data_ptr(), recv, static_cast<size_t>(t.numel()), dtype_of(t), rop, comm_of(handle),
                         stream_of(t)),
        "ncclAllReduce");
}

}  // namespace

void tea_register_rccl(pybind11::module_& m) {
  namespace py = pybind11;
  m.def("rccl_available", &rccl_available, "whether librccl.so.1 resolved for the direct communicators");
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId into a CPU uint8 [128]", py::arg("out"));
  m.def("rccl_comm_init", &rccl_comm_init, "ncclCommInitRank (collective over the group) -> handle",
        py::arg("id_bytes"), py::arg("nranks"), py::arg("rank"), py::arg("device"));
  m.def("rccl_comm_destroy", &rccl_comm_destroy, "ncclCommDestroy of a handle", py::arg("handle"));
  m.def("rccl_all_gather", &rccl_all_gather, "ncclAllGather on the current stream", py::arg("handle"),
        py::arg("src"), py::arg("dst"));
  m.def("rccl_all_reduce", &rccl_all_reduce,
        "ncclAllReduce on the current stream (op 0/1/2 = sum/max/min), in place or into out", py::arg("handle"),
        py::arg("t"), py::arg("op"), py::arg("out") = py::none());
}

TORCH_LIBRARY_FRAGMENT(torcheval_amd, m) {
  m.def("rccl_all_gather(int handle, Tensor src, Tensor(a!) dst) -> ()");
  m.def("rccl_all_reduce(int handle, Tensor(a!) t, int op, Tensor(b!)? out=None) -> ()");
}

TORCH_LIBRARY_IMPL(torcheval_amd, CUDA, m) {
  m.impl("rccl_all_gather", &rccl_all_gather);
  m.impl("rccl_all_reduce", &rccl_all_reduce);
}
