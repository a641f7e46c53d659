// pybind11 entry points of torcheval_amd._C.
//
// This TU is the only one that includes torch headers: it validates tensors, picks the
// current HIP stream of the tensor's device and forwards raw pointers to the launchers in
// csrc/kernels/*.hip.  Every op fails loudly (TORCH_CHECK) on shapes/dtypes the kernels do
// not assume, so no kernel ever runs with a mismatched grid.
#include <torch/extension.h>

#include <cstdlib>
#include <cstring>
#include <atomic>
#include <array>
#include <mutex>
#include <unordered_map>

#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "tea_kernels.h"
#include "tea_runtime.h"

namespace {

using at::Tensor;
using c10::optional;

tea::DType dt_of(const Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return tea::DType::f32;
    case at::kHalf: return tea::DType::f16;
    case at::kBFloat16: return tea::DType::bf16;
    case at::kDouble: return tea::DType::f64;
    case at::kLong: return tea::DType::i64;
    case at::kInt: return tea::DType::i32;
    case at::kByte: return tea::DType::u8;
    case at::kBool: return tea::DType::b8;
    case at::kChar: return tea::DType::i8;
    case at::kShort: return tea::DType::i16;
    default: TORCH_CHECK(false, "torcheval_amd._C: unsupported dtype ", t.scalar_type());
  }
  return tea::DType::f32;
}

hipStream_t stream_for(const Tensor& t) {
  return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(t.device().index()).stream();
}

void check_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "torcheval_amd._C: ", name, " must be a ROCm (cuda) tensor");
}

float* f32_out(const optional<Tensor>& t, const Tensor& ref, int64_t numel, const char* name) {
  if (!t.has_value()) return nullptr;
  const Tensor& x = *t;
  TORCH_CHECK(x.scalar_type() == at::kFloat, "torcheval_amd._C: ", name, " must be float32");
  TORCH_CHECK(x.is_contiguous(), "torcheval_amd._C: ", name, " must be contiguous");
  TORCH_CHECK(x.device() == ref.device(), "torcheval_amd._C: ", name, " on wrong device");
  TORCH_CHECK(x.numel() == numel, "torcheval_amd._C: ", name, " must have ", numel,
              " elements, got ", x.numel());
  return x.data_ptr<float>();
}

// Per-(device, stream) workspace for tea_fold.h: zeroed once, self-cleaning after every
// launch, so all kernels on one stream can share it (stream order serialises them).
// Allocate (warm up) before any HIP-graph capture that uses it.
unsigned long long* fold_workspace(const Tensor& like, hipStream_t stream) {
  static std::mutex mu;
  // process-lifetime (never destroyed): no device free from a static destructor at exit, after
  // the HIP runtime or an attached profiler has already shut down
  static auto& cache = *new std::unordered_map<uint64_t, Tensor>();
  const uint64_t key = (static_cast<uint64_t>(like.device().index()) << 56) ^
                       reinterpret_cast<uint64_t>(stream);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it == cache.end()) {
    Tensor ws = at::zeros({16 * tea::kFoldCells},
                          at::TensorOptions().dtype(at::kLong).device(like.device()));
    it = cache.emplace(key, ws).first;
  }
  return reinterpret_cast<unsigned long long*>(it->second.data_ptr<int64_t>());
}

// Self-cleaning scratch: zeroed once per (device, stream, slot), grown on demand; kernels that
// use it leave it zeroed again, so no memset launch per call.
void* zeroed_workspace(const Tensor& like, hipStream_t stream, int64_t bytes, int slot,
                       int64_t* capacity = nullptr) {
  static std::mutex mu;
  // process-lifetime (never destroyed): no device free from a static destructor at exit, after
  // the HIP runtime or an attached profiler has already shut down
  static auto& cache = *new std::unordered_map<uint64_t, Tensor>();
  const uint64_t key = (static_cast<uint64_t>(like.device().index()) << 56) ^
                       (static_cast<uint64_t>(slot) << 48) ^ reinterpret_cast<uint64_t>(stream);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it == cache.end() || it->second.numel() < bytes) {
    Tensor ws = at::zeros({std::max<int64_t>(bytes, 1 << 16)},
                          at::TensorOptions().dtype(at::kByte).device(like.device()));
    if (it == cache.end()) it = cache.emplace(key, ws).first;
    else it->second = ws;
  }
  if (capacity) *capacity = it->second.numel();
  return it->second.data_ptr();
}

// Scratch that kernels overwrite before reading (no zeroing contract): per (device, stream,
// slot), grown on demand.
void* scratch_workspace(const Tensor& like, hipStream_t stream, int64_t bytes, int slot) {
  static std::mutex mu;
  // process-lifetime (never destroyed): no device free from a static destructor at exit, after
  // the HIP runtime or an attached profiler has already shut down
  static auto& cache = *new std::unordered_map<uint64_t, Tensor>();
  const uint64_t key = (static_cast<uint64_t>(like.device().index()) << 56) ^
                       (static_cast<uint64_t>(slot) << 48) ^ reinterpret_cast<uint64_t>(stream);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it == cache.end() || it->second.numel() < bytes) {
    Tensor ws = at::empty({std::max<int64_t>(bytes, 1 << 16)},
                          at::TensorOptions().dtype(at::kByte).device(like.device()));
    if (it == cache.end()) it = cache.emplace(key, ws).first;
    else it->second = ws;
  }
  return it->second.data_ptr();
}

void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "torcheval_amd._C: ", what, " launch failed (code ", rc, ")");
}

// ---------------------------------------------------------------- K1 classification counts
void cls_counts(const Tensor& input, const Tensor& target, int64_t k, int64_t num_classes,
                const optional<Tensor>& micro_correct, const optional<Tensor>& micro_total,
                const optional<Tensor>& cls_correct, const optional<Tensor>& cls_label,
                const optional<Tensor>& cls_pred, const optional<Tensor>& confusion,
                const optional<Tensor>& err, int64_t max_blocks,
                const optional<Tensor>& micro_incorrect, const optional<Tensor>& micro_total2,
                const optional<Tensor>& cls_fp) {
  check_gpu(input, "input");
  check_gpu(target, "target");
  TORCH_CHECK(target.dim() == 1, "cls_counts: target must be 1-D");
  TORCH_CHECK(input.dim() == 1 || input.dim() == 2, "cls_counts: input must be 1-D or 2-D");
  TORCH_CHECK(input.size(0) == target.size(0), "cls_counts: first dims differ");
  TORCH_CHECK(target.is_contiguous(), "cls_counts: target must be contiguous");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  tea::ClsCountsArgs a;
  Tensor in = input;
  if (input.dim() == 2) {
    if (in.stride(1) != 1) in = in.contiguous();
    a.c = in.size(1);
    a.row_stride = in.stride(0);
    TORCH_CHECK(a.c < (int64_t(1) << 31), "cls_counts: too many classes");
    TORCH_CHECK(k >= 1 && k <= a.c || a.c == 0, "cls_counts: k out of range");
    if (num_classes <= 0) num_classes = a.c;
    TORCH_CHECK(num_classes == a.c, "cls_counts: num_classes must match input.size(1)");
  } else {
    if (!in.is_contiguous()) in = in.contiguous();
    TORCH_CHECK(k == 1, "cls_counts: k > 1 needs 2-D scores");
  }
  const int64_t C = num_classes;
  a.input = in.data_ptr();
  a.in_dt = dt_of(in);
  a.n = in.size(0);
  a.target = target.data_ptr();
  a.tg_dt = dt_of(target);
  a.k = static_cast<int>(k);
  a.num_classes = C;
  a.micro_correct = f32_out(micro_correct, input, 1, "micro_correct");
  a.micro_total = f32_out(micro_total, input, 1, "micro_total");
  a.cls_correct = f32_out(cls_correct, input, C, "cls_correct");
  a.cls_label = f32_out(cls_label, input, C, "cls_label");
  a.cls_pred = f32_out(cls_pred, input, C, "cls_pred");
  a.confusion = f32_out(confusion, input, C * C, "confusion");
  a.micro_incorrect = f32_out(micro_incorrect, input, 1, "micro_incorrect");
  a.micro_total2 = f32_out(micro_total2, input, 1, "micro_total2");
  a.cls_fp = f32_out(cls_fp, input, C, "cls_fp");
  TORCH_CHECK(!(k > 1 && (a.cls_pred || a.confusion || a.cls_fp)),
              "cls_counts: predictions are undefined for k > 1");
  TORCH_CHECK((a.cls_correct || a.cls_label || a.cls_pred || a.confusion || a.cls_fp) == false ||
                  C > 0,
              "cls_counts: num_classes required for histograms");
  if (err.has_value()) {
    TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= 1 && err->device() == input.device(),
                "cls_counts: err must be an int32 tensor on the input device");
    a.err = err->data_ptr<int>();
    if (err->numel() >= 3) a.err_max = a.err + 1;  // [flags, max bad target, max bad prediction]
    a.check_target = 1;
  }
  a.max_blocks = static_cast<int>(max_blocks);
  const hipStream_t stream = stream_for(input);
  if (a.micro_correct || a.micro_incorrect) a.fold_ws = fold_workspace(input, stream);
  const int rc = tea::launch_cls_counts(a, stream);
  TORCH_CHECK(rc != -1, "cls_counts: unsupported input dtype ", input.scalar_type());
  check_launch(rc, "cls_counts");
}

// Lean entry of the north-star update (MulticlassAccuracy micro, k=1): every precondition of
// the wide K1 launch is tested here, and anything unusual returns false so the caller takes
// the general Python path (which raises the reference's own errors).  One pybind call with
// four positional tensors instead of the 15-argument cls_counts plus its Python-side checks.
bool micro_accuracy_update(const Tensor& input, const Tensor& target, const Tensor& correct,
                           const Tensor& total, int64_t num_classes, const optional<Tensor>& pend) {
  if (!input.is_cuda() || input.dim() != 2 || target.dim() != 1) return false;
  const int64_t n = input.size(0), c = input.size(1);
  if (target.size(0) != n || c <= 0 || c >= (int64_t(1) << 31) || input.stride(1) != 1) return false;
  // a metric built with num_classes only accepts [N, num_classes] scores: anything else goes
  // to the Python path, which raises the reference's ValueError (accuracy.py:340-346)
  if (num_classes > 0 && c != num_classes) return false;
  const auto st = input.scalar_type();
  if (st != at::kFloat && st != at::kBFloat16 && st != at::kHalf) return false;
  switch (target.scalar_type()) {
    case at::kLong: case at::kInt: case at::kShort: case at::kChar: case at::kByte: case at::kBool:
      break;
    default: return false;
  }
  if (!target.is_contiguous()) return false;
  const auto dev = input.device();
  if (target.device() != dev || correct.device() != dev || total.device() != dev) return false;
  if (correct.scalar_type() != at::kFloat || total.scalar_type() != at::kFloat ||
      correct.numel() != 1 || total.numel() != 1)
    return false;
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(dev);
  tea::ClsCountsArgs a;
  a.input = input.data_ptr();
  a.in_dt = dt_of(input);
  a.n = n;
  a.c = c;
  a.row_stride = input.stride(0);
  a.target = target.data_ptr();
  a.tg_dt = dt_of(target);
  a.k = 1;
  a.num_classes = c;
  a.micro_correct = correct.data_ptr<float>();
  a.micro_total = total.data_ptr<float>();
  const hipStream_t stream = stream_for(input);
  if (pend.has_value()) {
    if (pend->scalar_type() != at::kLong || pend->numel() < tea::kPendCells * tea::kPendStride ||
        pend->device() != dev || !pend->is_contiguous())
      return false;
    a.pend = reinterpret_cast<unsigned long long*>(pend->data_ptr<int64_t>());
  } else {
    a.fold_ws = fold_workspace(input, stream);
  }
  check_launch(tea::launch_cls_counts(a, stream), "micro_accuracy_update");
  return true;
}

// Fold the K1 micro kernel's pending cells into ``correct`` (cells zeroed); with ``out``, also
// write correct / total there: the deferred fold and the accuracy division in one launch.
void micro_accuracy_finish(const Tensor& pend, const Tensor& correct, const Tensor& total,
                           const optional<Tensor>& out) {
  check_gpu(pend, "pend");
  TORCH_CHECK(pend.scalar_type() == at::kLong && pend.is_contiguous() &&
                  pend.numel() >= tea::kPendCells * tea::kPendStride,
              "micro_accuracy_finish: pend must be int64 [>= 512]");
  TORCH_CHECK(correct.scalar_type() == at::kFloat && total.scalar_type() == at::kFloat && correct.numel() == 1 &&
                  total.numel() == 1 && correct.device() == pend.device() && total.device() == pend.device(),
              "micro_accuracy_finish: float32 scalar states on the pending cells' device");
  float* o = nullptr;
  if (out.has_value()) {
    TORCH_CHECK(out->scalar_type() == at::kFloat && out->numel() == 1 && out->device() == pend.device(),
                "micro_accuracy_finish: out must be a float32 scalar");
    o = out->data_ptr<float>();
  }
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(pend.device());
  check_launch(tea::launch_micro_finish(reinterpret_cast<unsigned long long*>(pend.data_ptr<int64_t>()),
                                        correct.data_ptr<float>(), total.data_ptr<float>(), o, stream_for(pend)),
               "micro_accuracy_finish");
}

// ---------------------------------------------------------------- K10 rank-of-target scores
Tensor rank_scores(const Tensor& input, const Tensor& target, int64_t mode, int64_t k,
                   const optional<Tensor>& err) {
  check_gpu(input, "input");
  check_gpu(target, "target");
  TORCH_CHECK(input.dim() == 2 && target.dim() == 1 && input.size(0) == target.size(0),
              "rank_scores: input [n, c] and target [n] expected");
  TORCH_CHECK(mode == 0 || mode == 1, "rank_scores: mode must be 0 (hit) or 1 (reciprocal)");
  TORCH_CHECK(input.size(1) < (int64_t(1) << 31), "rank_scores: too many columns");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  Tensor in = input.stride(1) == 1 ? input : input.contiguous();
  Tensor tg = target.contiguous();
  tea::RankArgs a;
  a.input = in.data_ptr();
  a.in_dt = dt_of(in);
  a.n = in.size(0);
  a.c = in.size(1);
  a.row_stride = in.stride(0);
  a.target = tg.data_ptr();
  a.tg_dt = dt_of(tg);
  a.mode = static_cast<int>(mode);
  a.k = static_cast<int>(k);
  Tensor out = at::empty({a.n}, input.options().dtype(at::kFloat));
  a.out = out.data_ptr<float>();
  if (err.has_value()) {
    TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= 1 && err->device() == input.device(),
                "rank_scores: err must be an int32 tensor on the input device");
    a.err = err->data_ptr<int>();
  }
  const int rc = tea::launch_rank_scores(a, stream_for(input));
  TORCH_CHECK(rc != -1, "rank_scores: unsupported input dtype ", input.scalar_type());
  check_launch(rc, "rank_scores");
  return out;
}

void binary_counts(const Tensor& input, const Tensor& target, const optional<Tensor>& weight,
                   double threshold, const optional<Tensor>& tp, const optional<Tensor>& fp,
                   const optional<Tensor>& tn, const optional<Tensor>& fn,
                   const optional<Tensor>& total, int64_t strict, int64_t max_blocks,
                   const optional<Tensor>& tp2, const optional<Tensor>& fp2,
                   const optional<Tensor>& tn2, const optional<Tensor>& fn2) {
  check_gpu(input, "input");
  check_gpu(target, "target");
  TORCH_CHECK(input.numel() == target.numel(), "binary_counts: size mismatch");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  Tensor in = input.contiguous();
  Tensor tg = target.contiguous();
  Tensor w;
  tea::BinaryCountsArgs a;
  if (weight.has_value()) {
    w = weight->contiguous();
    TORCH_CHECK(w.numel() == in.numel(), "binary_counts: weight size mismatch");
    a.weight = w.data_ptr();
    a.w_dt = dt_of(w);
  }
  a.input = in.data_ptr();
  a.in_dt = dt_of(in);
  a.target = tg.data_ptr();
  a.tg_dt = dt_of(tg);
  a.n = in.numel();
  a.threshold = static_cast<float>(threshold);
  a.strict_binary = static_cast<int>(strict);
  a.out[0] = f32_out(tp, input, 1, "tp");
  a.out[1] = f32_out(fp, input, 1, "fp");
  a.out[2] = f32_out(tn, input, 1, "tn");
  a.out[3] = f32_out(fn, input, 1, "fn");
  a.total = f32_out(total, input, 1, "total");
  a.out2[0] = f32_out(tp2, input, 1, "tp2");
  a.out2[1] = f32_out(fp2, input, 1, "fp2");
  a.out2[2] = f32_out(tn2, input, 1, "tn2");
  a.out2[3] = f32_out(fn2, input, 1, "fn2");
  a.max_blocks = static_cast<int>(max_blocks);
  check_launch(tea::launch_binary_counts(a, stream_for(input)), "binary_counts");
}

// ---------------------------------------------------------------- K3 sort-scan
// sorted/order: [rows, n] (descending scores and their permutation); target: [rows, n] binary
// targets or (class_mode) [n] labels; weight: optional [rows, n]; outputs float64 [rows].
// shared argument set-up of the K3 scans (auc_scan, the K3c curve passes); tg / w keep any
// contiguous copies alive for the launch
static tea::AucScanArgs scan_args(const Tensor& sorted, const Tensor& order, const Tensor& target,
                                  const optional<Tensor>& weight, bool class_mode, int64_t payload_kind,
                                  Tensor& tg, Tensor& w, const char* who) {
  check_gpu(sorted, "sorted");
  TORCH_CHECK(sorted.dim() == 2 && order.dim() == 2 && sorted.sizes() == order.sizes(),
              who, ": sorted/order must be [rows, n]");
  TORCH_CHECK(sorted.stride(1) == 1 && order.stride(1) == 1, who, ": rows must be contiguous");
  TORCH_CHECK(sorted.scalar_type() == at::kFloat || sorted.scalar_type() == at::kDouble,
              who, ": scores must be float32/float64");
  TORCH_CHECK(order.scalar_type() == at::kLong || order.scalar_type() == at::kInt,
              who, ": order must be int64 or int32");
  const int64_t rows = sorted.size(0), n = sorted.size(1);
  tea::AucScanArgs a;
  a.sorted = sorted.data_ptr();
  a.key_dt = dt_of(sorted);
  a.key_stride = sorted.stride(0);
  if (order.scalar_type() == at::kLong) a.order = order.data_ptr<int64_t>();
  else a.order32 = order.data_ptr<int32_t>();
  a.order_stride = order.stride(0);
  tg = target;
  // with a payload (kinds 1, 2) the sort carried the targets / labels and no kernel reads
  // `target` (tea_scan.h sample_ab): no layout copy for it (a transposed [n, L] multilabel
  // target used to cost one strided ATen transpose per launch here)
  const bool read_target = payload_kind == 0;
  if (class_mode) {
    TORCH_CHECK(tg.dim() == 1 && tg.size(0) == n, who, ": class-mode target must be [n]");
    if (read_target) tg = tg.contiguous();
  } else {
    TORCH_CHECK(tg.dim() == 2 && tg.size(0) == rows && tg.size(1) == n, who, ": target must be [rows, n]");
    if (read_target && tg.stride(1) != 1) tg = tg.contiguous();
    a.target_stride = tg.stride(0);
  }
  a.target = tg.data_ptr();
  a.tg_dt = dt_of(tg);
  if (weight.has_value()) {
    w = *weight;
    TORCH_CHECK(w.dim() == 2 && w.size(0) == rows && w.size(1) == n, who, ": weight must be [rows, n]");
    if (w.stride(1) != 1) w = w.contiguous();
    a.weight = w.data_ptr();
    a.w_dt = dt_of(w);
    a.weight_stride = w.stride(0);
  }
  a.class_mode = class_mode ? 1 : 0;
  TORCH_CHECK(payload_kind == 0 || (order.scalar_type() == at::kInt && !weight.has_value()),
              who, ": a payload order must be int32 and unweighted");
  a.payload_kind = static_cast<int>(payload_kind);
  a.rows = rows;
  a.n = n;
  return a;
}

void auc_scan(const Tensor& sorted, const Tensor& order, const Tensor& target,
              const optional<Tensor>& weight, bool class_mode, const optional<Tensor>& out_auroc,
              const optional<Tensor>& out_auprc, const optional<Tensor>& init,
              const optional<Tensor>& out_raw, int64_t payload_kind, const optional<Tensor>& tsum) {
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(sorted.device());
  Tensor tg, w;
  tea::AucScanArgs a = scan_args(sorted, order, target, weight, class_mode, payload_kind, tg, w, "auc_scan");
  const int64_t rows = a.rows, n = a.n;
  if (tsum.has_value()) {  // tile totals folded by sort_desc (payload kinds 1 / 2 only)
    TORCH_CHECK(payload_kind != 0 && tsum->scalar_type() == at::kDouble && tsum->is_contiguous() &&
                    tsum->device() == sorted.device() && tsum->numel() == rows * ((n + 1023) / 1024) * 2,
                "auc_scan: tsum must be sort_desc's float64 [rows, ceil(n / 1024), 2] fold of a payload sort");
    a.tsum_ext = tsum->data_ptr<double>();
  }
  auto f64_out = [&](const optional<Tensor>& t, const char* name) -> double* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kDouble && t->is_contiguous() && t->numel() == rows &&
                    t->device() == sorted.device(),
                "auc_scan: ", name, " must be a contiguous float64 [rows] tensor");
    return t->data_ptr<double>();
  };
  a.out_auroc = f64_out(out_auroc, "out_auroc");
  a.out_auprc = f64_out(out_auprc, "out_auprc");
  if (init.has_value()) {
    TORCH_CHECK(init->scalar_type() == at::kDouble && init->is_contiguous() && init->numel() == 2 * rows,
                "auc_scan: init must be contiguous float64 [rows, 2]");
    a.init = init->data_ptr<double>();
  }
  if (out_raw.has_value()) {
    TORCH_CHECK(out_raw->scalar_type() == at::kDouble && out_raw->is_contiguous() && out_raw->numel() == 4 * rows,
                "auc_scan: out_raw must be contiguous float64 [rows, 4]");
    a.out_raw = out_raw->data_ptr<double>();
  }
  // the latest onesweep sort's timeout word on this stream (zero when none ever ran or it was clean)
  a.sort_fault = static_cast<const uint32_t*>(zeroed_workspace(sorted, stream_for(sorted), 16 * 4, 10)) + 8;
  Tensor ws = at::empty({tea::auc_scan_workspace_bytes(rows, n)},
                        at::TensorOptions().dtype(at::kByte).device(sorted.device()));
  check_launch(tea::launch_auc_scan(a, ws.data_ptr(), stream_for(sorted)), "auc_scan");
}

// ---------------------------------------------------------------- K3c curves
int64_t curve_workspace_bytes(int64_t rows, int64_t n, bool rafp) {
  return tea::curve_workspace_bytes(rows, n, rafp);
}

// passes 1-2: tile totals / tie-group tails and per-row scans into `workspace`; G_r -> sizes
void curve_count(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode,
                 int64_t payload_kind, const Tensor& workspace, const Tensor& sizes) {
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(sorted.device());
  Tensor tg, w;
  tea::AucScanArgs a = scan_args(sorted, order, target, c10::nullopt, class_mode, payload_kind, tg, w, "curve_count");
  TORCH_CHECK(workspace.is_contiguous() && workspace.scalar_type() == at::kByte &&
                  workspace.numel() >= tea::curve_workspace_bytes(a.rows, a.n, false),
              "curve_count: workspace too small");
  TORCH_CHECK(sizes.scalar_type() == at::kLong && sizes.is_contiguous() && sizes.numel() == a.rows,
              "curve_count: sizes must be contiguous int64 [rows]");
  a.sizes = sizes.data_ptr<int64_t>();
  check_launch(tea::launch_curve_count(a, workspace.data_ptr(), false, stream_for(sorted)), "curve_count");
}

// pass 3: ascending curves into the exact outputs (row_off: int64 [rows] threshold offsets)
void curve_emit(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode,
                int64_t payload_kind, const Tensor& workspace, const Tensor& sizes, const Tensor& row_off,
                const Tensor& out_prec, const Tensor& out_rec, const Tensor& out_thr) {
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(sorted.device());
  Tensor tg, w;
  tea::AucScanArgs a = scan_args(sorted, order, target, c10::nullopt, class_mode, payload_kind, tg, w, "curve_emit");
  TORCH_CHECK(workspace.is_contiguous() && workspace.numel() >= tea::curve_workspace_bytes(a.rows, a.n, false),
              "curve_emit: workspace too small");
  TORCH_CHECK(sizes.scalar_type() == at::kLong && sizes.numel() == a.rows && row_off.scalar_type() == at::kLong &&
                  row_off.numel() == a.rows && row_off.is_contiguous() && row_off.device() == sorted.device(),
              "curve_emit: sizes / row_off must be int64 [rows] on the device");
  TORCH_CHECK(out_prec.scalar_type() == at::kFloat && out_rec.scalar_type() == at::kFloat &&
                  out_prec.is_contiguous() && out_rec.is_contiguous() && out_thr.is_contiguous() &&
                  out_thr.scalar_type() == sorted.scalar_type() && out_prec.numel() == out_thr.numel() + a.rows &&
                  out_rec.numel() == out_prec.numel(),
              "curve_emit: outputs must be contiguous f32 [sum G + rows] x2 and key-dtype [sum G]");
  a.sizes = sizes.data_ptr<int64_t>();
  a.row_off = row_off.data_ptr<int64_t>();
  a.out_prec = out_prec.data_ptr<float>();
  a.out_rec = out_rec.data_ptr<float>();
  a.out_thr = out_thr.data_ptr();
  check_launch(tea::launch_curve_emit(a, workspace.data_ptr(), false, stream_for(sorted)), "curve_emit");
}

// recall at fixed precision per row, no host synchronisation
void rafp(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode,
          int64_t payload_kind, double min_precision, const Tensor& out_max_recall, const Tensor& out_best_thr) {
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(sorted.device());
  Tensor tg, w;
  tea::AucScanArgs a = scan_args(sorted, order, target, c10::nullopt, class_mode, payload_kind, tg, w, "rafp");
  TORCH_CHECK(out_max_recall.scalar_type() == at::kFloat && out_max_recall.is_contiguous() &&
                  out_max_recall.numel() == a.rows && out_best_thr.scalar_type() == sorted.scalar_type() &&
                  out_best_thr.is_contiguous() && out_best_thr.numel() == a.rows,
              "rafp: outputs must be contiguous f32 [rows] and key-dtype [rows]");
  Tensor sizes = at::empty({a.rows}, sorted.options().dtype(at::kLong));
  Tensor ws = at::empty({tea::curve_workspace_bytes(a.rows, a.n, true)}, sorted.options().dtype(at::kByte));
  a.sizes = sizes.data_ptr<int64_t>();
  a.min_precision = static_cast<float>(min_precision);
  a.out_max_recall = out_max_recall.data_ptr<float>();
  a.out_best_thr = out_best_thr.data_ptr();
  check_launch(tea::launch_rafp(a, ws.data_ptr(), stream_for(sorted)), "rafp");
}

// ---------------------------------------------------------------- K3m sorted-run merge
// keys: R 1-D float32 runs, each sorted descending (NaN first).  payloads: optional R 32-bit
// runs carried with their keys (e.g. the f32 target of each sample, so K3 needs no gather);
// without them the payload is each sample's position in the concatenation of the runs.
// Returns (merged keys, merged int32 payload): log2(R) pairwise merge rounds - the merge-path
// kernel on ROCm tensors, a stable host merge on CPU tensors.  The first round reads the runs
// in place (no concatenation copy) and positions are generated there (no arange).
std::vector<Tensor> merge_sorted_runs(const std::vector<Tensor>& keys, const optional<std::vector<Tensor>>& payloads) {
  TORCH_CHECK(!keys.empty(), "merge_sorted_runs: no runs");
  const bool carry = payloads.has_value();
  TORCH_CHECK(!carry || payloads->size() == keys.size(), "merge_sorted_runs: one payload per run");
  const auto dev = keys[0].device();
  const bool gpu = keys[0].is_cuda();
  int64_t n = 0;
  std::vector<int64_t> len;
  for (size_t r = 0; r < keys.size(); ++r) {
    const Tensor& k = keys[r];
    TORCH_CHECK(k.dim() == 1 && k.scalar_type() == at::kFloat && k.is_contiguous() && k.device() == dev,
                "merge_sorted_runs: keys must be contiguous float32 [n] runs on one device");
    if (carry) {
      const Tensor& v = (*payloads)[r];
      TORCH_CHECK(v.dim() == 1 && v.numel() == k.numel() && v.is_contiguous() && v.element_size() == 4 &&
                      v.device() == dev,
                  "merge_sorted_runs: payloads must be contiguous 32-bit runs matching the keys");
    }
    len.push_back(k.numel());
    n += k.numel();
  }
  TORCH_CHECK(n < (int64_t{1} << 31), "merge_sorted_runs: fewer than 2^31 samples");
  const auto fopt = keys[0].options();
  Tensor k0 = at::empty({n}, fopt), v0 = at::empty({n}, fopt.dtype(at::kInt));
  Tensor k1 = at::empty({n}, fopt), v1 = at::empty({n}, fopt.dtype(at::kInt));
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(gpu ? c10::optional<c10::Device>(dev) : c10::nullopt);
  hipStream_t st = gpu ? stream_for(keys[0]) : nullptr;
  // split scratch for the largest pair (every pair of a round is stream-ordered after the last)
  Tensor splits = gpu ? at::empty({tea::merge_splits_count(n)}, fopt.dtype(at::kLong)) : Tensor();
  auto lt = [](float x, float y) {  // descending, NaN first: x goes before y
    const bool xn = x != x, yn = y != y;
    if (xn || yn) return xn && !yn;
    return x > y;
  };
  // one stable two-run merge; va / vb null: payload = base + index
  auto merge2 = [&](const float* ka, const uint32_t* va, int64_t na, uint32_t base_a, const float* kb,
                    const uint32_t* vb, int64_t nb, uint32_t base_b, float* ko, uint32_t* vo) {
    if (gpu) {
      check_launch(tea::launch_merge_desc(ka, va, na, base_a, kb, vb, nb, base_b, ko, vo, splits.data_ptr<int64_t>(), st),
                   "merge_sorted_runs");
      return;
    }
    int64_t i = 0, j = 0, o = 0;
    while (i < na || j < nb) {
      const bool take_a = j >= nb || (i < na && !lt(kb[j], ka[i]));
      if (take_a) {
        ko[o] = ka[i];
        vo[o] = va ? va[i] : base_a + static_cast<uint32_t>(i);
        ++i;
      } else {
        ko[o] = kb[j];
        vo[o] = vb ? vb[j] : base_b + static_cast<uint32_t>(j);
        ++j;
      }
      ++o;
    }
  };
  auto pay = [&](size_t r) -> const uint32_t* {
    return carry ? static_cast<const uint32_t*>((*payloads)[r].data_ptr()) : nullptr;
  };
  // round 1: from the runs in place into (k0, v0)
  std::vector<int64_t> runs;
  {
    float* ko = k0.data_ptr<float>();
    uint32_t* vo = reinterpret_cast<uint32_t*>(v0.data_ptr<int32_t>());
    int64_t off = 0;
    for (size_t r = 0; r < keys.size(); r += 2) {
      const int64_t na = len[r], nb = r + 1 < keys.size() ? len[r + 1] : 0;
      const float* ka = keys[r].data_ptr<float>();
      const float* kb = nb ? keys[r + 1].data_ptr<float>() : ka;
      merge2(ka, pay(r), na, static_cast<uint32_t>(off), kb, nb ? pay(r + 1) : nullptr, nb,
             static_cast<uint32_t>(off + na), ko + off, vo + off);
      runs.push_back(na + nb);
      off += na + nb;
    }
  }
  while (runs.size() > 1) {
    std::vector<int64_t> next;
    int64_t off = 0;
    const float* ki = k0.data_ptr<float>();
    const uint32_t* vi = reinterpret_cast<const uint32_t*>(v0.data_ptr<int32_t>());
    float* ko = k1.data_ptr<float>();
    uint32_t* vo = reinterpret_cast<uint32_t*>(v1.data_ptr<int32_t>());
    for (size_t r = 0; r < runs.size(); r += 2) {
      const int64_t na = runs[r], nb = r + 1 < runs.size() ? runs[r + 1] : 0;
      // (an odd run out is "merged" with an empty run: one pass-through copy)
      merge2(ki + off, vi + off, na, 0, ki + off + na, vi + off + na, nb, 0, ko + off, vo + off);
      next.push_back(na + nb);
      off += na + nb;
    }
    std::swap(k0, k1);
    std::swap(v0, v1);
    runs.swap(next);
  }
  return {k0, v0};
}

// ---------------------------------------------------------------- K10b retrieval top-k
// Merges a batch into RetrievalPrecision's [Q, k] top-k state rows in place (see
// retrieval.hip).  x, t: float32 [n]; q: int64 [n] query ids or None (all query 0).
void retrieval_topk_update(const Tensor& x, const Tensor& t, const optional<Tensor>& q, const Tensor& topk,
                           const Tensor& target, const Tensor& count) {
  check_gpu(x, "scores");
  const int64_t n = x.numel();
  TORCH_CHECK(x.dim() == 1 && x.scalar_type() == at::kFloat && x.is_contiguous(), "retrieval_topk: x must be f32 [n]");
  TORCH_CHECK(t.dim() == 1 && t.numel() == n && t.scalar_type() == at::kFloat && t.is_contiguous() &&
                  t.device() == x.device(), "retrieval_topk: t must be f32 [n]");
  TORCH_CHECK(topk.dim() == 2 && topk.scalar_type() == at::kFloat && topk.is_contiguous() &&
                  target.sizes() == topk.sizes() && target.scalar_type() == at::kFloat && target.is_contiguous() &&
                  topk.device() == x.device() && target.device() == x.device(),
              "retrieval_topk: state rows must be contiguous f32 [Q, k]");
  const int64_t Q = topk.size(0), k = topk.size(1);
  TORCH_CHECK(count.dim() == 1 && count.numel() == Q && count.scalar_type() == at::kLong && count.is_contiguous() &&
                  count.device() == x.device(), "retrieval_topk: count must be int64 [Q]");
  TORCH_CHECK(k >= 1 && k <= 64 && 2 * Q * 4 <= tea::kRetrievalMaxLds && n < (int64_t{1} << 31),
              "retrieval_topk: needs 1 <= k <= 64, Q <= 8192, n < 2^31");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  tea::RetrievalArgs a;
  a.x = x.data_ptr<float>();
  a.t = t.data_ptr<float>();
  if (q.has_value()) {
    TORCH_CHECK(q->dim() == 1 && q->numel() == n && q->scalar_type() == at::kLong && q->is_contiguous() &&
                    q->device() == x.device(), "retrieval_topk: q must be int64 [n]");
    a.q = q->data_ptr<int64_t>();
  }
  a.n = n;
  a.Q = Q;
  a.k = static_cast<int>(k);
  a.topk = topk.data_ptr<float>();
  a.target_state = target.data_ptr<float>();
  a.count = count.data_ptr<int64_t>();
  hipStream_t st = stream_for(x);
  a.counts = static_cast<int*>(zeroed_workspace(x, st, Q * 4, 7));
  auto* ws = static_cast<char*>(scratch_workspace(x, st, (2 * Q + 2) * 4 + 2 * n * 4, 1));
  a.offsets = reinterpret_cast<int*>(ws);
  a.cursor = a.offsets + Q + 1;
  a.rec_key = reinterpret_cast<uint32_t*>(a.cursor + Q + 1);
  a.rec_idx = a.rec_key + n;
  check_launch(tea::launch_retrieval_topk(a, st), "retrieval_topk_update");
}

// ---------------------------------------------------------------- K5b per-row weighted sums
// x: [rows, n] view (t, w: the same shape, any strides; w may be absent -> w_scalar).
// outs[k] receives stat codes[k] / 8 with op codes[k] % 4 (see tea::RowStat / tea::RowOp), bit 2
// of the code = row 0 only (a scalar state): f32 / f64 tensors of `rows` elements (any stride:
// a ring-buffer column works), or of one element for row-0-only outputs.  CUDA tensors
// run K5b (one launch, two for rows > 64K elements); CPU tensors the host twin.
static tea::RowSumsArgs row_sums_args(const Tensor& x_in, const optional<Tensor>& t_in, const optional<Tensor>& w_in,
                                      double w_scalar, const std::vector<Tensor>& outs,
                                      const std::vector<int64_t>& codes, int64_t rows, Tensor* x_out) {
  // any shape: a [rows, n] view is used as is, anything else is viewed as rows x (numel / rows)
  auto as_rows = [&](const Tensor& v) -> Tensor {
    if (v.dim() == 2 && v.size(0) == rows) return v;
    TORCH_CHECK(rows > 0 && v.numel() % rows == 0, "row_sums: numel not divisible by rows");
    return v.reshape({rows, v.numel() / rows});
  };
  const Tensor x = as_rows(x_in);
  const optional<Tensor> t = t_in.has_value() ? optional<Tensor>(as_rows(*t_in)) : c10::nullopt;
  const optional<Tensor> w = w_in.has_value() ? optional<Tensor>(as_rows(*w_in)) : c10::nullopt;
  TORCH_CHECK(outs.size() == codes.size() && outs.size() <= static_cast<size_t>(tea::kRowSumsMaxOut),
              "row_sums: outs / codes mismatch");
  const bool gpu = x.is_cuda();
  tea::RowSumsArgs a;
  a.rows = x.size(0);
  a.n = x.size(1);
  auto bind_in = [&](const Tensor& v, const void*& p, tea::DType& dt, int64_t& rs, int64_t& cs, const char* nm) {
    TORCH_CHECK(v.dim() == 2 && v.size(0) == a.rows && v.size(1) == a.n, "row_sums: ", nm, " must match x");
    TORCH_CHECK(v.is_cuda() == gpu && (!gpu || v.device() == x.device()), "row_sums: ", nm, " on another device");
    p = v.data_ptr();
    dt = dt_of(v);
    rs = v.stride(0);
    cs = v.stride(1);
  };
  bind_in(x, a.x, a.x_dt, a.x_rs, a.x_cs, "x");
  if (t.has_value()) bind_in(*t, a.t, a.t_dt, a.t_rs, a.t_cs, "t");
  if (w.has_value()) bind_in(*w, a.w, a.w_dt, a.w_rs, a.w_cs, "w");
  a.w_scalar = w_scalar;
  a.nout = static_cast<int>(outs.size());
  int need = 0;
  for (size_t k = 0; k < outs.size(); ++k) {
    const Tensor& o = outs[k];
    TORCH_CHECK(o.scalar_type() == at::kFloat || o.scalar_type() == at::kDouble, "row_sums: outputs must be f32/f64");
    const bool first = (codes[k] & 4) != 0;
    TORCH_CHECK((o.numel() == a.rows || (first && o.numel() == 1)) && o.is_cuda() == gpu,
                "row_sums: output ", k, " must hold rows elements");
    TORCH_CHECK(o.dim() <= 1, "row_sums: outputs must be 0-d or 1-d");
    a.out[k].p = o.data_ptr();
    a.out[k].dt = o.scalar_type() == at::kFloat ? tea::DType::f32 : tea::DType::f64;
    a.out[k].stride = o.dim() == 1 ? o.stride(0) : 0;
    a.out[k].stat = static_cast<int>(codes[k] / 8);
    a.out[k].op = static_cast<int>(codes[k] % 4);
    a.out[k].first_row_only = first ? 1 : 0;
    TORCH_CHECK(a.out[k].stat >= 0 && a.out[k].stat <= tea::kRANGE, "row_sums: bad stat");
    if (a.out[k].stat < tea::kCOUNT) need |= 1 << a.out[k].stat;
    if (a.out[k].stat == tea::kRANGE) need |= (1 << tea::kTMIN) | (1 << tea::kTMAX);
  }
  a.need = need;
  *x_out = x;
  return a;
}

void row_sums(const Tensor& x_in, const optional<Tensor>& t_in, const optional<Tensor>& w_in, double w_scalar,
              const std::vector<Tensor>& outs, const std::vector<int64_t>& codes, int64_t rows) {
  Tensor x;
  tea::RowSumsArgs a = row_sums_args(x_in, t_in, w_in, w_scalar, outs, codes, rows, &x);
  const bool gpu = x.is_cuda();
  if (!gpu) {
    tea::row_sums_host(a);
    return;
  }
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  // long rows: partials + ordered combine in two launches by default (TORCHEVAL_AMD_K5B_MODE=1:
  // the fat-block fold with a release fence per block; =2: one launch with write-through
  // partials and a last-block combine - measured 14.5 vs 11.4 us for Sum 8192 x 1000,
  // profiles/odd_width_cliff_r5_k5.json: the hand-off sits on the launch's tail)
  static const int mode = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K5B_MODE");
    return (e != nullptr && e[0] != '\0') ? std::atoi(e) : 0;
  }();
  a.blocks = mode == 0 ? tea::row_sums_blocks(a.rows, a.n)
                       : mode == 1 ? tea::row_sums_fold_blocks(a.rows, a.n) : tea::row_sums_wt_blocks(a.rows, a.n);
  if (a.blocks > 1) {  // stream-ordered scratch, fully rewritten by every call: cached, no allocation
    a.ws = static_cast<double*>(zeroed_workspace(x, stream_for(x), a.rows * a.blocks * tea::kRowRaw * 8, 3));
    if (mode != 0) {  // self-cleaning arrival tickets
      a.ticket = static_cast<unsigned*>(zeroed_workspace(x, stream_for(x), a.rows * 4, 9));
      a.wt = mode == 2;
    }
  }
  if (a.n == 0 && a.rows > 0) a.blocks = 1;
  check_launch(tea::launch_row_sums(a, stream_for(x)), "row_sums");
}

// deferred-mode K5b update (rows longer than one block; ADD outputs of sums / W / COUNT): the
// grid blocks add their pre-scaled FP64 partials to their slots of `pend` (float64, zeroed,
// rows * kRowPendStats * kRowPendBlocks); returns the blocks used (0: not applicable, the
// caller runs row_sums).  row_sums_fold applies the slots to the same outputs and zeroes them.
int64_t row_sums_pend(const Tensor& x_in, const optional<Tensor>& t_in, const optional<Tensor>& w_in,
                      double w_scalar, const std::vector<Tensor>& outs, const std::vector<int64_t>& codes,
                      int64_t rows, const Tensor& pend) {
  Tensor x;
  tea::RowSumsArgs a = row_sums_args(x_in, t_in, w_in, w_scalar, outs, codes, rows, &x);
  if (!x.is_cuda() || a.n == 0) return 0;
  for (int k = 0; k < a.nout; ++k) {  // sums / COUNT added, extrema min / max, RANGE set
    const auto& o = a.out[k];
    const bool ok = o.stat == tea::kTMIN ? o.op == tea::kMin : o.stat == tea::kTMAX ? o.op == tea::kMax
                  : o.stat == tea::kRANGE ? o.op == tea::kSet : o.op == tea::kAdd;
    if (!ok) return 0;
  }
  const int blocks = tea::row_sums_blocks(a.rows, a.n);
  if (blocks < 2 || blocks > tea::kRowPendBlocks) return 0;
  TORCH_CHECK(pend.scalar_type() == at::kDouble && pend.is_contiguous() && pend.device() == x.device() &&
                  pend.numel() >= a.rows * tea::kRowPendStats * tea::kRowPendBlocks,
              "row_sums_pend: pend must be float64 [rows * ", tea::kRowPendStats, " * ", tea::kRowPendBlocks, "]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  a.blocks = blocks;
  a.pend = pend.data_ptr<double>();
  a.pend_blocks = tea::kRowPendBlocks;
  check_launch(tea::launch_row_sums(a, stream_for(x)), "row_sums_pend");
  return blocks;
}

void row_sums_fold(const Tensor& pend, int64_t used, const std::vector<Tensor>& outs,
                   const std::vector<int64_t>& codes, int64_t rows) {
  TORCH_CHECK(!outs.empty(), "row_sums_fold: no outputs");
  const Tensor carrier = at::empty({rows, 0}, pend.options().dtype(at::kFloat));
  Tensor x;
  tea::RowSumsArgs a = row_sums_args(carrier, c10::nullopt, c10::nullopt, 1.0, outs, codes, rows, &x);
  TORCH_CHECK(pend.scalar_type() == at::kDouble && pend.is_cuda() &&
                  pend.numel() >= a.rows * tea::kRowPendStats * tea::kRowPendBlocks,
              "row_sums_fold: bad pend buffer");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(pend.device());
  a.pend = pend.data_ptr<double>();
  a.pend_blocks = tea::kRowPendBlocks;
  check_launch(tea::launch_row_sums_fold(a, static_cast<int>(used), stream_for(pend)), "row_sums_fold");
}

// ---------------------------------------------------------------- K4b per-sample binned AUROC
// input float32 [n, c] (unit column stride), target int64 / int32 [n], thr float32 [T] ascending
// (contiguous), out float32 [n], err int32 [>= 1] (bit 0: a label outside [0, c))
void sample_binned_auroc(const Tensor& input, const Tensor& target, const Tensor& thr, const Tensor& out,
                         const Tensor& err) {
  check_gpu(input, "input");
  TORCH_CHECK(input.dim() == 2 && input.scalar_type() == at::kFloat && input.stride(1) == 1,
              "sample_binned_auroc: input must be float32 [n, c] with unit column stride");
  TORCH_CHECK(target.dim() == 1 && target.size(0) == input.size(0) && target.device() == input.device() &&
                  (target.scalar_type() == at::kLong || target.scalar_type() == at::kInt),
              "sample_binned_auroc: target must be int64 / int32 [n] on the input's device");
  TORCH_CHECK(thr.dim() == 1 && thr.scalar_type() == at::kFloat && thr.is_contiguous() && thr.device() == input.device(),
              "sample_binned_auroc: thresholds must be a contiguous float32 vector on the input's device");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == input.size(0) &&
                  out.device() == input.device(),
              "sample_binned_auroc: out must be float32 [n]");
  TORCH_CHECK(err.scalar_type() == at::kInt && err.numel() >= 1 && err.device() == input.device(),
              "sample_binned_auroc: err must be int32");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  tea::SampleAurocArgs a;
  a.input = input.data_ptr<float>();
  a.n = input.size(0);
  a.c = input.size(1);
  a.row_stride = input.stride(0);
  a.target = target.data_ptr();
  a.tg_dt = dt_of(target);
  a.tg_stride = target.stride(0);
  a.thr = thr.data_ptr<float>();
  a.T = static_cast<int>(thr.numel());
  a.out = out.data_ptr<float>();
  a.err = err.data_ptr<int>();
  const int rc = tea::launch_sample_binned_auroc(a, stream_for(input));
  TORCH_CHECK(rc != -1, "sample_binned_auroc: unsupported arguments (needs c >= 1, T >= 1)");
  check_launch(rc, "sample_binned_auroc");
}

// ---------------------------------------------------------------- K4 binned histograms
// input: [n, c] view (any strides); target: [n, c] view (mode 0) or [n] labels (mode 1);
// thr: float32 [T] sorted; tp/fp/fn: float32 [T, c] views sharing strides (accumulated).
void binned_counts(const Tensor& input, const Tensor& target, const Tensor& thr, int64_t mode,
                   const optional<Tensor>& tp, const optional<Tensor>& fp,
                   const optional<Tensor>& fn, int64_t uniform) {
  check_gpu(input, "input");
  TORCH_CHECK(input.dim() == 2, "binned_counts: input must be a 2-D view [n, c]");
  TORCH_CHECK(thr.dim() == 1 && thr.scalar_type() == at::kFloat && thr.is_contiguous(),
              "binned_counts: thresholds must be a contiguous float32 vector");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  tea::BinnedArgs a;
  a.input = input.data_ptr();
  a.in_dt = dt_of(input);
  a.n = input.size(0);
  a.c = input.size(1);
  a.in_row_stride = input.stride(0);
  a.in_col_stride = input.stride(1);
  a.mode = static_cast<int>(mode);
  if (mode == 1) {
    TORCH_CHECK(target.dim() == 1 && target.size(0) == a.n, "binned_counts: labels must be [n]");
    a.tg_row_stride = target.stride(0);
  } else {
    TORCH_CHECK(target.dim() == 2 && target.size(0) == a.n && target.size(1) == a.c,
                "binned_counts: target must match input");
    a.tg_row_stride = target.stride(0);
    a.tg_col_stride = target.stride(1);
  }
  a.target = target.data_ptr();
  a.tg_dt = dt_of(target);
  a.thr = thr.data_ptr<float>();
  a.T = static_cast<int>(thr.numel());
  a.uniform = uniform != 0 && a.T >= 2;
  int64_t ks = -1, cs = -1;
  auto out = [&](const optional<Tensor>& t, const char* name) -> float* {
    if (!t.has_value()) return nullptr;
    TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(0) == a.T &&
                    t->size(1) == a.c && t->device() == input.device(),
                "binned_counts: ", name, " must be float32 [T, c] on the input device");
    TORCH_CHECK(ks < 0 || (ks == t->stride(0) && cs == t->stride(1)),
                "binned_counts: outputs must share strides");
    ks = t->stride(0);
    cs = t->stride(1);
    return t->data_ptr<float>();
  };
  a.tp = out(tp, "tp");
  a.fp = out(fp, "fp");
  a.fn = out(fn, "fn");
  a.out_k_stride = ks;
  a.out_c_stride = cs;
  a.ws = reinterpret_cast<unsigned*>(
      zeroed_workspace(input, stream_for(input), tea::binned_workspace_words(a.T, a.c) * 4, 1));
  if (const int64_t sw = tea::binned_slab_words(a.T, a.c))
    a.slab = reinterpret_cast<unsigned*>(zeroed_workspace(input, stream_for(input), sw * 4, 2));
  const int rc = tea::launch_binned(a, stream_for(input));
  TORCH_CHECK(rc != -1, "binned_counts: too many thresholds (", a.T, ") for the LDS histogram");
  check_launch(rc, "binned_counts");
}

// ---------------------------------------------------------------- K5 / K6 reductions
// x, t: [n, d] views (t optional); w: optional [n]; outputs float32 (accumulated):
// sse/st/stt/sx as [d] views sharing one stride, sw scalar.
// x, t: [n, d] views; w: [n]; outputs float32 [d] sharing a stride, sw scalar (shared by
// column_moments / column_moments_pend / column_moments_fold)
static tea::MomentsArgs moments_args(const optional<Tensor>& x, const optional<Tensor>& t,
                                     const optional<Tensor>& w, const optional<Tensor>& sse,
                                     const optional<Tensor>& st, const optional<Tensor>& stt,
                                     const optional<Tensor>& sx, const optional<Tensor>& sw, const Tensor& ref) {
  tea::MomentsArgs a;
  a.n = ref.size(0);
  a.d = ref.size(1);
  if (x.has_value()) {
    TORCH_CHECK(x->sizes() == ref.sizes(), "column_moments: x shape");
    a.x = x->data_ptr();
    a.x_dt = dt_of(*x);
    a.x_row_stride = x->stride(0);
    a.x_col_stride = x->stride(1);
  }
  if (t.has_value()) {
    TORCH_CHECK(t->sizes() == ref.sizes(), "column_moments: t shape must match x");
    a.t = t->data_ptr();
    a.t_dt = dt_of(*t);
    a.t_row_stride = t->stride(0);
    a.t_col_stride = t->stride(1);
  }
  if (w.has_value()) {
    TORCH_CHECK(w->dim() == 1 && w->size(0) == a.n, "column_moments: w must be [n]");
    a.w = w->data_ptr();
    a.w_dt = dt_of(*w);
    a.w_stride = w->stride(0);
  }
  int64_t os = -1;
  auto out = [&](const optional<Tensor>& o, const char* name) -> float* {
    if (!o.has_value()) return nullptr;
    TORCH_CHECK(o->scalar_type() == at::kFloat && o->numel() == a.d && o->device() == ref.device(),
                "column_moments: ", name, " must be float32 with d elements");
    const int64_t s = o->dim() == 0 ? 1 : o->stride(-1);
    TORCH_CHECK(os < 0 || os == s, "column_moments: outputs must share a stride");
    os = s;
    return o->data_ptr<float>();
  };
  a.sse = out(sse, "sse");
  a.st = out(st, "st");
  a.stt = out(stt, "stt");
  a.sx = out(sx, "sx");
  a.out_stride = os < 0 ? 1 : os;
  if (sw.has_value()) {
    TORCH_CHECK(sw->scalar_type() == at::kFloat && sw->numel() == 1, "column_moments: sw scalar f32");
    a.sw = sw->data_ptr<float>();
  }
  return a;
}

// deferred-mode pend buffer size for d columns and statistic set `need` (the one place the
// slot layout is computed; Python sizes its buffers from here)
int64_t column_moments_pend_numel(int64_t d, int64_t need) {
  const int ns = tea::moments_ns_of(static_cast<int>(need));
  TORCH_CHECK(ns > 0, "column_moments_pend: the slot layout covers the statistic sets {sse}, {sse, st, stt} and "
              "{sse, st, stt, sx} only (need = ", need, ")");
  return tea::kMomentsPendSlots * (ns * d + 1);
}

static void bind_pend(tea::MomentsArgs& a, const Tensor& pend, const Tensor& ref) {
  TORCH_CHECK(tea::moments_ns(a) > 0, "column_moments: deferred mode needs the statistic set {sse}, {sse, st, stt} "
              "or {sse, st, stt, sx} (need = ", tea::moments_need(a), ")");
  TORCH_CHECK(pend.scalar_type() == at::kDouble && pend.is_contiguous() && pend.device() == ref.device() &&
                  pend.numel() >= tea::kMomentsPendSlots * (tea::moments_ns(a) * a.d + 1),
              "column_moments: pend must be a contiguous float64 buffer of slots * (ns * d + 1)");
  a.pend = pend.data_ptr<double>();
  a.pend_slots = tea::kMomentsPendSlots;
}

// deferred-mode class update: FP64 column partials ADDED to the slots of `pend` (zero-initialised
// by the caller, zeroed again by column_moments_fold); the states are only the statistic
// selection here.  Returns the slots used (0: not applicable, the caller takes another path).
int64_t column_moments_pend(const optional<Tensor>& x, const optional<Tensor>& t, const optional<Tensor>& w,
                            const optional<Tensor>& sse, const optional<Tensor>& st, const optional<Tensor>& stt,
                            const optional<Tensor>& sx, const optional<Tensor>& sw, const Tensor& pend) {
  const Tensor& ref = x.has_value() ? *x : *t;
  check_gpu(ref, "x/t");
  TORCH_CHECK(ref.dim() == 2, "column_moments: inputs must be [n, d] views");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ref.device());
  tea::MomentsArgs a = moments_args(x, t, w, sse, st, stt, sx, sw, ref);
  if (a.n == 0 || a.d == 0) return 0;
  bind_pend(a, pend, ref);
  int64_t wsd = 0, tk = 0;
  if (!tea::column_moments_v2_plan(a, &wsd, &tk)) return 0;
  check_launch(tea::launch_column_moments(a, stream_for(ref)), "column_moments_pend");
  return a.v2_r;
}

// fold the first `slots` pending slots into the states (float32 +=) and zero them
void column_moments_fold(const Tensor& pend, int64_t slots, const optional<Tensor>& sse,
                         const optional<Tensor>& st, const optional<Tensor>& stt, const optional<Tensor>& sx,
                         const optional<Tensor>& sw) {
  const Tensor& like = sse.has_value() ? *sse : st.has_value() ? *st : *stt;
  check_gpu(like, "states");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(like.device());
  const Tensor ref = at::empty({0, like.numel()}, like.options());  // shape carrier: n = 0, d
  tea::MomentsArgs a = moments_args(c10::nullopt, c10::nullopt, c10::nullopt, sse, st, stt, sx, sw, ref);
  bind_pend(a, pend, like);
  check_launch(tea::launch_moments_fold(a, static_cast<int>(slots), stream_for(like)), "column_moments_fold");
}

void column_moments(const optional<Tensor>& x, const optional<Tensor>& t,
                    const optional<Tensor>& w, const optional<Tensor>& sse,
                    const optional<Tensor>& st, const optional<Tensor>& stt,
                    const optional<Tensor>& sx, const optional<Tensor>& sw, int64_t overwrite,
                    int64_t mse_mode, const optional<Tensor>& mse_out, int64_t num_regressors) {
  const Tensor& ref = x.has_value() ? *x : *t;
  check_gpu(ref, "x/t");
  TORCH_CHECK(ref.dim() == 2, "column_moments: inputs must be [n, d] views");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ref.device());
  tea::MomentsArgs a = moments_args(x, t, w, sse, st, stt, sx, sw, ref);
  a.overwrite = overwrite != 0;
  a.mse_mode = static_cast<int>(mse_mode);
  Tensor raw_scratch;
  if (a.mse_mode) {
    const bool raw = a.mse_mode == 1 || a.mse_mode == 3;
    TORCH_CHECK(a.mse_mode >= 1 && a.mse_mode <= 5 && a.overwrite && a.sse && mse_out.has_value() &&
                    mse_out->scalar_type() == at::kFloat && mse_out->is_contiguous() &&
                    mse_out->device() == ref.device() && mse_out->numel() == (raw ? a.d : 1),
                "column_moments: fused compute needs overwrite, sse and a float32 output of d (raw) or 1 elements");
    TORCH_CHECK(a.mse_mode < 3 || (a.st && a.stt), "column_moments: fused R2 needs st and stt");
    a.mse_out = mse_out->data_ptr<float>();
    a.num_obs = a.n;
    a.num_regressors = static_cast<int>(num_regressors);
    if (!raw) {
      raw_scratch = at::empty({2 * a.d}, ref.options().dtype(at::kFloat));
      a.mse_part_f = raw_scratch.data_ptr<float>();
    }
  }
  if (a.n == 0 || a.d == 0) return;
  int64_t v2_doubles = 0, v2_tickets = 0;
  if (tea::column_moments_v2_plan(a, &v2_doubles, &v2_tickets)) {  // one launch (K5 v2)
    hipStream_t st = stream_for(ref);
    a.part = static_cast<double*>(scratch_workspace(ref, st, v2_doubles * 8, 8));
    a.tickets = static_cast<unsigned*>(zeroed_workspace(ref, st, v2_tickets * 4, 8));
    check_launch(tea::launch_column_moments(a, st), "column_moments");
    return;
  }
  a.ws_blocks = tea::column_moments_blocks(a.n, a.d);
  const int64_t nstats = (a.sse != nullptr) + (a.st != nullptr) + (a.stt != nullptr) + (a.sx != nullptr);
  Tensor ws = at::empty({a.ws_blocks * (nstats * a.d + 1)}, ref.options().dtype(at::kDouble));
  a.ws = ws.data_ptr<double>();
  check_launch(tea::launch_column_moments(a, stream_for(ref)), "column_moments");
}

// x, t: [rows, n] (rows contiguous); w optional [rows, n]; out float64 [rows, 3] accumulated.
void ne_sums(const Tensor& x, const Tensor& t, const optional<Tensor>& w, bool from_logits,
             const Tensor& out, const optional<Tensor>& err, bool deterministic) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && t.sizes() == x.sizes(), "ne_sums: x/t must be [rows, n]");
  TORCH_CHECK(x.stride(1) == 1 && t.stride(1) == 1, "ne_sums: rows must be contiguous");
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.is_contiguous() && out.numel() == x.size(0) * 3,
              "ne_sums: out must be float64 [rows, 3]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  tea::NeArgs a;
  a.x = x.data_ptr();
  a.x_dt = dt_of(x);
  a.x_row_stride = x.stride(0);
  a.t = t.data_ptr();
  a.t_dt = dt_of(t);
  a.t_row_stride = t.stride(0);
  if (w.has_value()) {
    TORCH_CHECK(w->sizes() == x.sizes() && w->stride(1) == 1, "ne_sums: weight must match x");
    a.w = w->data_ptr();
    a.w_dt = dt_of(*w);
    a.w_row_stride = w->stride(0);
  }
  a.rows = x.size(0);
  a.n = x.size(1);
  a.from_logits = from_logits ? 1 : 0;
  a.out = out.data_ptr<double>();
  if (err.has_value()) {
    TORCH_CHECK(err->scalar_type() == at::kInt, "ne_sums: err must be int32");
    a.err = err->data_ptr<int>();
    // [flag, pad, range keys as 2 x u64] (8-byte aligned: caching-allocator blocks are)
    if (err->numel() >= 6) a.range = reinterpret_cast<unsigned long long*>(a.err + 2);
  }
  Tensor ws;
  if (deterministic && a.rows > 0) {
    ws = at::empty({a.rows * 3 * tea::ne_sums_blocks(a.n)}, out.options());
    a.ordered_ws = ws.data_ptr<double>();
  }
  check_launch(tea::launch_ne_sums(a, stream_for(x)), "ne_sums");
}

// ---------------------------------------------------------------- K7 perplexity
// input: [rows, v] logits (unit column stride); target: [rows]; out float64 [2] accumulated.
void perplexity_sums(const Tensor& input, const Tensor& target, optional<int64_t> ignore_index,
                     const Tensor& out, const optional<Tensor>& err, bool deterministic) {
  check_gpu(input, "input");
  TORCH_CHECK(input.dim() == 2 && input.stride(1) == 1, "perplexity: input must be [rows, v]");
  TORCH_CHECK(target.dim() == 1 && target.size(0) == input.size(0), "perplexity: target must be [rows]");
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.numel() == 2 && out.is_contiguous(),
              "perplexity: out must be float64 [2]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  tea::PerplexityArgs a;
  a.input = input.data_ptr();
  a.in_dt = dt_of(input);
  a.rows = input.size(0);
  a.v = input.size(1);
  a.row_stride = input.stride(0);
  a.target = target.data_ptr();
  a.tg_dt = dt_of(target);
  a.tg_stride = target.stride(0);
  if (ignore_index.has_value()) {
    a.has_ignore = 1;
    a.ignore_index = *ignore_index;
  }
  a.out = out.data_ptr<double>();
  if (err.has_value()) a.err = err->data_ptr<int>();
  Tensor ws;
  if (deterministic && a.rows > 0) {
    ws = at::empty({2 * tea::perplexity_blocks(a)}, out.options());
    a.ordered_ws = ws.data_ptr<double>();
  }
  const int rc = tea::launch_perplexity(a, stream_for(input));
  TORCH_CHECK(rc != -1, "perplexity: unsupported logits dtype ", input.scalar_type());
  TORCH_CHECK(rc != -2, "perplexity: logits storage is not element-aligned");
  check_launch(rc, "perplexity");
}

// ---------------------------------------------------------------- K8 FID covariance
void fid_cov_update(const Tensor& act_in, const Tensor& cov, const optional<Tensor>& colsum) {
  check_gpu(act_in, "activations");
  TORCH_CHECK(act_in.dim() == 2 && act_in.scalar_type() == at::kFloat && act_in.stride(1) == 1,
              "fid_cov_update: activations must be float32 [n, d] with unit column stride");
  const int64_t d = act_in.size(1);
  // K8 stages 16-byte pieces: rows must start 16-byte aligned and a width that is not a
  // multiple of 4 is zero-padded (one copy; the FID feature widths 64 / 192 / 768 / 2048 never
  // need it)
  Tensor act = act_in;
  if (d % 4 != 0) act = at::constant_pad_nd(act_in, {0, 4 - d % 4}, 0);
  TORCH_CHECK(act.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(act.data_ptr()) % 16 == 0,
              "fid_cov_update: activation rows must be 16-byte aligned");
  TORCH_CHECK(cov.scalar_type() == at::kFloat && cov.is_contiguous() && cov.numel() == d * d &&
                  cov.device() == act.device(),
              "fid_cov_update: cov must be a contiguous float32 [d, d] on the same device");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(act.device());
  tea::FidCovArgs a;
  a.act = act.data_ptr<float>();
  a.n = act.size(0);
  a.d = d;
  a.ld = act.size(1);
  a.row_stride = act.stride(0);
  a.cov = cov.data_ptr<float>();
  a.zeros = static_cast<const float*>(zeroed_workspace(act, stream_for(act), 64, 6));
  if (colsum.has_value()) {
    TORCH_CHECK(colsum->scalar_type() == at::kFloat && colsum->is_contiguous() && colsum->numel() == d,
                "fid_cov_update: colsum must be float32 [d]");
    a.colsum = colsum->data_ptr<float>();
  }
  a.split = tea::fid_cov_split(a.n, d);
  if (a.split > 1)
    a.ws = static_cast<float*>(scratch_workspace(act, stream_for(act), tea::fid_cov_workspace_bytes(d, a.split), 0));
  check_launch(tea::launch_fid_cov(a, stream_for(act)), "fid_cov_update");
}


// ---------------------------------------------------------------- K9b symmetric eigenvalues
// Eigenvalues (ascending) of a symmetric FP64 [n, n] matrix by the on-chip (register-resident) one-launch
// Householder reduction + multisection (csrc/kernels/symeig.hip).  Returns 0 when launched
// (then status[0] != 0 after the stream reaches it means the grid aborted and lam is
// invalid), non-zero when this device / size is not handled (nothing launched).
int64_t sym_eigvals(const Tensor& m, const Tensor& lam, const Tensor& status) {
  check_gpu(m, "matrix");
  TORCH_CHECK(m.dim() == 2 && m.size(0) == m.size(1) && m.scalar_type() == at::kDouble && m.is_contiguous(),
              "sym_eigvals: matrix must be a contiguous float64 [n, n]");
  const int64_t n = m.size(0);
  TORCH_CHECK(lam.scalar_type() == at::kDouble && lam.is_contiguous() && lam.numel() == n &&
                  lam.device() == m.device(),
              "sym_eigvals: lam must be a contiguous float64 [n] on the matrix's device");
  TORCH_CHECK(status.scalar_type() == at::kInt && status.numel() >= 1 && status.device() == m.device(),
              "sym_eigvals: status must be an int32 tensor on the matrix's device");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(m.device());
  int grid = 0, rows = 0;
  if (tea::symeig_plan(n, &grid, &rows) != 0) return 1;
  const hipStream_t stream = stream_for(m);
  tea::SymEigArgs a;
  a.a = m.data_ptr<double>();
  a.n = n;
  a.ld = tea::symeig_slot_stride(n);
  // layout: ctl (2 KB), d [ld], e [ld], the 2 hand-off slot planes (sentinel-filled by the
  // launcher on every call, so no state carries over between launches), the Sturm-count grid,
  // the tail kernel's trailing block
  const int64_t bytes = 2048 + 2 * a.ld * (int64_t)sizeof(double) + tea::symeig_slot_bytes(n) + tea::symeig_grid_bytes() +
                        tea::symeig_tail_bytes();
  char* ws = static_cast<char*>(scratch_workspace(m, stream, bytes, 3));
  a.ctl = reinterpret_cast<unsigned*>(ws);
  a.d = reinterpret_cast<double*>(ws + 2048);
  a.e = a.d + a.ld;
  a.slots = reinterpret_cast<unsigned long long*>(a.e + a.ld);
  a.grid = reinterpret_cast<int*>(reinterpret_cast<char*>(a.slots) + tea::symeig_slot_bytes(n));
  a.tail = reinterpret_cast<double*>(reinterpret_cast<char*>(a.grid) + tea::symeig_grid_bytes());
  a.lam = lam.data_ptr<double>();
  const int rc = tea::launch_symeig(a, stream);
  if (rc == 1 || rc == 3) return rc;
  check_launch(rc, "sym_eigvals");
  TORCH_CHECK(hipMemcpyAsync(status.data_ptr<int>(), a.ctl + 1, sizeof(int), hipMemcpyDeviceToDevice, stream) ==
                  hipSuccess,
              "sym_eigvals: status copy failed");
  return 0;
}

// K9c: one diagonal block of the blocked FP64 Cholesky (factor in place + inverse).
void potrf_block(const Tensor& a, int64_t k0, int64_t b, const Tensor& linv, const Tensor& info) {
  check_gpu(a, "matrix");
  TORCH_CHECK(a.dim() == 2 && a.size(0) == a.size(1) && a.scalar_type() == at::kDouble && a.is_contiguous(),
              "potrf_block: matrix must be a contiguous float64 [n, n]");
  TORCH_CHECK(k0 >= 0 && b >= 1 && b <= tea::potrf_block_size() && k0 + b <= a.size(0),
              "potrf_block: block out of range");
  TORCH_CHECK(linv.scalar_type() == at::kDouble && linv.is_contiguous() && linv.numel() == b * b &&
                  linv.device() == a.device(),
              "potrf_block: linv must be a contiguous float64 [b, b]");
  TORCH_CHECK(info.scalar_type() == at::kInt && info.numel() >= 1 && info.device() == a.device(),
              "potrf_block: info must be int32 on the matrix's device");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  check_launch(tea::launch_potrf_block(a.data_ptr<double>(), a.size(1), (int)k0, (int)b, linv.data_ptr<double>(),
                                       info.data_ptr<int>(), stream_for(a)),
               "potrf_block");
}

// K9d: the whole blocked FP64 Cholesky in one persistent launch (csrc/kernels/cholesky.hip).
// l: padded [64 nt, 64 nt] float64 output (upper triangle zeroed), linv: >= nt * 4096 float64
// scratch, ctl: >= 1 int32 scratch, status: >= 2 int32 -> [LAPACK info, abort].
void cholesky_factor(const Tensor& a, const Tensor& l, const Tensor& linv, const Tensor& ctl, const Tensor& status) {
  check_gpu(a, "matrix");
  TORCH_CHECK(a.dim() == 2 && a.size(0) == a.size(1) && a.scalar_type() == at::kDouble && a.stride(1) == 1,
              "cholesky_factor: matrix must be a row-contiguous float64 [n, n]");
  const int64_t n = a.size(0);
  const int64_t N = 64 * static_cast<int64_t>(tea::cholesky_tiles(n));
  TORCH_CHECK(l.scalar_type() == at::kDouble && l.is_contiguous() && l.numel() == N * N && l.device() == a.device(),
              "cholesky_factor: l must be a contiguous float64 [", N, ", ", N, "]");
  TORCH_CHECK(linv.scalar_type() == at::kDouble && linv.is_contiguous() && linv.numel() >= (N / 64) * 4096 &&
                  linv.device() == a.device(),
              "cholesky_factor: linv too small");
  TORCH_CHECK(ctl.scalar_type() == at::kInt && ctl.numel() >= 1 && ctl.device() == a.device(), "cholesky_factor: ctl");
  TORCH_CHECK(status.scalar_type() == at::kInt && status.is_contiguous() && status.numel() >= 2 &&
                  status.device() == a.device(),
              "cholesky_factor: status must be int32 [2]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  check_launch(tea::launch_cholesky(a.data_ptr<double>(), a.stride(0), n, l.data_ptr<double>(), linv.data_ptr<double>(),
                                    ctl.data_ptr<int>(), status.data_ptr<int>(), stream_for(a)),
               "cholesky_factor");
}

// K9p: pivoted (rank-revealing) FP64 Cholesky of a symmetric PSD matrix in one cooperative
// launch (csrc/kernels/pivchol.hip).  slots: int64 [pivchol_slot_words(n)] scratch, w: contiguous
// float64 [N, N], N = pivchol_padded(n) (row j = factor column j in the original feature order),
// piv: int32 [n], info: int32 [2] -> [rank, status (1 NaN in the matrix, 2 aborted)], ctl: int32
// [>= 1] scratch.  Returns 0 launched, 3 the grid could not be co-scheduled, 4 n unsupported.
int64_t pivchol_impl(const Tensor& a, const Tensor& slots, const Tensor& w, const Tensor& piv, const Tensor& info,
                     const Tensor& ctl, unsigned long long* trace) {
  check_gpu(a, "matrix");
  TORCH_CHECK(a.dim() == 2 && a.size(0) == a.size(1) && a.scalar_type() == at::kDouble && a.stride(1) == 1,
              "pivchol: matrix must be a row-contiguous float64 [n, n]");
  const int64_t n = a.size(0);
  const int64_t N = tea::pivchol_padded(n);
  TORCH_CHECK(slots.scalar_type() == at::kLong && slots.is_contiguous() && slots.numel() >= tea::pivchol_slot_words(n) &&
                  slots.device() == a.device(),
              "pivchol: slots must be int64 [pivchol_slot_words(n)]");
  TORCH_CHECK(w.scalar_type() == at::kDouble && w.is_contiguous() && w.numel() == N * N && w.device() == a.device(),
              "pivchol: w must be a contiguous float64 [", N, ", ", N, "]");
  TORCH_CHECK(piv.scalar_type() == at::kInt && piv.is_contiguous() && piv.numel() >= n && piv.device() == a.device(),
              "pivchol: piv must be int32 [n]");
  TORCH_CHECK(info.scalar_type() == at::kInt && info.is_contiguous() && info.numel() >= 2 && info.device() == a.device(),
              "pivchol: info must be int32 [2]");
  TORCH_CHECK(ctl.scalar_type() == at::kInt && ctl.is_contiguous() && ctl.numel() >= 1 && ctl.device() == a.device(),
              "pivchol: ctl must be int32 [1]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  const int rc = tea::launch_pivchol(a.data_ptr<double>(), a.stride(0), n,
                                     reinterpret_cast<unsigned long long*>(slots.data_ptr<int64_t>()), w.data_ptr<double>(),
                                     piv.data_ptr<int>(), info.data_ptr<int>(),
                                     reinterpret_cast<unsigned*>(ctl.data_ptr<int>()), stream_for(a), trace);
  TORCH_CHECK(rc != 2, "pivchol: launch setup failed");
  return rc;
}
int64_t pivchol(const Tensor& a, const Tensor& slots, const Tensor& w, const Tensor& piv, const Tensor& info,
                const Tensor& ctl) {
  return pivchol_impl(a, slots, w, piv, info, ctl, nullptr);
}
// profiling hook: pivchol with the launcher's phase stamps in trace (int64 >= 80)
int64_t pivchol_traced(const Tensor& a, const Tensor& slots, const Tensor& w, const Tensor& piv, const Tensor& info,
                       const Tensor& ctl, const Tensor& trace) {
  TORCH_CHECK(trace.scalar_type() == at::kLong && trace.is_contiguous() && trace.numel() >= 80 &&
                  trace.device() == a.device(),
              "pivchol_traced: trace must be int64 [80]");
  return pivchol_impl(a, slots, w, piv, info, ctl, reinterpret_cast<unsigned long long*>(trace.data_ptr<int64_t>()));
}

// test / profiling hook: cholesky_factor with per-tile-column phase stamps (s_memrealtime,
// 100 MHz) of the pair-owner tasks in trace (int64 [nt * 8]), then the shader-clock stamps of every
// column of tile column 1's factorisation (wave 0: [nt * 8, + 65), wave 1: [nt * 8 + 65, + 65))
void cholesky_factor_traced(const Tensor& a, const Tensor& l, const Tensor& linv, const Tensor& ctl,
                            const Tensor& status, const Tensor& trace) {
  const int64_t nt = tea::cholesky_tiles(a.size(0));
  TORCH_CHECK(trace.scalar_type() == at::kLong && trace.is_contiguous() && trace.numel() >= nt * 8 + 130 &&
                  trace.device() == a.device(),
              "cholesky_factor_traced: trace must be int64 [nt * 8 + 130]");
  check_gpu(a, "matrix");
  TORCH_CHECK(l.numel() == 64 * nt * 64 * nt && linv.numel() >= nt * 4096 && status.numel() >= 2,
              "cholesky_factor_traced: workspace sizes");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(a.device());
  check_launch(tea::launch_cholesky(a.data_ptr<double>(), a.stride(0), a.size(0), l.data_ptr<double>(),
                                    linv.data_ptr<double>(), ctl.data_ptr<int>(), status.data_ptr<int>(), stream_for(a),
                                    reinterpret_cast<unsigned long long*>(trace.data_ptr<int64_t>())),
               "cholesky_factor_traced");
}

// K3t: trapezoid area per row of x-sorted (x, y) pairs (csrc/kernels/trapz.hip); y is the f32
// payload K3a carried through its sort (the int32 order buffer, reinterpreted)
void trapz_sorted(const Tensor& x, const Tensor& y_bits, const Tensor& out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kFloat && x.is_contiguous(), "trapz_sorted: x must be contiguous f32 [rows, n]");
  TORCH_CHECK((y_bits.scalar_type() == at::kInt || y_bits.scalar_type() == at::kFloat) && y_bits.is_contiguous() &&
                  y_bits.sizes() == x.sizes() && y_bits.device() == x.device(),
              "trapz_sorted: y must be contiguous f32 / int32 bits shaped like x");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == x.size(0) &&
                  out.device() == x.device(),
              "trapz_sorted: out must be f32 [rows]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const hipStream_t st = stream_for(x);
  auto* part = static_cast<double*>(scratch_workspace(x, st, x.size(0) * tea::trapz_blocks(x.size(1)) * 8, 13));
  check_launch(tea::launch_trapz_sorted(x.data_ptr<float>(), static_cast<const float*>(y_bits.data_ptr()), x.size(0),
                                        x.size(1), part, out.data_ptr<float>(), st),
               "trapz_sorted");
}

// FID compute glue (csrc/kernels/fid_prep.hip): FP64 symmetric covariance from the FP32 states.
void cov_finalize(const Tensor& cov_sum, const Tensor& colsum, double n, const Tensor& out) {
  check_gpu(cov_sum, "cov_sum");
  const int64_t d = colsum.numel();
  TORCH_CHECK(cov_sum.scalar_type() == at::kFloat && cov_sum.is_contiguous() && cov_sum.numel() == d * d,
              "cov_finalize: cov_sum must be a contiguous float32 [d, d]");
  TORCH_CHECK(colsum.scalar_type() == at::kFloat && colsum.is_contiguous() && colsum.device() == cov_sum.device(),
              "cov_finalize: colsum must be a contiguous float32 [d]");
  TORCH_CHECK(out.scalar_type() == at::kDouble && out.is_contiguous() && out.numel() == d * d &&
                  out.device() == cov_sum.device(),
              "cov_finalize: out must be a contiguous float64 [d, d]");
  TORCH_CHECK(n > 1.0, "cov_finalize: needs n > 1");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(cov_sum.device());
  check_launch(tea::launch_cov_finalize(cov_sum.data_ptr<float>(), colsum.data_ptr<float>(), n, d,
                                        out.data_ptr<double>(), stream_for(cov_sum)),
               "cov_finalize");
}

// FID's closing combination: |sum1 / n1 - sum2 / n2|^2 + tr S1 + tr S2 - 2 sum sqrt(max(lam, 0))
// -> out (float32 scalar), one launch
void fid_finish(const Tensor& sum1, double n1, const Tensor& sum2, double n2, const Tensor& s1, const Tensor& s2,
                const Tensor& lam, const Tensor& out) {
  check_gpu(sum1, "sum1");
  const int64_t d = sum1.numel();
  TORCH_CHECK(sum1.scalar_type() == at::kFloat && sum1.is_contiguous() && sum2.scalar_type() == at::kFloat &&
                  sum2.is_contiguous() && sum2.numel() == d,
              "fid_finish: sums must be contiguous float32 [d]");
  for (const Tensor* s : {&s1, &s2})
    TORCH_CHECK(s->scalar_type() == at::kDouble && s->dim() == 2 && s->size(0) == d && s->size(1) == d &&
                    s->stride(1) == 1 && s->device() == sum1.device(),
                "fid_finish: covariances must be row-contiguous float64 [d, d]");
  TORCH_CHECK(lam.scalar_type() == at::kDouble && lam.is_contiguous() && lam.device() == sum1.device(),
              "fid_finish: eigenvalues must be contiguous float64");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() == 1 && out.device() == sum1.device(),
              "fid_finish: out must be a float32 scalar");
  TORCH_CHECK(n1 > 0 && n2 > 0, "fid_finish: needs samples on both sides");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(sum1.device());
  check_launch(tea::launch_fid_finish(sum1.data_ptr<float>(), n1, sum2.data_ptr<float>(), n2, d, s1.data_ptr<double>(),
                                      s1.stride(0), s2.data_ptr<double>(), s2.stride(0), lam.data_ptr<double>(),
                                      lam.numel(), out.data_ptr<float>(), stream_for(sum1)),
               "fid_finish");
}

void sym_fill_upper(const Tensor& m) {
  check_gpu(m, "matrix");
  TORCH_CHECK(m.dim() == 2 && m.size(0) == m.size(1) && m.scalar_type() == at::kDouble && m.stride(1) == 1 &&
                  m.stride(0) >= m.size(1),
              "sym_fill_upper: matrix must be a row-contiguous float64 [n, n]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(m.device());
  check_launch(tea::launch_sym_fill_upper(m.data_ptr<double>(), m.stride(0), m.size(0), stream_for(m)),
               "sym_fill_upper");
}

// K2: multilabel accuracy counts straight into float32 state scalars.
void multilabel_counts(const Tensor& input, const Tensor& target, double threshold, int64_t k,
                       int64_t criteria, const Tensor& num_correct, const optional<Tensor>& num_total,
                       double total) {
  check_gpu(input, "input");
  check_gpu(target, "target");
  TORCH_CHECK(input.dim() == 2 && target.sizes() == input.sizes(),
              "multilabel_counts: input/target must be [n, c] of equal shape");
  TORCH_CHECK(input.stride(1) == 1 && target.stride(1) == 1,
              "multilabel_counts: rows must be contiguous");
  TORCH_CHECK(num_correct.scalar_type() == at::kFloat && num_correct.numel() == 1 &&
                  num_correct.device() == input.device(),
              "multilabel_counts: num_correct must be a float32 scalar on the input device");
  TORCH_CHECK(criteria >= 0 && criteria <= 4, "multilabel_counts: bad criteria");
  TORCH_CHECK(k == 0 || (k >= 1 && k <= input.size(1) && input.size(1) <= tea::multilabel_max_topk_cols()),
              "multilabel_counts: top-k needs 1 <= k <= c <= ", tea::multilabel_max_topk_cols());
  TORCH_CHECK(criteria != 1 || input.numel() < (int64_t{1} << 31),
              "multilabel_counts: hamming counts must fit 31 bits per launch");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(input.device());
  hipStream_t stream = stream_for(input);
  tea::MultilabelArgs a;
  a.x = input.data_ptr();
  a.x_dt = dt_of(input);
  a.x_row_stride = input.stride(0);
  a.t = target.data_ptr();
  a.t_dt = dt_of(target);
  a.t_row_stride = target.stride(0);
  a.n = input.size(0);
  a.c = input.size(1);
  a.threshold = static_cast<float>(threshold);
  a.k = static_cast<int>(k);
  a.criteria = static_cast<int>(criteria);
  a.num_correct = num_correct.data_ptr<float>();
  if (num_total.has_value()) {
    TORCH_CHECK(num_total->scalar_type() == at::kFloat && num_total->numel() == 1,
                "multilabel_counts: num_total must be a float32 scalar");
    a.num_total = num_total->data_ptr<float>();
    a.total = total;
  }
  a.fold_ws = fold_workspace(input, stream);
  const int rc = tea::launch_multilabel(a, stream);
  TORCH_CHECK(rc != -1, "multilabel_counts: unsupported dtypes ", input.scalar_type(), "/",
              target.scalar_type());
  check_launch(rc, "multilabel_counts");
}


// [n, c] (unit column stride) -> contiguous [c, n]
void transpose_f32(const Tensor& x, const Tensor& out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kFloat && x.stride(1) == 1, "transpose_f32: x [n, c] f32");
  TORCH_CHECK(out.is_contiguous() && out.scalar_type() == at::kFloat && out.size(0) == x.size(1) &&
                  out.size(1) == x.size(0), "transpose_f32: out must be contiguous [c, n]");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  check_launch(tea::launch_transpose_f32(x.data_ptr<float>(), x.size(0), x.size(1), x.stride(0),
                                         out.data_ptr<float>(), stream_for(x)), "transpose_f32");
}

// K3a: segmented descending radix sort of f32 rows -> (sorted scores, int32 permutation)
// Onesweep look-back timeouts (RadixArgs::os_hdr[8], set by a pass whose tile gave up waiting on
// its predecessors - forward progress relies on in-order workgroup dispatch per XCD).  Surfaced,
// never silent: the K3 scan reading that sort's output returns NaN (AucScanArgs::sort_fault), the
// word is copied asynchronously into pinned host memory after every onesweep sort, and the next
// sort on the stream that finds it set warns and sends every later sort of the process through
// the legacy (upsweep + downsweep) passes, which never wait on other workgroups.
struct OnesweepHealth {
  std::mutex mu;
  std::unordered_map<uint64_t, uint32_t*> host_word;  // (device, stream) -> pinned copy of hdr[8]
  std::atomic<bool> disabled{false};
};

OnesweepHealth& onesweep_health() {
  static auto& h = *new OnesweepHealth();  // process lifetime (no teardown after HIP's)
  return h;
}

uint64_t stream_key(const Tensor& x, hipStream_t st) {
  return (static_cast<uint64_t>(x.device().index()) << 56) ^ reinterpret_cast<uint64_t>(st);
}

// true when a previous onesweep sort on this stream reported a timeout (then the device word is
// cleared and onesweep is off for the process)
bool onesweep_faulted(const Tensor& x, hipStream_t st) {
  auto& h = onesweep_health();
  if (h.disabled.load()) return true;
  std::lock_guard<std::mutex> lock(h.mu);
  auto it = h.host_word.find(stream_key(x, st));
  if (it == h.host_word.end() || *reinterpret_cast<volatile uint32_t*>(it->second) == 0u) return false;
  h.disabled.store(true);
  auto* hdr = static_cast<uint32_t*>(zeroed_workspace(x, st, 16 * 4, 10));
  TORCH_CHECK(hipMemsetAsync(hdr + 8, 0, 4, st) == hipSuccess, "sort_desc: timeout word reset failed");
  static const char* kMsg =
      "torcheval_amd K3a: an onesweep radix sort timed out in its look-back (its K3 result was NaN); "
      "every later sort of this process takes the legacy radix passes";
  // a Python warning when called from Python (pybind11 entry points hold the GIL; TORCH_WARN from a
  // plain pybind11 function only reaches stderr), else c10's handler
  if (Py_IsInitialized() && PyGILState_Check()) {
    if (PyErr_WarnEx(PyExc_UserWarning, kMsg, 1) != 0) throw pybind11::error_already_set();
  } else {
    TORCH_WARN(kMsg);
  }
  return true;
}

// the pinned host word of this (device, stream) that each onesweep sort's histogram launch fills
// with the PREVIOUS sort's timeout word (RadixArgs::os_watch): a timed-out sort is reported one
// sort later (its own K3 scan already returned NaN from the device word), and no sort pays a
// device-to-host copy on its stream (the hipMemcpyAsync of round 5 was a ~5 us blit kernel in
// every binary_auroc's timeline)
uint32_t* onesweep_watch_word(const Tensor& x, hipStream_t st) {
  auto& h = onesweep_health();
  std::lock_guard<std::mutex> lock(h.mu);
  auto it = h.host_word.find(stream_key(x, st));
  if (it == h.host_word.end()) {
    void* p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent) != hipSuccess) return nullptr;
    std::memset(p, 0, 64);
    it = h.host_word.emplace(stream_key(x, st), static_cast<uint32_t*>(p)).first;
  }
  return it->second;
}

// `fold` (optional, float64 [rows, ceil(n / 1024), 2]): with a target / label payload on the
// onesweep path, the last pass also writes the K3 scan's 1024-sample tile totals there
// (RadixArgs::fold_ab) and the call returns true; pass it to auc_scan as `tsum`.  False: not
// folded (legacy sort, no payload), auc_scan must run its own tile_sums.
bool sort_desc(const Tensor& x, const Tensor& out_sorted, const Tensor& out_order,
               const optional<Tensor>& payload, int64_t payload_kind, const optional<Tensor>& fold,
               bool ascending = false) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kFloat && x.stride(1) == 1,
              "sort_desc: x must be float32 [rows, n] with contiguous rows");
  TORCH_CHECK(out_sorted.scalar_type() == at::kFloat && out_sorted.is_contiguous() &&
                  out_sorted.sizes() == x.sizes(), "sort_desc: out_sorted must be contiguous f32 [rows, n]");
  TORCH_CHECK(out_order.scalar_type() == at::kInt && out_order.is_contiguous() &&
                  out_order.sizes() == x.sizes(), "sort_desc: out_order must be contiguous int32 [rows, n]");
  TORCH_CHECK(x.size(1) < (int64_t{1} << 31), "sort_desc: rows longer than 2^31");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  tea::RadixArgs a;
  a.in = x.data_ptr<float>();
  a.in_row_stride = x.stride(0);
  a.rows = x.size(0);
  a.n = x.size(1);
  if (a.rows == 0 || a.n == 0) return false;
  a.tiles = tea::radix_sort_tiles(a.rows, a.n);
  const int64_t m = a.rows * a.n;
  Tensor ws = at::empty({4 * m + a.rows * 256 * a.tiles + a.rows * 512}, x.options().dtype(at::kInt));
  uint32_t* base = reinterpret_cast<uint32_t*>(ws.data_ptr<int32_t>());
  a.keys0 = base;
  a.vals0 = base + m;
  a.keys1 = base + 2 * m;
  a.vals1 = base + 3 * m;
  a.hist = base + 4 * m;
  uint32_t* bkt = a.hist + a.rows * 256 * a.tiles;  // splitter-bucket mode: splitters, bucket sizes
  a.ngroups = tea::radix_sort_groups(a.tiles);
  // self-cleaning: [header: cells left dirty in region 3 | pad | 4 regions of `region` cells]
  int64_t cap = 0;
  uint32_t* gws = static_cast<uint32_t*>(
      zeroed_workspace(x, stream_for(x), (4 + 4 * a.rows * a.ngroups * 256) * 4, 4, &cap));
  a.dirty = gws;
  a.groups = gws + 4;
  a.region = (cap / 4 - 4) / 4;  // fixed per buffer, so the next call finds region 3 at the same place
  a.out_sorted = out_sorted.data_ptr<float>();
  a.out_order = out_order.data_ptr<int32_t>();
  a.key_xor = ascending ? ~0u : 0u;  // stable either way; ascending puts NaN last (torch.sort)
  static const bool onesweep = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K3_ONESWEEP");
    return e == nullptr || e[0] != '0';
  }();
  a.spin_limit = [] {
    const char* e = std::getenv("TORCHEVAL_AMD_K3_SPIN_LIMIT");  // test hook: force timeouts
    const int v = e != nullptr ? std::atoi(e) : 0;
    return v > 0 ? v : (1 << 22);
  }();
  if (onesweep && tea::radix_onesweep_ok(a.rows, a.n) && !onesweep_faulted(x, stream_for(x))) {
    // self-cleaning onesweep state (tea_kernels.h RadixArgs): header + digit totals, the status
    // planes and the group planes in three zeroed workspaces whose plane strides depend only on
    // their capacity; if any of them is (re)allocated, all three restart from zero together
    hipStream_t st = stream_for(x);
    int64_t scap = 0, gcap = 0;
    auto* hdr = static_cast<uint32_t*>(zeroed_workspace(x, st, (16 + a.rows * 8 * 4 * 256) * 4, 10));
    auto* sws = static_cast<uint32_t*>(
        zeroed_workspace(x, st, 2 * tea::radix_onesweep_status_words(a.rows, a.n) * 4, 11, &scap));
    auto* gws = static_cast<unsigned long long*>(
        zeroed_workspace(x, st, 2 * tea::radix_onesweep_group_words(a.rows, a.n) * 8, 12, &gcap));
    {
      static std::mutex mu;
      static auto& seen = *new std::unordered_map<uint64_t, std::array<const void*, 3>>();
      const uint64_t key = (static_cast<uint64_t>(x.device().index()) << 56) ^ reinterpret_cast<uint64_t>(st);
      std::lock_guard<std::mutex> lock(mu);
      const std::array<const void*, 3> now{hdr, sws, gws};
      auto it = seen.find(key);
      if (it != seen.end() && it->second != now) {
        // one buffer is new (zero) while the others may hold another layout's dirty words
        TORCH_CHECK(hipMemsetAsync(hdr, 0, (16 + a.rows * 8 * 4 * 256) * 4, st) == hipSuccess &&
                        hipMemsetAsync(sws, 0, scap, st) == hipSuccess && hipMemsetAsync(gws, 0, gcap, st) == hipSuccess,
                    "sort_desc: workspace reset failed");
      }
      seen[key] = now;
    }
    a.os_hdr = hdr;
    a.os_g = hdr + 16;
    a.os_status = sws;
    a.os_splane = scap / 8;  // two u32 planes
    a.os_gacc = gws;
    a.os_gplane = gcap / 16;  // two u64 planes
    a.bkt_spl = bkt;
    a.bkt_cnt = bkt + a.rows * 256;
    a.os_watch = onesweep_watch_word(x, st);
  }
  Tensor pl;
  if (payload.has_value() && payload_kind != 0) {
    TORCH_CHECK(payload_kind == 1 || payload_kind == 2, "sort_desc: payload_kind must be 0, 1 or 2");
    pl = *payload;
    TORCH_CHECK(pl.device() == x.device(), "sort_desc: payload on another device");
    // [n] (shared by every row) or [rows, n], unit stride along samples
    if (pl.dim() == 1) {
      TORCH_CHECK(pl.size(0) == a.n, "sort_desc: payload must have n samples");
      if (!pl.is_contiguous()) pl = pl.contiguous();
      a.payload_row_stride = 0;
    } else {
      TORCH_CHECK(pl.dim() == 2 && pl.size(0) == a.rows && pl.size(1) == a.n, "sort_desc: payload must be [rows, n]");
      if (pl.stride(1) != 1) pl = pl.contiguous();
      a.payload_row_stride = pl.stride(0);
    }
    const auto st = pl.scalar_type();
    TORCH_CHECK(payload_kind == 1 ? (st == at::kFloat || st == at::kLong || st == at::kInt || st == at::kByte ||
                                     st == at::kBool)
                                  : (st == at::kLong || st == at::kInt),
                "sort_desc: unsupported payload dtype ", st);
    a.payload_kind = static_cast<int>(payload_kind);
    a.payload = pl.data_ptr();
    a.payload_dt = dt_of(pl);
  }
  const int64_t otiles = (a.n + 1023) / 1024;
  if (fold.has_value()) {
    TORCH_CHECK(fold->scalar_type() == at::kDouble && fold->is_contiguous() && fold->device() == x.device() &&
                    fold->numel() == a.rows * otiles * 2,
                "sort_desc: fold must be contiguous float64 [rows, ceil(n / 1024), 2] on the device of x");
    if (a.os_hdr != nullptr && a.payload_kind != 0) {
      a.fold_ab = fold->data_ptr<double>();
      a.fold_otiles = otiles;
      static const int probe = [] {
        const char* e = std::getenv("TORCHEVAL_AMD_K3_FOLD_PROBE");
        return e ? std::atoi(e) : 0;
      }();
      a.fold_probe = probe;
    }
  }
  check_launch(tea::launch_radix_sort_desc(a, stream_for(x)), "sort_desc");
  return a.fold_ab != nullptr;
}


// test hook: the onesweep look-back timeout word of `x`'s device / stream (0 = every spin of every
// sort on it completed), optionally cleared; one device-to-host read
int64_t sort_desc_timeouts(const Tensor& x, bool clear) {
  check_gpu(x, "x");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  hipStream_t st = stream_for(x);
  auto* hdr = static_cast<uint32_t*>(zeroed_workspace(x, st, 16 * 4, 10));
  uint32_t v = 0;
  TORCH_CHECK(hipMemcpyAsync(&v, hdr + 8, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
                  hipStreamSynchronize(st) == hipSuccess,
              "sort_desc_timeouts: read failed");
  if (clear && v != 0) TORCH_CHECK(hipMemsetAsync(hdr + 8, 0, 4, st) == hipSuccess, "sort_desc_timeouts: clear failed");
  return v;
}

// binned AUROC / AUPRC from [T, rows] float32 counts in one launch
void binned_finalize(const Tensor& tp, const Tensor& fp, const optional<Tensor>& fn,
                     const optional<Tensor>& out_auroc, const optional<Tensor>& out_auprc,
                     const optional<Tensor>& out_prec, const optional<Tensor>& out_rec) {
  check_gpu(tp, "tp");
  TORCH_CHECK(tp.dim() == 2 && tp.scalar_type() == at::kFloat && fp.sizes() == tp.sizes() &&
                  fp.strides() == tp.strides() && fp.scalar_type() == at::kFloat,
              "binned_finalize: tp/fp must be float32 [T, rows] with equal strides");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(tp.device());
  tea::BinnedFinalizeArgs a;
  a.tp = tp.data_ptr<float>();
  a.fp = fp.data_ptr<float>();
  a.k_stride = tp.stride(0);
  a.r_stride = tp.stride(1);
  a.T = static_cast<int>(tp.size(0));
  a.rows = tp.size(1);
  if (out_auprc.has_value()) {
    TORCH_CHECK(fn.has_value() && fn->sizes() == tp.sizes() && fn->strides() == tp.strides() &&
                    fn->scalar_type() == at::kFloat, "binned_finalize: AUPRC needs fn like tp");
    TORCH_CHECK(out_auprc->scalar_type() == at::kFloat && out_auprc->is_contiguous() &&
                    out_auprc->numel() == a.rows, "binned_finalize: out_auprc float32 [rows]");
    a.fn = fn->data_ptr<float>();
    a.out_auprc = out_auprc->data_ptr<float>();
  }
  if (out_auroc.has_value()) {
    TORCH_CHECK(out_auroc->scalar_type() == at::kDouble && out_auroc->is_contiguous() &&
                    out_auroc->numel() == a.rows, "binned_finalize: out_auroc float64 [rows]");
    a.out_auroc = out_auroc->data_ptr<double>();
  }
  if (out_prec.has_value() || out_rec.has_value()) {
    TORCH_CHECK(out_prec.has_value() && out_rec.has_value() && fn.has_value() &&
                    fn->sizes() == tp.sizes() && fn->strides() == tp.strides() &&
                    fn->scalar_type() == at::kFloat,
                "binned_finalize: a curve needs fn like tp and both out_prec / out_rec");
    for (const Tensor* o : {&*out_prec, &*out_rec})
      TORCH_CHECK(o->scalar_type() == at::kFloat && o->is_contiguous() &&
                      o->numel() == a.rows * (a.T + 1) && o->device() == tp.device(),
                  "binned_finalize: curve outputs must be contiguous float32 [rows, T + 1]");
    a.fn = fn->data_ptr<float>();
    a.out_prec = out_prec->data_ptr<float>();
    a.out_rec = out_rec->data_ptr<float>();
  }
  check_launch(tea::launch_binned_finalize(a, stream_for(tp)), "binned_finalize");
}


// ---------------------------------------------------------------- C3 flags inside the all-reduce
void snapshot_flags(const Tensor& src, const Tensor& dst, const optional<Tensor>& err, int64_t words, int64_t rank,
                    int64_t ws) {
  check_gpu(src, "src");
  TORCH_CHECK(src.scalar_type() == at::kByte && dst.scalar_type() == at::kByte && src.is_contiguous() &&
                  dst.is_contiguous() && dst.device() == src.device() && src.numel() % 16 == 0 &&
                  dst.numel() == src.numel() + ws * words * 8,
              "snapshot_flags: uint8 src [16k] and dst [src + ws * words * 8] on one device");
  const int* e = nullptr;
  if (err.has_value()) {
    TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= words && err->device() == src.device(),
                "snapshot_flags: err must be int32 [>= words]");
    e = err->data_ptr<int>();
  }
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  check_launch(tea::launch_snapshot_flags(src.data_ptr(), dst.data_ptr(), src.numel(), e, (int)words, (int)rank, (int)ws,
                                          stream_for(src)),
               "snapshot_flags");
}

void merge_flag_slots(const Tensor& slots, const Tensor& out, int64_t words, int64_t ws) {
  check_gpu(slots, "slots");
  TORCH_CHECK(slots.scalar_type() == at::kFloat && slots.is_contiguous() && slots.numel() == ws * words * 2 &&
                  out.scalar_type() == at::kInt && out.numel() == words && out.device() == slots.device(),
              "merge_flag_slots: float32 [ws * words * 2] slots and int32 [words] out");
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(slots.device());
  check_launch(tea::launch_merge_flag_slots(slots.data_ptr<float>(), out.data_ptr<int>(), (int)words, (int)ws,
                                            stream_for(slots)),
               "merge_flag_slots");
}

// ---------------------------------------------------------------- C3 gathered-state reduction
void seg_reduce_rows(const Tensor& rows, const Tensor& out, int64_t ws, at::IntArrayRef offs,
                     at::IntArrayRef counts, at::IntArrayRef dtypes, at::IntArrayRef ops) {
  check_gpu(rows, "rows");
  TORCH_CHECK(rows.scalar_type() == at::kByte && out.scalar_type() == at::kByte && rows.is_contiguous() &&
                  out.is_contiguous() && out.device() == rows.device(),
              "seg_reduce_rows: contiguous uint8 rows / out on one device expected");
  const int64_t nseg = static_cast<int64_t>(offs.size());
  TORCH_CHECK(nseg >= 1 && nseg <= tea::kSegMax && counts.size() == offs.size() && dtypes.size() == offs.size() &&
                  ops.size() == offs.size(),
              "seg_reduce_rows: 1..", tea::kSegMax, " segments with offs / counts / dtypes / ops each");
  TORCH_CHECK(ws >= 1 && rows.numel() == ws * out.numel(), "seg_reduce_rows: rows must be [ws * row_bytes]");
  static const int esize[] = {4, 2, 2, 8, 8, 4, 1, 1, 1, 2};  // by tea::DType
  tea::SegReduceArgs a;
  a.rows = rows.data_ptr<uint8_t>();
  a.out = out.data_ptr<uint8_t>();
  a.ws = static_cast<int>(ws);
  a.row_bytes = out.numel();
  a.nseg = static_cast<int>(nseg);
  for (int64_t s = 0; s < nseg; ++s) {
    TORCH_CHECK(dtypes[s] >= 0 && dtypes[s] <= 9 && ops[s] >= 0 && ops[s] <= 2 && counts[s] >= 0,
                "seg_reduce_rows: bad segment ", s);
    const int es = esize[dtypes[s]];
    TORCH_CHECK(offs[s] >= 0 && offs[s] % es == 0 && offs[s] + counts[s] * es <= a.row_bytes,
                "seg_reduce_rows: segment ", s, " outside the row or misaligned");
    a.off[s] = offs[s];
    a.first[s + 1] = a.first[s] + counts[s];
    a.dtype[s] = static_cast<int>(dtypes[s]);
    a.op[s] = static_cast<int>(ops[s]);
  }
  c10::hip::OptionalHIPGuardMasqueradingAsCUDA guard(rows.device());
  check_launch(tea::launch_seg_reduce(a, stream_for(rows)), "seg_reduce_rows");
}
}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "torcheval_amd native ops: hand-written HIP/CDNA4 kernels for MI355X (gfx950)";
  m.attr("ARCH") = "gfx950";
  m.def("rank_scores", &rank_scores, "K10 rank-of-target scores (hit rate / reciprocal rank)",
        py::arg("input"), py::arg("target"), py::arg("mode"), py::arg("k"), py::arg("err") = py::none());
  m.def("snapshot_flags", &snapshot_flags, "C3 snapshot of a state region + this rank's flag slot (f32 hi/lo)",
        py::arg("src"), py::arg("dst"), py::arg("err"), py::arg("words"), py::arg("rank"), py::arg("ws"));
  m.def("merge_flag_slots", &merge_flag_slots, "C3 summed flag slots -> int32 words (max over ranks)",
        py::arg("slots"), py::arg("out"), py::arg("words"), py::arg("ws"));
  m.def("seg_reduce_rows", &seg_reduce_rows,
        "C3 reduce a gathered [ws][row] state buffer per (op, dtype) segment in one launch", py::arg("rows"),
        py::arg("out"), py::arg("ws"), py::arg("offs"), py::arg("counts"), py::arg("dtypes"), py::arg("ops"));
  m.def("micro_accuracy_update", &micro_accuracy_update,
        "K1 micro accuracy (k=1) accumulated into float32 scalar states; false = not handled", py::arg("input"),
        py::arg("target"), py::arg("correct"), py::arg("total"), py::arg("num_classes") = 0,
        py::arg("pend") = py::none());
  m.def("micro_accuracy_finish", &micro_accuracy_finish,
        "fold the micro kernel's pending cells into correct (and write correct / total to out)", py::arg("pend"),
        py::arg("correct"), py::arg("total"), py::arg("out") = py::none());
  m.def("cls_counts", &cls_counts, "K1 fused classification counts", py::arg("input"),
        py::arg("target"), py::arg("k"), py::arg("num_classes"), py::arg("micro_correct"),
        py::arg("micro_total"), py::arg("cls_correct"), py::arg("cls_label"),
        py::arg("cls_pred"), py::arg("confusion"), py::arg("err"), py::arg("max_blocks") = 0,
        py::arg("micro_incorrect") = py::none(), py::arg("micro_total2") = py::none(),
        py::arg("cls_fp") = py::none());
  m.def("binary_counts", &binary_counts, "K1b thresholded binary counts", py::arg("input"),
        py::arg("target"), py::arg("weight"), py::arg("threshold"), py::arg("tp"),
        py::arg("fp"), py::arg("tn"), py::arg("fn"), py::arg("total"), py::arg("strict") = 0,
        py::arg("max_blocks") = 0, py::arg("tp2") = py::none(), py::arg("fp2") = py::none(),
        py::arg("tn2") = py::none(), py::arg("fn2") = py::none());
  m.def("auc_scan", &auc_scan, "K3 tie-aware scan -> AUROC / AUPRC per row", py::arg("sorted"),
        py::arg("order"), py::arg("target"), py::arg("weight"), py::arg("class_mode"),
        py::arg("out_auroc"), py::arg("out_auprc"), py::arg("init") = py::none(),
        py::arg("out_raw") = py::none(), py::arg("payload_kind") = 0, py::arg("tsum") = py::none());
  m.def("curve_workspace_bytes", &curve_workspace_bytes, "K3c workspace bytes", py::arg("rows"), py::arg("n"),
        py::arg("rafp"));
  m.def("curve_count", &curve_count, "K3c tile totals + tie-group tails + per-row scans (G_r -> sizes)",
        py::arg("sorted"), py::arg("order"), py::arg("target"), py::arg("class_mode"), py::arg("payload_kind"),
        py::arg("workspace"), py::arg("sizes"));
  m.def("curve_emit", &curve_emit, "K3c ascending precision / recall / threshold curves", py::arg("sorted"),
        py::arg("order"), py::arg("target"), py::arg("class_mode"), py::arg("payload_kind"), py::arg("workspace"),
        py::arg("sizes"), py::arg("row_off"), py::arg("out_prec"), py::arg("out_rec"), py::arg("out_thr"));
  m.def("rafp", &rafp, "K3c recall at fixed precision per row (sync-free)", py::arg("sorted"), py::arg("order"),
        py::arg("target"), py::arg("class_mode"), py::arg("payload_kind"), py::arg("min_precision"),
        py::arg("out_max_recall"), py::arg("out_best_thr"));
  m.def("merge_sorted_runs", &merge_sorted_runs,
        "K3m merge of descending-sorted runs -> (keys, int32 payload: carried or positions)", py::arg("keys"),
        py::arg("payloads") = py::none());
  m.def("retrieval_topk_update", &retrieval_topk_update,
        "K10b segmented streaming top-k merge into RetrievalPrecision state rows", py::arg("x"), py::arg("t"),
        py::arg("q"), py::arg("topk"), py::arg("target"), py::arg("count"));
  m.def("row_sums", &row_sums, "K5b per-row weighted sums merged into state tensors (GPU kernel / host twin)",
        py::arg("x"), py::arg("t"), py::arg("w"), py::arg("w_scalar"), py::arg("outs"), py::arg("codes"),
        py::arg("rows") = 1);
  m.def("binned_counts", &binned_counts, "K4 binned TP/FP/FN per (threshold, class)",
        py::arg("input"), py::arg("target"), py::arg("thr"), py::arg("mode"), py::arg("tp"),
        py::arg("fp"), py::arg("fn"), py::arg("uniform") = 0);
  m.def("column_moments", &column_moments, "K5 weighted column moments (+ fused MSE compute)",
        py::arg("x"), py::arg("t"), py::arg("w"), py::arg("sse"), py::arg("st"), py::arg("stt"),
        py::arg("sx"), py::arg("sw"), py::arg("overwrite") = 0, py::arg("mse_mode") = 0,
        py::arg("mse_out") = py::none(), py::arg("num_regressors") = 0);
  m.def("sample_binned_auroc", &sample_binned_auroc,
        "K4b per-sample multiclass binned AUROC (the reference default), labels checked into err",
        py::arg("input"), py::arg("target"), py::arg("thr"), py::arg("out"), py::arg("err"));
  m.def("row_sums_pend", &row_sums_pend,
        "K5b deferred-mode update: pre-scaled FP64 block partials added to pending slots; returns blocks used",
        py::arg("x"), py::arg("t"), py::arg("w"), py::arg("w_scalar"), py::arg("outs"), py::arg("codes"),
        py::arg("rows"), py::arg("pend"));
  m.def("row_sums_fold", &row_sums_fold, "K5b pending slots -> outputs (ADD), slots zeroed", py::arg("pend"),
        py::arg("used"), py::arg("outs"), py::arg("codes"), py::arg("rows"));
  m.def("column_moments_pend_numel", &column_moments_pend_numel, "deferred-mode pend buffer numel for (d, need)");
  m.def("column_moments_pend", &column_moments_pend,
        "K5 deferred-mode class update: FP64 column partials added to pending slots; returns the slots used",
        py::arg("x"), py::arg("t"), py::arg("w"), py::arg("sse"), py::arg("st"), py::arg("stt"), py::arg("sx"),
        py::arg("sw"), py::arg("pend"));
  m.def("column_moments_fold", &column_moments_fold, "K5 pending slots -> float32 states (+=), slots zeroed",
        py::arg("pend"), py::arg("slots"), py::arg("sse"), py::arg("st"), py::arg("stt"), py::arg("sx"),
        py::arg("sw"));
  m.def("ne_sums", &ne_sums, "K6 normalized-entropy row sums", py::arg("x"), py::arg("t"),
        py::arg("w"), py::arg("from_logits"), py::arg("out"), py::arg("err"),
        py::arg("deterministic") = false);
  m.def("perplexity_sums", &perplexity_sums, "K7 fused log-softmax gather", py::arg("input"),
        py::arg("target"), py::arg("ignore_index"), py::arg("out"), py::arg("err"),
        py::arg("deterministic") = false);
  m.def("multilabel_counts", &multilabel_counts, "K2 multilabel accuracy counts", py::arg("input"),
        py::arg("target"), py::arg("threshold"), py::arg("k"), py::arg("criteria"),
        py::arg("num_correct"), py::arg("num_total") = py::none(), py::arg("total") = 0.0);
  m.def("transpose_f32", &transpose_f32, "LDS-tiled [n, c] -> [c, n] float32 transpose", py::arg("x"),
        py::arg("out"));
  m.def("sort_desc_timeouts", &sort_desc_timeouts, "test hook: onesweep look-back timeout word (0 = none)",
        pybind11::arg("x"), pybind11::arg("clear") = true);
  m.def("sort_desc", &sort_desc, "K3a segmented stable radix sort, descending or ascending (f32 -> sorted, int32 order)",
        py::arg("x"), py::arg("out_sorted"), py::arg("out_order"), py::arg("payload") = py::none(),
        py::arg("payload_kind") = 0, py::arg("fold") = py::none(), py::arg("ascending") = false);
  m.def("binned_finalize", &binned_finalize, "binned AUROC / AUPRC / PR-curve points from counts",
        py::arg("tp"), py::arg("fp"), py::arg("fn") = py::none(), py::arg("out_auroc") = py::none(),
        py::arg("out_auprc") = py::none(), py::arg("out_prec") = py::none(),
        py::arg("out_rec") = py::none());
  m.def("fid_cov_update", &fid_cov_update, "K8 FP32-MFMA symmetric rank-k covariance update",
        py::arg("act"), py::arg("cov"), py::arg("colsum"));
  m.def("potrf_block", &potrf_block, "K9c diagonal-block FP64 Cholesky + inverse (blocked Cholesky step)",
        py::arg("a"), py::arg("k0"), py::arg("b"), py::arg("linv"), py::arg("info"));
  m.def("potrf_block_size", &tea::potrf_block_size, "K9c block size");
  m.def("cholesky_factor", &cholesky_factor, "K9d one-launch blocked FP64 Cholesky (padded factor, info, abort)",
        py::arg("a"), py::arg("l"), py::arg("linv"), py::arg("ctl"), py::arg("status"));
  m.def("cholesky_tiles", &tea::cholesky_tiles, "K9d 64 x 64 tiles per side");
  m.def("pivchol", &pivchol, "K9p pivoted FP64 Cholesky (rank-revealing, W rows in feature order)",
        py::arg("a"), py::arg("slots"), py::arg("w"), py::arg("piv"), py::arg("info"), py::arg("ctl"));
  m.def("pivchol_padded", &tea::pivchol_padded, "K9p factor row stride");
  m.def("fid_finish", &fid_finish, "FID's closing combination in one launch");
  m.def("pivchol_slot_words", &tea::pivchol_slot_words, "K9p hand-off slot words");
  m.def("pivchol_traced", &pivchol_traced, "K9p with per-panel phase stamps (profiling hook)");
  m.def("cholesky_factor_traced", &cholesky_factor_traced, "K9d with per-column phase stamps (profiling hook)");
  m.def("trapz_sorted", &trapz_sorted, "K3t trapezoid area per row of x-sorted (x, y)", py::arg("x"),
        py::arg("y_bits"), py::arg("out"));
  m.def("cov_finalize", &cov_finalize, "FP64 symmetric covariance from FP32 FID states",
        py::arg("cov_sum"), py::arg("colsum"), py::arg("n"), py::arg("out"));
  m.def("sym_fill_upper", &sym_fill_upper, "mirror the lower triangle of a float64 matrix into its upper",
        py::arg("m"));
  m.def("sym_eigvals", &sym_eigvals, "K9b eigenvalues of a symmetric float64 matrix (on-chip Householder + multisection)",
        py::arg("m"), py::arg("lam"), py::arg("status"));
  tea_register_runtime(m);
  tea_register_cpu_metrics(m);
  tea_register_rccl(m);
  tea_register_hostread(m);
}

// ---------------------------------------------------------------- torch dispatcher registration
// The same kernels as schema'd operators, ``torch.ops.torcheval_amd.<name>``: visible to the
// dispatcher (device routing, torch.compile graphs via the Meta kernels, profiler names,
// custom-op tooling).  The metric classes keep calling the pybind entry points above directly:
// one dispatcher hop costs a few us of host time per call, which the per-batch updates avoid.
// Every op mutates its outputs in place and returns nothing, so the Meta kernels are no-ops.
namespace {

void op_row_sums(const Tensor& x, const optional<Tensor>& t, const optional<Tensor>& w, double w_scalar,
                 at::TensorList outs, at::IntArrayRef codes, int64_t rows) {
  row_sums(x, t, w, w_scalar, outs.vec(), codes.vec(), rows);
}
void op_sort_desc(const Tensor& x, const Tensor& s, const Tensor& o, const optional<Tensor>& p, int64_t kind,
                  bool ascending) {
  sort_desc(x, s, o, p, kind, c10::nullopt, ascending);
}
void op_auc_scan(const Tensor& sorted, const Tensor& order, const Tensor& target, const optional<Tensor>& weight,
                 bool class_mode, const optional<Tensor>& out_auroc, const optional<Tensor>& out_auprc,
                 const optional<Tensor>& init, const optional<Tensor>& out_raw, int64_t payload_kind) {
  auc_scan(sorted, order, target, weight, class_mode, out_auroc, out_auprc, init, out_raw, payload_kind, c10::nullopt);
}
void op_rafp(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode, int64_t kind,
             double p, const Tensor& out_rec, const Tensor& out_thr) {
  rafp(sorted, order, target, class_mode, kind, p, out_rec, out_thr);
}
void op_fid_cov_update(const Tensor& act, const Tensor& cov, const optional<Tensor>& colsum) {
  fid_cov_update(act, cov, colsum);
}
void op_perplexity_sums(const Tensor& input, const Tensor& target, optional<int64_t> ignore_index,
                        const Tensor& out, const optional<Tensor>& err, bool deterministic) {
  perplexity_sums(input, target, ignore_index, out, err, deterministic);
}
void op_transpose_f32(const Tensor& x, const Tensor& out) { transpose_f32(x, out); }
void op_cls_counts(const Tensor& input, const Tensor& target, int64_t k, int64_t num_classes,
                   const optional<Tensor>& micro_correct, const optional<Tensor>& micro_total,
                   const optional<Tensor>& cls_correct, const optional<Tensor>& cls_label,
                   const optional<Tensor>& cls_pred, const optional<Tensor>& confusion,
                   const optional<Tensor>& err) {
  cls_counts(input, target, k, num_classes, micro_correct, micro_total, cls_correct, cls_label, cls_pred,
             confusion, err, 0, c10::nullopt, c10::nullopt, c10::nullopt);
}

// ---- dispatcher wrappers of the remaining entry points (schemas below annotate mutation)
void op_micro_accuracy(const Tensor& input, const Tensor& target, const Tensor& correct, const Tensor& total) {
  TORCH_CHECK(micro_accuracy_update(input, target, correct, total, 0, c10::nullopt),
              "micro_accuracy: unsupported input (needs [N, C] f32/bf16/f16 scores with unit column stride, "
              "[N] integer targets and float32 scalar states on one ROCm device)");
}
Tensor op_rank_scores(const Tensor& input, const Tensor& target, int64_t mode, int64_t k, const optional<Tensor>& err) {
  return rank_scores(input, target, mode, k, err);
}
void op_binary_counts(const Tensor& input, const Tensor& target, const optional<Tensor>& weight, double threshold,
                      const optional<Tensor>& tp, const optional<Tensor>& fp, const optional<Tensor>& tn,
                      const optional<Tensor>& fn, const optional<Tensor>& total, int64_t strict) {
  binary_counts(input, target, weight, threshold, tp, fp, tn, fn, total, strict, 0, c10::nullopt, c10::nullopt,
                c10::nullopt, c10::nullopt);
}
void op_curve_count(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode,
                    int64_t payload_kind, const Tensor& workspace, const Tensor& sizes) {
  curve_count(sorted, order, target, class_mode, payload_kind, workspace, sizes);
}
void op_curve_emit(const Tensor& sorted, const Tensor& order, const Tensor& target, bool class_mode,
                   int64_t payload_kind, const Tensor& workspace, const Tensor& sizes, const Tensor& row_off,
                   const Tensor& out_prec, const Tensor& out_rec, const Tensor& out_thr) {
  curve_emit(sorted, order, target, class_mode, payload_kind, workspace, sizes, row_off, out_prec, out_rec, out_thr);
}
std::vector<Tensor> op_merge_sorted_runs(at::TensorList keys, at::TensorList payloads) {
  optional<std::vector<Tensor>> pays;
  if (!payloads.empty()) pays = payloads.vec();  // [] = no payloads (positions come back)
  return merge_sorted_runs(keys.vec(), pays);
}
void op_retrieval_topk_update(const Tensor& x, const Tensor& t, const optional<Tensor>& q, const Tensor& topk,
                              const Tensor& target, const Tensor& count) {
  retrieval_topk_update(x, t, q, topk, target, count);
}
void op_binned_counts(const Tensor& input, const Tensor& target, const Tensor& thr, int64_t mode, const Tensor& tp,
                      const Tensor& fp, const Tensor& fn, int64_t uniform) {
  binned_counts(input, target, thr, mode, tp, fp, fn, uniform);
}
void op_column_moments(const optional<Tensor>& x, const optional<Tensor>& t, const optional<Tensor>& w,
                       const optional<Tensor>& sse, const optional<Tensor>& st, const optional<Tensor>& stt,
                       const optional<Tensor>& sx, const optional<Tensor>& sw, int64_t overwrite, int64_t mse_mode,
                       const optional<Tensor>& mse_out, int64_t num_regressors) {
  column_moments(x, t, w, sse, st, stt, sx, sw, overwrite, mse_mode, mse_out, num_regressors);
}
void op_ne_sums(const Tensor& x, const Tensor& t, const optional<Tensor>& w, bool from_logits, const Tensor& out,
                const optional<Tensor>& err, bool deterministic) {
  ne_sums(x, t, w, from_logits, out, err, deterministic);
}
void op_multilabel_counts(const Tensor& input, const Tensor& target, double threshold, int64_t k, int64_t criteria,
                          const Tensor& num_correct, const optional<Tensor>& num_total, double total) {
  multilabel_counts(input, target, threshold, k, criteria, num_correct, num_total, total);
}
void op_binned_finalize(const Tensor& tp, const Tensor& fp, const optional<Tensor>& fn,
                        const optional<Tensor>& out_auroc, const optional<Tensor>& out_auprc,
                        const optional<Tensor>& out_prec, const optional<Tensor>& out_rec) {
  binned_finalize(tp, fp, fn, out_auroc, out_auprc, out_prec, out_rec);
}
int64_t op_sym_eigvals(const Tensor& m, const Tensor& lam, const Tensor& status) { return sym_eigvals(m, lam, status); }
void op_cholesky_factor(const Tensor& a, const Tensor& l, const Tensor& linv, const Tensor& ctl, const Tensor& status) {
  cholesky_factor(a, l, linv, ctl, status);
}
void op_potrf_block(const Tensor& a, int64_t k0, int64_t b, const Tensor& linv, const Tensor& info) {
  potrf_block(a, k0, b, linv, info);
}
void op_seg_reduce_rows(const Tensor& rows, const Tensor& out, int64_t ws, at::IntArrayRef offs,
                        at::IntArrayRef counts, at::IntArrayRef dtypes, at::IntArrayRef ops) {
  seg_reduce_rows(rows, out, ws, offs, counts, dtypes, ops);
}

}  // namespace

TORCH_LIBRARY(torcheval_amd, m) {
  m.def("micro_accuracy(Tensor input, Tensor target, Tensor(a!) correct, Tensor(b!) total) -> ()");
  m.def("rank_scores(Tensor input, Tensor target, int score_mode, int k, Tensor(a!)? err) -> Tensor");
  m.def("binary_counts(Tensor input, Tensor target, Tensor? weight, float threshold, Tensor(a!)? tp, "
        "Tensor(b!)? fp, Tensor(c!)? tn, Tensor(d!)? fn, Tensor(e!)? total, int strict) -> ()");
  m.def("curve_count(Tensor sorted, Tensor order, Tensor target, bool class_mode, int payload_kind, "
        "Tensor(a!) workspace, Tensor(b!) sizes) -> ()");
  m.def("curve_emit(Tensor sorted, Tensor order, Tensor target, bool class_mode, int payload_kind, "
        "Tensor(a!) workspace, Tensor sizes, Tensor row_off, Tensor(b!) out_prec, Tensor(c!) out_rec, "
        "Tensor(d!) out_thr) -> ()");
  m.def("merge_sorted_runs(Tensor[] keys, Tensor[] payloads) -> Tensor[]");
  m.def("retrieval_topk_update(Tensor x, Tensor t, Tensor? q, Tensor(a!) topk, Tensor(b!) target, "
        "Tensor(c!) count) -> ()");
  m.def("binned_counts(Tensor input, Tensor target, Tensor thr, int target_mode, Tensor(a!) tp, Tensor(b!) fp, "
        "Tensor(c!) fn, int uniform) -> ()");
  m.def("column_moments(Tensor? x, Tensor? t, Tensor? w, Tensor(a!)? sse, Tensor(b!)? st, Tensor(c!)? stt, "
        "Tensor(d!)? sx, Tensor(e!)? sw, int overwrite, int mse_mode, Tensor(f!)? mse_out, int num_regressors) -> ()");
  m.def("ne_sums(Tensor x, Tensor t, Tensor? w, bool from_logits, Tensor(a!) out, Tensor(b!)? err, "
        "bool deterministic) -> ()");
  m.def("multilabel_counts(Tensor input, Tensor target, float threshold, int k, int criteria, "
        "Tensor(a!) num_correct, Tensor(b!)? num_total, float total) -> ()");
  m.def("binned_finalize(Tensor tp, Tensor fp, Tensor? fn, Tensor(a!)? out_auroc, Tensor(b!)? out_auprc, "
        "Tensor(c!)? out_prec, Tensor(d!)? out_rec) -> ()");
  m.def("sym_eigvals(Tensor m, Tensor(a!) lam, Tensor(b!) status) -> int");
  m.def("potrf_block(Tensor(a!) a, int k0, int b, Tensor(b!) linv, Tensor(c!) info) -> ()");
  m.def("cholesky_factor(Tensor a, Tensor(a!) l, Tensor(b!) linv, Tensor(c!) ctl, Tensor(d!) status) -> ()");
  m.def("pivchol(Tensor a, Tensor(a!) slots, Tensor(b!) w, Tensor(c!) piv, Tensor(d!) info, Tensor(e!) ctl) -> int");
  m.def("cov_finalize(Tensor cov_sum, Tensor colsum, float n, Tensor(a!) out) -> ()");
  m.def("sym_fill_upper(Tensor(a!) m) -> ()");
  m.def("fid_finish(Tensor sum1, float n1, Tensor sum2, float n2, Tensor s1, Tensor s2, Tensor lam, Tensor(a!) out) -> ()");
  m.def("trapz_sorted(Tensor x, Tensor y_bits, Tensor(a!) out) -> ()");
  m.def("seg_reduce_rows(Tensor rows, Tensor(a!) out, int ws, int[] offs, int[] counts, int[] dtypes, "
        "int[] ops) -> ()");
  m.def("row_sums(Tensor x, Tensor? t, Tensor? w, float w_scalar, Tensor(a!)[] outs, int[] codes, int rows) -> ()");
  m.def("sort_desc(Tensor x, Tensor(a!) sorted, Tensor(b!) order, Tensor? payload, int payload_kind, bool ascending=False) -> ()");
  m.def("auc_scan(Tensor sorted, Tensor order, Tensor target, Tensor? weight, bool class_mode, "
        "Tensor(a!)? out_auroc, Tensor(b!)? out_auprc, Tensor? init, Tensor(c!)? out_raw, int payload_kind) -> ()");
  m.def("rafp(Tensor sorted, Tensor order, Tensor target, bool class_mode, int payload_kind, float min_precision, "
        "Tensor(a!) out_max_recall, Tensor(b!) out_best_thr) -> ()");
  m.def("fid_cov_update(Tensor act, Tensor(a!) cov, Tensor(b!)? colsum) -> ()");
  m.def("perplexity_sums(Tensor input, Tensor target, int? ignore_index, Tensor(a!) out, Tensor(b!)? err, "
        "bool deterministic) -> ()");
  m.def("transpose_f32(Tensor x, Tensor(a!) out) -> ()");
  m.def("cls_counts(Tensor input, Tensor target, int k, int num_classes, Tensor(a!)? micro_correct, "
        "Tensor(b!)? micro_total, Tensor(c!)? cls_correct, Tensor(d!)? cls_label, Tensor(e!)? cls_pred, "
        "Tensor(f!)? confusion, Tensor(g!)? err) -> ()");
}

TORCH_LIBRARY_IMPL(torcheval_amd, CUDA, m) {
  m.impl("micro_accuracy", &op_micro_accuracy);
  m.impl("rank_scores", &op_rank_scores);
  m.impl("binary_counts", &op_binary_counts);
  m.impl("curve_count", &op_curve_count);
  m.impl("curve_emit", &op_curve_emit);
  m.impl("merge_sorted_runs", &op_merge_sorted_runs);
  m.impl("retrieval_topk_update", &op_retrieval_topk_update);
  m.impl("binned_counts", &op_binned_counts);
  m.impl("column_moments", &op_column_moments);
  m.impl("ne_sums", &op_ne_sums);
  m.impl("multilabel_counts", &op_multilabel_counts);
  m.impl("binned_finalize", &op_binned_finalize);
  m.impl("sym_eigvals", &op_sym_eigvals);
  m.impl("potrf_block", &op_potrf_block);
  m.impl("cholesky_factor", &op_cholesky_factor);
  m.impl("cov_finalize", &cov_finalize);
  m.impl("pivchol", &pivchol);
  m.impl("sym_fill_upper", &sym_fill_upper);
  m.impl("fid_finish", &fid_finish);
  m.impl("trapz_sorted", &trapz_sorted);
  m.impl("seg_reduce_rows", &op_seg_reduce_rows);
  m.impl("row_sums", &op_row_sums);
  m.impl("sort_desc", &op_sort_desc);
  m.impl("auc_scan", &op_auc_scan);
  m.impl("rafp", &op_rafp);
  m.impl("fid_cov_update", &op_fid_cov_update);
  m.impl("perplexity_sums", &op_perplexity_sums);
  m.impl("transpose_f32", &op_transpose_f32);
  m.impl("cls_counts", &op_cls_counts);
}

TORCH_LIBRARY_IMPL(torcheval_amd, CPU, m) {
  m.impl("row_sums", &op_row_sums);  // the C++ host twin
}

TORCH_LIBRARY_IMPL(torcheval_amd, Meta, m) {
  m.impl("micro_accuracy", [](const Tensor&, const Tensor&, const Tensor&, const Tensor&) {});
  m.impl("rank_scores", [](const Tensor& input, const Tensor&, int64_t, int64_t, const optional<Tensor>&) {
    return at::empty({input.size(0)}, input.options().dtype(at::kFloat));
  });
  m.impl("binary_counts", [](const Tensor&, const Tensor&, const optional<Tensor>&, double, const optional<Tensor>&,
                             const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&,
                             const optional<Tensor>&, int64_t) {});
  m.impl("retrieval_topk_update", [](const Tensor&, const Tensor&, const optional<Tensor>&, const Tensor&,
                                     const Tensor&, const Tensor&) {});
  m.impl("binned_counts", [](const Tensor&, const Tensor&, const Tensor&, int64_t, const Tensor&, const Tensor&,
                             const Tensor&, int64_t) {});
  m.impl("column_moments", [](const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&,
                              const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&,
                              const optional<Tensor>&, const optional<Tensor>&, int64_t, int64_t,
                              const optional<Tensor>&, int64_t) {});
  m.impl("ne_sums", [](const Tensor&, const Tensor&, const optional<Tensor>&, bool, const Tensor&,
                       const optional<Tensor>&, bool) {});
  m.impl("multilabel_counts", [](const Tensor&, const Tensor&, double, int64_t, int64_t, const Tensor&,
                                 const optional<Tensor>&, double) {});
  m.impl("binned_finalize", [](const Tensor&, const Tensor&, const optional<Tensor>&, const optional<Tensor>&,
                               const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&) {});
  m.impl("potrf_block", [](const Tensor&, int64_t, int64_t, const Tensor&, const Tensor&) {});
  m.impl("cholesky_factor", [](const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&) {});
  m.impl("cov_finalize", [](const Tensor&, const Tensor&, double, const Tensor&) {});
  m.impl("pivchol", [](const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&, const Tensor&) {
    return int64_t{0};
  });
  m.impl("sym_fill_upper", [](const Tensor&) {});
  m.impl("fid_finish", [](const Tensor&, double, const Tensor&, double, const Tensor&, const Tensor&, const Tensor&,
                          const Tensor&) {});
  m.impl("trapz_sorted", [](const Tensor&, const Tensor&, const Tensor&) {});
  m.impl("seg_reduce_rows", [](const Tensor&, const Tensor&, int64_t, at::IntArrayRef, at::IntArrayRef,
                               at::IntArrayRef, at::IntArrayRef) {});
  m.impl("cls_counts", [](const Tensor&, const Tensor&, int64_t, int64_t, const optional<Tensor>&,
                          const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&,
                          const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&) {});
  m.impl("auc_scan", [](const Tensor&, const Tensor&, const Tensor&, const optional<Tensor>&, bool,
                        const optional<Tensor>&, const optional<Tensor>&, const optional<Tensor>&,
                        const optional<Tensor>&, int64_t) {});
  m.impl("rafp", [](const Tensor&, const Tensor&, const Tensor&, bool, int64_t, double, const Tensor&,
                    const Tensor&) {});
  m.impl("perplexity_sums", [](const Tensor&, const Tensor&, optional<int64_t>, const Tensor&,
                               const optional<Tensor>&, bool) {});
  m.impl("row_sums", [](const Tensor&, const optional<Tensor>&, const optional<Tensor>&, double, at::TensorList,
                        at::IntArrayRef, int64_t) {});
  m.impl("sort_desc", [](const Tensor&, const Tensor&, const Tensor&, const optional<Tensor>&, int64_t, bool) {});
  m.impl("fid_cov_update", [](const Tensor&, const Tensor&, const optional<Tensor>&) {});
  m.impl("transpose_f32", [](const Tensor&, const Tensor&) {});
}
