// pybind11 entry points of torcheval_amd._C.
//
// This TU is the only one that includes torch headers: it validates tensors, picks the
// current HIP stream of the tensor's device and forwards raw pointers to the launchers in
// csrc/kernels/*.hip.  Every op fails loudly (TORCH_CHECK) on shapes/dtypes the kernels do
// not assume, so no kernel ever runs with a mismatched grid.
#include <torch/extension.h>

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
  static std::unordered_map<uint64_t, Tensor> cache;
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

void check_launch(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "torcheval_amd._C: ", what, " launch failed (code ", rc, ")");
}

// ---------------------------------------------------------------- K1 classification counts
void cls_counts(const Tensor& input, const Tensor& target, int64_t k, int64_t num_classes,
                const optional<Tensor>& micro_correct, const optional<Tensor>& micro_total,
                const optional<Tensor>& cls_correct, const optional<Tensor>& cls_label,
                const optional<Tensor>& cls_pred, const optional<Tensor>& confusion,
                const optional<Tensor>& err, int64_t max_blocks) {
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
  TORCH_CHECK(!(k > 1 && (a.cls_pred || a.confusion)),
              "cls_counts: predictions are undefined for k > 1");
  TORCH_CHECK((a.cls_correct || a.cls_label || a.cls_pred || a.confusion) == false || C > 0,
              "cls_counts: num_classes required for histograms");
  if (err.has_value()) {
    TORCH_CHECK(err->scalar_type() == at::kInt && err->numel() >= 1 && err->device() == input.device(),
                "cls_counts: err must be an int32 tensor on the input device");
    a.err = err->data_ptr<int>();
    a.check_target = 1;
  }
  a.max_blocks = static_cast<int>(max_blocks);
  const hipStream_t stream = stream_for(input);
  if (a.micro_correct) a.fold_ws = fold_workspace(input, stream);
  const int rc = tea::launch_cls_counts(a, stream);
  TORCH_CHECK(rc != -1, "cls_counts: unsupported input dtype ", input.scalar_type());
  check_launch(rc, "cls_counts");
}

void binary_counts(const Tensor& input, const Tensor& target, const optional<Tensor>& weight,
                   double threshold, const optional<Tensor>& tp, const optional<Tensor>& fp,
                   const optional<Tensor>& tn, const optional<Tensor>& fn,
                   const optional<Tensor>& total, int64_t strict, int64_t max_blocks) {
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
  a.max_blocks = static_cast<int>(max_blocks);
  check_launch(tea::launch_binary_counts(a, stream_for(input)), "binary_counts");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "torcheval_amd native ops: hand-written HIP/CDNA4 kernels for MI355X (gfx950)";
  m.attr("ARCH") = "gfx950";
  m.def("cls_counts", &cls_counts, "K1 fused classification counts", py::arg("input"),
        py::arg("target"), py::arg("k"), py::arg("num_classes"), py::arg("micro_correct"),
        py::arg("micro_total"), py::arg("cls_correct"), py::arg("cls_label"),
        py::arg("cls_pred"), py::arg("confusion"), py::arg("err"), py::arg("max_blocks") = 0);
  m.def("binary_counts", &binary_counts, "K1b thresholded binary counts", py::arg("input"),
        py::arg("target"), py::arg("weight"), py::arg("threshold"), py::arg("tp"),
        py::arg("fp"), py::arg("tn"), py::arg("fn"), py::arg("total"), py::arg("strict") = 0,
        py::arg("max_blocks") = 0);
  tea_register_runtime(m);
}
