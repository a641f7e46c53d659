// Host (CPU) fast path for small classification updates.
//
// BASELINE.json config 1 is ``multiclass_accuracy`` on CPU with bs = 8, C = 6 (the reference's
// simple_example plumbing).  There the reference's cost is entirely per-op framework overhead:
// argmax -> eq -> long -> sum -> torch.tensor(N) -> div is six ATen dispatches plus
// allocations for 48 scores (accuracy.py:250-291).  This C++ op does the whole update +
// micro compute in one call: one pass over the rows (argmax with torch's NaN-is-max /
// first-index tie rule, or the rank-of-target test for k > 1) and a single 0-d output.
#include <ATen/ATen.h>
#include <pybind11/pybind11.h>
#include <torch/extension.h>

#include <cmath>
#include <cstdint>

#include "tea_runtime.h"

namespace {

template <typename T>
int64_t count_correct(const T* x, int64_t n, int64_t c, int64_t ld, const int64_t* t, int64_t ts, int64_t k) {
  int64_t correct = 0;
  for (int64_t i = 0; i < n; ++i) {
    const T* row = x + i * ld;
    const int64_t y = t[i * ts];
    if (k == 1) {
      int64_t best = 0;
      T bv = row[0];
      bool bnan = std::isnan(static_cast<double>(bv));
      for (int64_t j = 1; j < c && !bnan; ++j) {
        const T v = row[j];
        if (std::isnan(static_cast<double>(v))) {
          best = j;
          bnan = true;
        } else if (v > bv) {
          bv = v;
          best = j;
        }
      }
      correct += (best == y);
    } else {
      TORCH_CHECK(y >= 0 && y < c, "index ", y, " is out of bounds for dimension 1 with size ", c);
      const T ty = row[y];
      int64_t above = 0;
      for (int64_t j = 0; j < c; ++j) above += (row[j] > ty);
      correct += (above < k);
    }
  }
  return correct;
}

// correct predictions of input [N, C] float32/float64 scores (or [N] int64 labels) vs target [N] int64
int64_t count_micro(const at::Tensor& input, const at::Tensor& target, int64_t k) {
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda(), "cpu_micro_accuracy: CPU tensors only");
  TORCH_CHECK(target.dim() == 1 && target.scalar_type() == at::kLong, "cpu_micro_accuracy: target [N] int64");
  const int64_t n = target.size(0);
  int64_t correct = 0;
  if (input.dim() == 1) {
    TORCH_CHECK(input.scalar_type() == at::kLong && input.size(0) == n, "cpu_micro_accuracy: labels [N] int64");
    const int64_t* p = input.data_ptr<int64_t>();
    const int64_t* t = target.data_ptr<int64_t>();
    for (int64_t i = 0; i < n; ++i) correct += (p[i * input.stride(0)] == t[i * target.stride(0)]);
  } else {
    TORCH_CHECK(input.dim() == 2 && input.size(0) == n && input.stride(1) == 1,
                "cpu_micro_accuracy: scores [N, C] with unit column stride");
    const int64_t c = input.size(1);
    if (input.scalar_type() == at::kFloat)
      correct = count_correct(input.data_ptr<float>(), n, c, input.stride(0), target.data_ptr<int64_t>(),
                              target.stride(0), k);
    else if (input.scalar_type() == at::kDouble)
      correct = count_correct(input.data_ptr<double>(), n, c, input.stride(0), target.data_ptr<int64_t>(),
                              target.stride(0), k);
    else
      TORCH_CHECK(false, "cpu_micro_accuracy: float32/float64 scores");
  }
  return correct;
}

// -> 0-d float32 micro accuracy
at::Tensor cpu_micro_accuracy(const at::Tensor& input, const at::Tensor& target, int64_t k) {
  const int64_t correct = count_micro(input, target, k);
  const int64_t n = target.size(0);
  at::Tensor out = at::empty({}, at::TensorOptions().dtype(at::kFloat));
  out.data_ptr<float>()[0] = static_cast<float>(static_cast<double>(correct) / static_cast<double>(n));
  return out;
}

// class-API update: correct / total (0-d float32 states) += this batch's counts, in place
void cpu_micro_accuracy_update(const at::Tensor& input, const at::Tensor& target, int64_t k, at::Tensor& correct,
                               at::Tensor& total) {
  TORCH_CHECK(correct.dim() == 0 && total.dim() == 0 && correct.scalar_type() == at::kFloat &&
                  total.scalar_type() == at::kFloat && !correct.is_cuda() && !total.is_cuda(),
              "cpu_micro_accuracy_update: 0-d float32 CPU states");
  const int64_t c = count_micro(input, target, k);
  const int64_t n = target.size(0);
  // float32 adds, like the reference's ``num_correct += mask.sum()`` on float32 states
  correct.data_ptr<float>()[0] += static_cast<float>(c);
  total.data_ptr<float>()[0] += static_cast<float>(n);
}

}  // namespace

void tea_register_cpu_metrics(pybind11::module_& m) {
  m.def("cpu_micro_accuracy_update", &cpu_micro_accuracy_update,
        "host fast path of MulticlassAccuracy.update (micro): counts added into the states",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("k"), pybind11::arg("correct"),
        pybind11::arg("total"));
  m.def("cpu_micro_accuracy", &cpu_micro_accuracy,
        "host fast path: fused argmax / top-k test + micro accuracy for small CPU batches",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("k") = 1);
}
