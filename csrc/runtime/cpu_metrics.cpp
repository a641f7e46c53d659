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

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <tuple>
#include <vector>

#include "tea_cpu_core.h"
#include "tea_runtime.h"

namespace {

template <typename T>
int64_t count_correct(const T* x, int64_t n, int64_t c, int64_t ld, const int64_t* t, int64_t ts, int64_t k) {
  int64_t bad = -1;
  const int64_t correct = tea_cpu::count_correct(x, n, c, ld, t, ts, k, &bad);
  if (bad >= 0) {
    const int64_t y = t[bad * ts];
    TORCH_CHECK(false, "index ", y, " is out of bounds for dimension 1 with size ", c);
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

// ---- class-count updates (the CPU twin of the K1 kernel's contract, ops.classification) ----

int64_t label_at(const at::Tensor& t, int64_t i) {
  return t.scalar_type() == at::kLong ? t.data_ptr<int64_t>()[i * t.stride(0)]
                                      : static_cast<int64_t>(t.data_ptr<int32_t>()[i * t.stride(0)]);
}

bool label_dtype(const at::Tensor& t) { return t.scalar_type() == at::kLong || t.scalar_type() == at::kInt; }

// every target (and 1-D label input) in [0, num_classes): the CPU counts then never skip a row
bool cpu_labels_valid(const at::Tensor& input, const at::Tensor& target, int64_t num_classes) {
  if (input.is_cuda() || target.is_cuda() || target.dim() != 1 || !label_dtype(target)) return false;
  const int64_t n = target.size(0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t y = label_at(target, i);
    if (y < 0 || y >= num_classes) return false;
  }
  if (input.dim() == 1) {
    if (!label_dtype(input) || input.size(0) != n) return false;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t p = label_at(input, i);
      if (p < 0 || p >= num_classes) return false;
    }
  }
  return true;
}

tea_cpu::Labels labels_of(const at::Tensor& t) {
  tea_cpu::Labels l;
  l.p = t.data_ptr();
  l.i64 = t.scalar_type() == at::kLong;
  l.stride = t.stride(0);
  return l;
}

// a 1-D / 2-D numeric tensor for tea_cpu::Doubles (unsupported dtypes raise with `who`)
tea_cpu::Doubles doubles_of(const at::Tensor& t, const char* who) {
  tea_cpu::Doubles d;
  d.p = t.data_ptr();
  d.s0 = t.dim() >= 1 ? t.stride(0) : 0;
  d.s1 = t.dim() >= 2 ? t.stride(1) : 0;
  switch (t.scalar_type()) {
    case at::kFloat: d.dt = tea_cpu::Num::f32; break;
    case at::kDouble: d.dt = tea_cpu::Num::f64; break;
    case at::kLong: d.dt = tea_cpu::Num::i64; break;
    case at::kInt: d.dt = tea_cpu::Num::i32; break;
    case at::kShort: d.dt = tea_cpu::Num::i16; break;
    case at::kChar: d.dt = tea_cpu::Num::i8; break;
    case at::kByte: d.dt = tea_cpu::Num::u8; break;
    case at::kBool: d.dt = tea_cpu::Num::b8; break;
    default: TORCH_CHECK(false, who, ": unsupported dtype ", t.scalar_type());
  }
  return d;
}

float* opt_f32(const c10::optional<at::Tensor>& t, int64_t numel, const char* name) {
  if (!t.has_value()) return nullptr;
  TORCH_CHECK(!t->is_cuda() && t->scalar_type() == at::kFloat && t->is_contiguous() && t->numel() == numel,
              "cpu_cls_counts: ", name, " must be a contiguous float32 CPU tensor of ", numel, " elements");
  return t->data_ptr<float>();
}

// Same arguments and semantics as the HIP ``cls_counts`` (csrc/bindings.cpp): per row the
// prediction (argmax of [N, C] scores or the [N] label) or, for k > 1, the rank-of-target
// test; then micro counts and the class histograms, accumulated in float32.  Rows with an
// out-of-range label are skipped and flagged in ``err`` as on the GPU (callers validate first
// with cpu_labels_valid, so that only happens on direct use).
void cpu_cls_counts(const at::Tensor& input, const at::Tensor& target, int64_t k, int64_t num_classes,
                    const c10::optional<at::Tensor>& micro_correct, const c10::optional<at::Tensor>& micro_total,
                    const c10::optional<at::Tensor>& cls_correct, const c10::optional<at::Tensor>& cls_label,
                    const c10::optional<at::Tensor>& cls_pred, const c10::optional<at::Tensor>& confusion,
                    const c10::optional<at::Tensor>& err, int64_t /*max_blocks*/,
                    const c10::optional<at::Tensor>& micro_incorrect, const c10::optional<at::Tensor>& micro_total2,
                    const c10::optional<at::Tensor>& cls_fp) {
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda(), "cpu_cls_counts: CPU tensors only");
  TORCH_CHECK(target.dim() == 1 && label_dtype(target), "cpu_cls_counts: target [N] int64 / int32");
  const int64_t n = target.size(0), C = num_classes;
  const bool scores = input.dim() == 2;
  if (scores) {
    TORCH_CHECK(input.size(0) == n && input.stride(1) == 1 &&
                    (input.scalar_type() == at::kFloat || input.scalar_type() == at::kDouble),
                "cpu_cls_counts: scores [N, C] float32 / float64 with unit column stride");
    TORCH_CHECK(C == input.size(1), "cpu_cls_counts: num_classes must match input.size(1)");
  } else {
    TORCH_CHECK(input.dim() == 1 && input.size(0) == n && label_dtype(input) && k == 1,
                "cpu_cls_counts: labels [N] int64 / int32 (k = 1)");
  }
  float* mc = opt_f32(micro_correct, 1, "micro_correct");
  float* mt = opt_f32(micro_total, 1, "micro_total");
  float* mi = opt_f32(micro_incorrect, 1, "micro_incorrect");
  float* mt2 = opt_f32(micro_total2, 1, "micro_total2");
  float* cc = opt_f32(cls_correct, C, "cls_correct");
  float* cl = opt_f32(cls_label, C, "cls_label");
  float* cp = opt_f32(cls_pred, C, "cls_pred");
  float* cf = opt_f32(cls_fp, C, "cls_fp");
  float* cm = opt_f32(confusion, C * C, "confusion");
  TORCH_CHECK(!(k > 1 && (cp || cm || cf)), "cpu_cls_counts: predictions are undefined for k > 1");
  int* eb = nullptr;
  if (err.has_value()) {
    TORCH_CHECK(!err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "cpu_cls_counts: err int32");
    eb = err->data_ptr<int>();
  }
  tea_cpu::ClsOut o;
  o.mc = mc;
  o.mt = mt;
  o.mi = mi;
  o.mt2 = mt2;
  o.cc = cc;
  o.cl = cl;
  o.cp = cp;
  o.cf = cf;
  o.cm = cm;
  o.err = eb;
  const tea_cpu::Labels tl = labels_of(target);
  const tea_cpu::Labels pl = scores ? tea_cpu::Labels{} : labels_of(input);
  if (!scores)
    tea_cpu::cls_counts<float>(nullptr, 0, pl, tl, n, C, k, o);
  else if (input.scalar_type() == at::kFloat)
    tea_cpu::cls_counts(input.data_ptr<float>(), input.stride(0), pl, tl, n, C, k, o);
  else
    tea_cpu::cls_counts(input.data_ptr<double>(), input.stride(0), pl, tl, n, C, k, o);
}

// ---- binned counts (the CPU twin of K4 for small batches, ops.binned) ----

template <typename S>
void binned_hist(const at::Tensor& scores, const at::Tensor& target, const at::Tensor& thr, int64_t mode,
                 std::vector<int64_t>& hist) {
  const tea_cpu::Doubles tv = doubles_of(thr, "cpu_binned_counts");
  std::vector<S> th(thr.size(0));  // thresholds in the score dtype, as thr.to(scores.dtype)
  for (int64_t k = 0; k < thr.size(0); ++k) th[k] = static_cast<S>(tv.at(k));
  tea_cpu::binned_hist(scores.data_ptr<S>(), scores.stride(0), scores.stride(1), scores.size(0), scores.size(1), th,
                       mode, doubles_of(target, "cpu_binned_counts"), hist);
}

// scores [n, C] float32 / float64 (any strides), target [n, C] (mode 0) or [n] labels (mode 1),
// thr [T] sorted; tp / fp / fn [T, C] float32 views += the binned counts (tp[k] = positives
// with score >= thr[k], fp the negatives, fn = positives - tp), as _binned_counts_aten
void cpu_binned_counts(const at::Tensor& scores, const at::Tensor& target, const at::Tensor& thr, int64_t mode,
                       at::Tensor& tp, at::Tensor& fp, at::Tensor& fn) {
  TORCH_CHECK(!scores.is_cuda() && !target.is_cuda() && !thr.is_cuda(), "cpu_binned_counts: CPU tensors only");
  TORCH_CHECK(scores.dim() == 2 && thr.dim() == 1, "cpu_binned_counts: scores [n, C], thr [T]");
  const int64_t n = scores.size(0), C = scores.size(1), T = thr.size(0);
  TORCH_CHECK(mode == 1 ? (target.dim() == 1 && target.size(0) == n)
                        : (target.dim() == 2 && target.size(0) == n && target.size(1) == C),
              "cpu_binned_counts: target shape");
  for (const at::Tensor* o : {&tp, &fp, &fn})
    TORCH_CHECK(o->scalar_type() == at::kFloat && !o->is_cuda() && o->dim() == 2 && o->size(0) == T &&
                    o->size(1) == C, "cpu_binned_counts: outputs must be float32 [T, C]");
  TORCH_CHECK(tp.strides() == fp.strides() && tp.strides() == fn.strides(), "cpu_binned_counts: outputs share strides");
  std::vector<int64_t> hist;
  if (scores.scalar_type() == at::kFloat) binned_hist<float>(scores, target, thr, mode, hist);
  else if (scores.scalar_type() == at::kDouble) binned_hist<double>(scores, target, thr, mode, hist);
  else TORCH_CHECK(false, "cpu_binned_counts: float32 / float64 scores");
  tea_cpu::binned_suffix(hist, T, C, tp.data_ptr<float>(), fp.data_ptr<float>(), fn.data_ptr<float>(), tp.stride(0),
                         tp.stride(1));
}

// ---- tie-aware binary AUROC / AUPRC rows (host twin of the K3 sort-scan, _curve.py) ----

// row r of a [rows, n] tensor (any strides) widened to double
void row_as_double(const at::Tensor& t, int64_t r, std::vector<double>& out) {
  const int64_t n = t.size(1), s0 = t.stride(0), s1 = t.stride(1);
  out.resize(n);
  switch (t.scalar_type()) {
#define TEA_ROW(ST, CT)                                                          \
  case ST: {                                                                     \
    const CT* p = t.data_ptr<CT>() + r * s0;                                     \
    for (int64_t i = 0; i < n; ++i) out[i] = static_cast<double>(p[i * s1]);   \
    break;                                                                       \
  }
    TEA_ROW(at::kFloat, float)
    TEA_ROW(at::kDouble, double)
    TEA_ROW(at::kLong, int64_t)
    TEA_ROW(at::kInt, int32_t)
    TEA_ROW(at::kByte, uint8_t)
    TEA_ROW(at::kBool, bool)
#undef TEA_ROW
    default: TORCH_CHECK(false, "cpu_binary_auc: unsupported dtype ", t.scalar_type());
  }
}

// x [rows, n] float32 / float64 scores, t [rows, n] targets, w optional [rows, n] weights ->
// (roc, pr) float64 [rows]: AUROC (0.5 when a row has no positives or no negatives) and AUPRC
// (0 without positives) with the reference's tie semantics
std::tuple<at::Tensor, at::Tensor> cpu_binary_auc(const at::Tensor& x, const at::Tensor& t,
                                                  const c10::optional<at::Tensor>& w) {
  TORCH_CHECK(!x.is_cuda() && !t.is_cuda() && (!w.has_value() || !w->is_cuda()), "cpu_binary_auc: CPU tensors");
  TORCH_CHECK(x.dim() == 2 && t.sizes() == x.sizes() && (!w.has_value() || w->sizes() == x.sizes()),
              "cpu_binary_auc: x, t (and w) [rows, n]");
  const int64_t rows = x.size(0), n = x.size(1);
  const auto f64 = at::TensorOptions().dtype(at::kDouble);
  at::Tensor roc = at::empty({rows}, f64), pr = at::empty({rows}, f64);
  double* pr_ = pr.data_ptr<double>();
  double* roc_ = roc.data_ptr<double>();
  std::vector<double> tv, wv;
  std::vector<int64_t> idx;
  for (int64_t r = 0; r < rows; ++r) {
    row_as_double(t, r, tv);
    if (w.has_value()) row_as_double(*w, r, wv);
    const std::vector<double>* wp = w.has_value() ? &wv : nullptr;
    if (x.scalar_type() == at::kFloat)
      tea_cpu::auc_row(x.data_ptr<float>() + r * x.stride(0), n, x.stride(1), tv, wp, idx, roc_[r], pr_[r]);
    else if (x.scalar_type() == at::kDouble)
      tea_cpu::auc_row(x.data_ptr<double>() + r * x.stride(0), n, x.stride(1), tv, wp, idx, roc_[r], pr_[r]);
    else
      TORCH_CHECK(false, "cpu_binary_auc: float32 / float64 scores");
  }
  return {roc, pr};
}

// ---- binary accuracy (host twin of binary_counts' accuracy contract) ----

int64_t count_binary(const at::Tensor& input, const at::Tensor& target, double threshold) {
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda() && input.dim() == 1 && target.dim() == 1 &&
                  input.size(0) == target.size(0), "cpu_binary_accuracy: CPU [N] input and target");
  const int64_t n = input.size(0);
  if (input.scalar_type() == at::kFloat)
    return tea_cpu::count_binary_correct(input.data_ptr<float>(), n, input.stride(0), doubles_of(target, "cpu_binary_accuracy"),
                                         static_cast<float>(threshold));
  TORCH_CHECK(input.scalar_type() == at::kDouble, "cpu_binary_accuracy: float32 / float64 input");
  return tea_cpu::count_binary_correct(input.data_ptr<double>(), n, input.stride(0),
                                       doubles_of(target, "cpu_binary_accuracy"), threshold);
}

// functional: 0-d float32 accuracy (NaN for an empty batch, like 0 / 0)
at::Tensor cpu_binary_accuracy(const at::Tensor& input, const at::Tensor& target, double threshold) {
  const int64_t c = count_binary(input, target, threshold);
  at::Tensor out = at::empty({}, at::TensorOptions().dtype(at::kFloat));
  out.data_ptr<float>()[0] = static_cast<float>(c) / static_cast<float>(target.size(0));
  return out;
}

// class update: 0-d float32 states += (correct, N)
void cpu_binary_accuracy_update(const at::Tensor& input, const at::Tensor& target, double threshold,
                                at::Tensor& correct, at::Tensor& total) {
  TORCH_CHECK(correct.dim() == 0 && total.dim() == 0 && correct.scalar_type() == at::kFloat &&
                  total.scalar_type() == at::kFloat && !correct.is_cuda() && !total.is_cuda(),
              "cpu_binary_accuracy_update: 0-d float32 CPU states");
  const int64_t c = count_binary(input, target, threshold);
  correct.data_ptr<float>()[0] += static_cast<float>(c);
  total.data_ptr<float>()[0] += static_cast<float>(target.size(0));
}

// ---- binary precision / recall / F1 (small CPU batches, integer / bool targets) ----

// target [N] as int64 values
void target_as_i64(const at::Tensor& t, std::vector<int64_t>& out) {
  const int64_t n = t.size(0), st = t.stride(0);
  out.resize(n);
  switch (t.scalar_type()) {
#define TEA_T(ST, CT)                                                          \
  case ST: {                                                                   \
    const CT* p = t.data_ptr<CT>();                                            \
    for (int64_t i = 0; i < n; ++i) out[i] = static_cast<int64_t>(p[i * st]);  \
    break;                                                                     \
  }
    TEA_T(at::kLong, int64_t)
    TEA_T(at::kInt, int32_t)
    TEA_T(at::kShort, int16_t)
    TEA_T(at::kChar, int8_t)
    TEA_T(at::kByte, uint8_t)
    TEA_T(at::kBool, bool)
#undef TEA_T
    default: TORCH_CHECK(false, "cpu_binary_prf: integer / bool target expected");
  }
}

void prf_all_sums(const at::Tensor& input, const at::Tensor& target, double threshold, int64_t* sums) {
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda() && input.dim() == 1 && target.dim() == 1 &&
                  input.size(0) == target.size(0), "cpu_binary_prf: CPU [N] input and target");
  std::vector<int64_t> tv;
  target_as_i64(target, tv);
  const int64_t n = input.size(0);
  if (input.scalar_type() == at::kFloat)
    tea_cpu::prf_sums(input.data_ptr<float>(), n, input.stride(0), static_cast<float>(threshold), tv, sums);
  else if (input.scalar_type() == at::kDouble)
    tea_cpu::prf_sums(input.data_ptr<double>(), n, input.stride(0), threshold, tv, sums);
  else
    TORCH_CHECK(false, "cpu_binary_prf: float32 / float64 input");
}

// class updates: 0-d float32 states += this batch's counts (each count cast to float32 first, as
// ``state += int64_sum`` does).  kind 0 precision: (num_tp, num_fp) += (sum(pred * t),
// sum(pred) - sum(pred * t)); kind 1 recall: (num_tp, num_true_labels) += (sum(pred & t), sum(t));
// kind 2 F1: (num_tp, num_label, num_prediction) += (sum(pred * t), sum(t), sum(pred))
void cpu_binary_prf_update(const at::Tensor& input, const at::Tensor& target, double threshold, int64_t kind,
                           at::Tensor& a, at::Tensor& b, const c10::optional<at::Tensor>& c) {
  TORCH_CHECK(kind >= 0 && kind <= 2 && (kind != 2 || c.has_value()), "cpu_binary_prf_update: bad kind / states");
  const at::Tensor* states[3] = {&a, &b, c.has_value() ? &*c : &a};
  for (const at::Tensor* st : states)
    TORCH_CHECK(st->dim() == 0 && st->scalar_type() == at::kFloat && !st->is_cuda(),
                "cpu_binary_prf_update: 0-d float32 CPU states");
  int64_t sm[4] = {0, 0, 0, 0};  // sum(pred * t), sum(pred & t), sum(t), sum(pred)
  prf_all_sums(input, target, threshold, sm);
  float* pa = a.data_ptr<float>();
  float* pb = b.data_ptr<float>();
  if (kind == 0) {
    pa[0] += static_cast<float>(sm[0]);
    pb[0] += static_cast<float>(sm[3] - sm[0]);
  } else if (kind == 1) {
    pa[0] += static_cast<float>(sm[1]);
    pb[0] += static_cast<float>(sm[2]);
  } else {
    pa[0] += static_cast<float>(sm[0]);
    pb[0] += static_cast<float>(sm[2]);
    c->data_ptr<float>()[0] += static_cast<float>(sm[3]);
  }
}

// kind 0: precision = sum(pred * t) / sum(pred)            (NaN -> 0)
// kind 1: recall    = sum(pred & t) / sum(t)               (NaN -> 0, warn)
// kind 2: F1 from p = sum(pred * t) / sum(pred), r = sum(pred * t) / sum(t):
//         nan_to_num(2 * p * r / (p + r)), warn when sum(t) == 0
// -> (0-d float32 value, warn); every division and product in float32 in the reference's order
std::tuple<at::Tensor, bool> cpu_binary_prf(const at::Tensor& input, const at::Tensor& target, double threshold,
                                            int64_t kind) {
  TORCH_CHECK(kind >= 0 && kind <= 2, "cpu_binary_prf: kind 0 (precision), 1 (recall) or 2 (F1)");
  int64_t sm[4] = {0, 0, 0, 0};
  prf_all_sums(input, target, threshold, sm);
  const int64_t s_prod = sm[0], s_and = sm[1], s_t = sm[2], s_pred = sm[3];
  float v = 0.f;
  bool warn = false;
  auto nz = [](float x) {  // torch.nan_to_num: NaN -> 0, +-inf -> +-FLT_MAX
    return std::isnan(x) ? 0.f : (std::isinf(x) ? (x > 0 ? FLT_MAX : -FLT_MAX) : x);
  };
  if (kind == 0) {
    v = nz(static_cast<float>(s_prod) / static_cast<float>(s_pred));
  } else if (kind == 1) {
    v = static_cast<float>(s_and) / static_cast<float>(s_t);
    if (std::isnan(v)) {
      warn = true;
      v = 0.f;
    }
  } else {
    warn = s_t == 0;
    const float p = static_cast<float>(s_prod) / static_cast<float>(s_pred);
    const float r = static_cast<float>(s_prod) / static_cast<float>(s_t);
    v = nz(2.f * p * r / (p + r));
  }
  at::Tensor out = at::empty({}, at::TensorOptions().dtype(at::kFloat));
  out.data_ptr<float>()[0] = v;
  return {out, warn};
}

// ---- functional mean_squared_error (small CPU batches) ----

template <typename S>
void mse_sums(const at::Tensor& x, const at::Tensor& t, const c10::optional<at::Tensor>& w, std::vector<double>& sse,
              double& sw) {
  const int64_t n = x.size(0), d = x.dim() == 2 ? x.size(1) : 1;
  tea_cpu::mse_sums(x.data_ptr<S>(), x.stride(0), x.dim() == 2 ? x.stride(1) : 0, t.data_ptr<S>(), t.stride(0),
                    t.dim() == 2 ? t.stride(1) : 0, w.has_value() ? w->data_ptr<S>() : nullptr,
                    w.has_value() ? w->stride(0) : 0, n, d, sse, sw);
}

// sse / (clamp(|sw|, eps) * sign(sw)) per column in the input dtype (the reference's
// _mean_squared_error_compute; sw = N without weights), then the column mean unless raw_values
at::Tensor cpu_mse(const at::Tensor& x, const at::Tensor& t, const c10::optional<at::Tensor>& w, bool raw_values) {
  TORCH_CHECK(!x.is_cuda() && !t.is_cuda() && x.sizes() == t.sizes() && (x.dim() == 1 || x.dim() == 2) &&
                  x.scalar_type() == t.scalar_type() &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kDouble),
              "cpu_mse: CPU float32 / float64 [n] or [n, d] input and target of one dtype");
  TORCH_CHECK(!w.has_value() || (w->dim() == 1 && w->size(0) == x.size(0) && w->scalar_type() == x.scalar_type()),
              "cpu_mse: weight [n] of the input dtype");
  std::vector<double> sse;
  double sw = 0.0;
  if (x.scalar_type() == at::kFloat) mse_sums<float>(x, t, w, sse, sw);
  else mse_sums<double>(x, t, w, sse, sw);
  const int64_t d = static_cast<int64_t>(sse.size());
  const bool f32 = x.scalar_type() == at::kFloat;
  const double eps = 2.220446049250313e-16;  // torch.finfo(torch.float64).eps
  // the divisor is float32 without weights (int64 count -> clamp(min=eps) promotes to float32)
  // and in the weights' dtype with them
  const double den_d = (std::fabs(sw) < eps ? eps : std::fabs(sw)) * (sw > 0 ? 1.0 : (sw < 0 ? -1.0 : 0.0));
  const bool den_f32 = f32 || !w.has_value();
  const double den = den_f32 ? static_cast<double>(static_cast<float>(den_d)) : den_d;
  at::Tensor raw = at::empty(x.dim() == 2 ? std::vector<int64_t>{d} : std::vector<int64_t>{}, x.options());
  double acc = 0.0;
  for (int64_t c = 0; c < d; ++c) {
    double r;
    if (f32) {
      const float v = static_cast<float>(sse[c]) / static_cast<float>(den);
      r = v;
      raw.data_ptr<float>()[c] = v;
    } else {
      r = sse[c] / den;
      raw.data_ptr<double>()[c] = r;
    }
    acc += r;
  }
  if (raw_values) return raw;
  at::Tensor out = at::empty({}, x.options());
  if (f32) out.data_ptr<float>()[0] = static_cast<float>(acc / static_cast<double>(d));
  else out.data_ptr<double>()[0] = acc / static_cast<double>(d);
  return out;
}

// ---- functional r2_score (small CPU batches) ----

template <typename S>
at::Tensor r2_impl(const at::Tensor& x, const at::Tensor& t, int64_t mode, int64_t k) {
  const int64_t n = x.size(0), d = x.dim() == 2 ? x.size(1) : 1;
  const int64_t xs0 = x.stride(0), xs1 = x.dim() == 2 ? x.stride(1) : 0;
  const int64_t ts0 = t.stride(0), ts1 = t.dim() == 2 ? t.stride(1) : 0;
  std::vector<double> sso, so, rss;
  tea_cpu::r2_sums(x.data_ptr<S>(), xs0, xs1, t.data_ptr<S>(), ts0, ts1, n, d, sso, so, rss);
  // the reference's arithmetic in the input dtype: tss = sso - so^2 / n, r2 = 1 - rss / tss
  std::vector<S> tss(d), r2(d);
  S tss_sum = 0;
  for (int64_t c = 0; c < d; ++c) {
    const S a = static_cast<S>(sso[c]), b = static_cast<S>(so[c]), r = static_cast<S>(rss[c]);
    tss[c] = a - (b * b) / static_cast<S>(n);
    r2[c] = S(1) - r / tss[c];
    tss_sum += tss[c];
  }
  at::Tensor out;
  if (mode == 0) {  // raw_values
    out = at::empty(x.dim() == 2 ? std::vector<int64_t>{d} : std::vector<int64_t>{}, x.options());
    for (int64_t c = 0; c < d; ++c) out.data_ptr<S>()[c] = r2[c];
  } else {
    double acc = 0.0;
    for (int64_t c = 0; c < d; ++c) acc += mode == 1 ? static_cast<double>(r2[c]) : static_cast<double>(r2[c] * tss[c] / tss_sum);
    out = at::empty({}, x.options());
    out.data_ptr<S>()[0] = static_cast<S>(mode == 1 ? acc / static_cast<double>(d) : acc);
  }
  if (k != 0) {
    S* po = out.data_ptr<S>();
    for (int64_t c = 0; c < out.numel(); ++c)
      po[c] = S(1) - (S(1) - po[c]) * static_cast<S>(n - 1) / static_cast<S>(n - k - 1);
  }
  return out;
}

// mode 0 raw_values, 1 uniform_average, 2 variance_weighted; k = num_regressors (adjusted R2);
// the caller has checked n >= 2 and k < n - 1 (the reference's ValueErrors)
at::Tensor cpu_r2(const at::Tensor& x, const at::Tensor& t, int64_t mode, int64_t k) {
  TORCH_CHECK(!x.is_cuda() && !t.is_cuda() && x.sizes() == t.sizes() && (x.dim() == 1 || x.dim() == 2) &&
                  x.scalar_type() == t.scalar_type() &&
                  (x.scalar_type() == at::kFloat || x.scalar_type() == at::kDouble) && x.size(0) >= 2 &&
                  mode >= 0 && mode <= 2 && k >= 0 && k < x.size(0) - 1,
              "cpu_r2: CPU float32 / float64 [n >= 2] or [n, d] input and target of one dtype");
  return x.scalar_type() == at::kFloat ? r2_impl<float>(x, t, mode, k) : r2_impl<double>(x, t, mode, k);
}

// ---- class-API regression updates (small CPU batches) ----

bool f32_state(const c10::optional<at::Tensor>& s, int64_t numel, int64_t dim, float** out) {
  *out = nullptr;
  if (!s.has_value()) return true;
  if (s->is_cuda() || s->scalar_type() != at::kFloat || !s->is_contiguous() || s->numel() != numel || s->dim() != dim)
    return false;
  *out = s->data_ptr<float>();
  return true;
}

// MeanSquaredError / R2Score.update: this batch's FP64 column sums (tea_cpu::moment_sums) rounded
// to float32 and added into the states in place, as the reference's ``state += batch.sum(dim=0)``
// does; sw += sum w, or += n (``count``, and without weights).  x, t: float32 [n] or [n, d];
// the [d] states are 1-D for 2-D batches and 0-d for 1-D ones, sw is 0-d.  False (nothing
// written) for anything else: the caller's general path runs.
bool cpu_moments_update(const at::Tensor& x, const at::Tensor& t, const c10::optional<at::Tensor>& w,
                        const c10::optional<at::Tensor>& sse, const c10::optional<at::Tensor>& st,
                        const c10::optional<at::Tensor>& stt, const c10::optional<at::Tensor>& sw, bool count) {
  if (x.is_cuda() || t.is_cuda() || x.sizes() != t.sizes() || (x.dim() != 1 && x.dim() != 2) ||
      x.scalar_type() != at::kFloat || t.scalar_type() != at::kFloat || x.numel() == 0)
    return false;
  if (w.has_value() &&
      (w->is_cuda() || w->dim() != 1 || w->size(0) != x.size(0) || w->scalar_type() != at::kFloat))
    return false;
  const int64_t n = x.size(0), d = x.dim() == 2 ? x.size(1) : 1, sdim = x.dim() == 2 ? 1 : 0;
  float *psse, *pst, *pstt, *psw;
  if (!f32_state(sse, d, sdim, &psse) || !f32_state(st, d, sdim, &pst) || !f32_state(stt, d, sdim, &pstt) ||
      !f32_state(sw, 1, 0, &psw))
    return false;
  std::vector<double> buf(3 * d);
  double wsum = 0.0;
  tea_cpu::moment_sums(x.data_ptr<float>(), x.stride(0), x.dim() == 2 ? x.stride(1) : 0, t.data_ptr<float>(),
                       t.stride(0), t.dim() == 2 ? t.stride(1) : 0, w.has_value() ? w->data_ptr<float>() : nullptr,
                       w.has_value() ? w->stride(0) : 0, n, d, psse ? buf.data() : nullptr,
                       pst ? buf.data() + d : nullptr, pstt ? buf.data() + 2 * d : nullptr, wsum);
  for (int64_t c = 0; c < d; ++c) {
    if (psse) psse[c] += static_cast<float>(buf[c]);
    if (pst) pst[c] += static_cast<float>(buf[d + c]);
    if (pstt) pstt[c] += static_cast<float>(buf[2 * d + c]);
  }
  if (psw) psw[0] += static_cast<float>(count || !w.has_value() ? static_cast<double>(n) : wsum);
  return true;
}

// ---- macro / weighted averages of per-class counts (small CPU states) ----

// -> (0-d float32 average, some class has no label, recall's NaN positions in the masked vector);
// kinds and averages as tea_cpu::class_average
std::tuple<at::Tensor, bool, std::vector<int64_t>> cpu_class_average(int64_t kind, int64_t avg, const at::Tensor& a,
                                                                     const at::Tensor& b,
                                                                     const c10::optional<at::Tensor>& c) {
  TORCH_CHECK(kind >= 0 && kind <= 3 && (avg == 0 || (avg == 1 && kind != 0)) && (kind == 0 || c.has_value()),
              "cpu_class_average: bad kind / average");
  auto ok = [&](const at::Tensor& v) {
    return !v.is_cuda() && v.scalar_type() == at::kFloat && v.dim() == 1 && v.is_contiguous() && v.numel() == a.numel();
  };
  TORCH_CHECK(ok(a) && ok(b) && (!c.has_value() || ok(*c)), "cpu_class_average: contiguous float32 [C] CPU counts");
  bool label_zero = false;
  std::vector<int64_t> nan_idx;
  at::Tensor out = at::empty({}, at::TensorOptions().dtype(at::kFloat));
  out.data_ptr<float>()[0] = tea_cpu::class_average(static_cast<int>(kind), static_cast<int>(avg), a.data_ptr<float>(),
                                                    b.data_ptr<float>(), c.has_value() ? c->data_ptr<float>() : nullptr,
                                                    a.numel(), &label_zero, &nan_idx);
  return {out, label_zero, nan_idx};
}

// The macro / weighted multiclass functionals of a small CPU batch in one call: the class
// histograms (tea_cpu::cls_counts into local float32 arrays) and then tea_cpu::class_average.
// None when a label is out of range (the caller's ATen path raises the reference's error).
c10::optional<std::tuple<at::Tensor, bool, std::vector<int64_t>>> cpu_class_metric(int64_t kind, int64_t avg,
                                                                                   const at::Tensor& input,
                                                                                   const at::Tensor& target, int64_t C,
                                                                                   int64_t k) {
  TORCH_CHECK(kind >= 0 && kind <= 3 && (avg == 0 || (avg == 1 && kind != 0)) && C > 0 && k >= 1 &&
                  (k == 1 || kind == 0),
              "cpu_class_metric: bad kind / average / k");
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda() && target.dim() == 1 && label_dtype(target),
              "cpu_class_metric: CPU [N] int64 / int32 target");
  const int64_t n = target.size(0);
  const bool scores = input.dim() == 2;
  if (scores) {
    TORCH_CHECK(input.size(0) == n && input.size(1) == C && input.stride(1) == 1 &&
                    (input.scalar_type() == at::kFloat || input.scalar_type() == at::kDouble),
                "cpu_class_metric: scores [N, C] float32 / float64 with unit column stride");
  } else {
    TORCH_CHECK(input.dim() == 1 && input.size(0) == n && label_dtype(input) && k == 1,
                "cpu_class_metric: labels [N] int64 / int32");
  }
  if (!cpu_labels_valid(input, target, C)) return c10::nullopt;
  std::vector<float> cc(C, 0.f), cl(C, 0.f), cp(C, 0.f), cf(C, 0.f);
  tea_cpu::ClsOut o;
  o.cc = cc.data();
  o.cl = cl.data();
  if (k == 1) {
    o.cp = cp.data();
    o.cf = cf.data();
  }
  const tea_cpu::Labels tl = labels_of(target);
  if (!scores)
    tea_cpu::cls_counts<float>(nullptr, 0, labels_of(input), tl, n, C, k, o);
  else if (input.scalar_type() == at::kFloat)
    tea_cpu::cls_counts(input.data_ptr<float>(), input.stride(0), tea_cpu::Labels{}, tl, n, C, k, o);
  else
    tea_cpu::cls_counts(input.data_ptr<double>(), input.stride(0), tea_cpu::Labels{}, tl, n, C, k, o);
  // (a, b, c) per kind, as cpu_class_average
  const float* a = cc.data();
  const float* b = kind == 2 ? cf.data() : cl.data();
  const float* c = kind == 2 ? cl.data() : cp.data();
  bool label_zero = false;
  std::vector<int64_t> nan_idx;
  at::Tensor out = at::empty({}, at::TensorOptions().dtype(at::kFloat));
  out.data_ptr<float>()[0] = tea_cpu::class_average(static_cast<int>(kind), static_cast<int>(avg), a, b, c, C,
                                                    &label_zero, &nan_idx);
  return std::make_tuple(out, label_zero, nan_idx);
}

// ---- confusion matrices of small CPU batches ----

// [C, C] counts in the target's dtype (the reference's ``ones_like(target)`` values), or None when
// some label is out of range (the caller's checking path then raises the reference's error).
// binary: input [N] float scores thresholded (torch.where(x < thr, 0, 1)); else argmax of [N, C]
// float scores or [N] labels.
c10::optional<at::Tensor> cpu_confusion(const at::Tensor& input, const at::Tensor& target, int64_t C,
                                        double threshold, bool binary) {
  TORCH_CHECK(!input.is_cuda() && !target.is_cuda() && target.dim() == 1 && label_dtype(target) &&
                  input.size(0) == target.size(0) && C >= 2,
              "cpu_confusion: CPU [N] int64 / int32 target");
  const int64_t n = target.size(0);
  const bool flt = input.scalar_type() == at::kFloat || input.scalar_type() == at::kDouble;
  if (binary) {
    TORCH_CHECK(input.dim() == 1 && flt && C == 2, "cpu_confusion: binary input [N] float32 / float64");
  } else if (input.dim() == 2) {
    TORCH_CHECK(flt && input.size(1) == C && input.stride(1) == 1, "cpu_confusion: scores [N, C] float32 / float64");
  } else {
    TORCH_CHECK(input.dim() == 1 && label_dtype(input), "cpu_confusion: labels [N] int64 / int32");
  }
  std::vector<int64_t> cm(C * C, 0);
  const tea_cpu::Labels tl = labels_of(target);
  bool ok;
  if (!binary && input.dim() == 1)
    ok = tea_cpu::confusion_counts<float>(nullptr, 0, labels_of(input), false, 0.0, tl, n, C, cm.data());
  else if (input.scalar_type() == at::kFloat)
    ok = tea_cpu::confusion_counts(input.data_ptr<float>(), input.stride(0), tea_cpu::Labels{},
                                   binary, threshold, tl, n, C, cm.data());
  else
    ok = tea_cpu::confusion_counts(input.data_ptr<double>(), input.stride(0), tea_cpu::Labels{}, binary, threshold,
                                   tl, n, C, cm.data());
  if (!ok) return c10::nullopt;
  at::Tensor out = at::empty({C, C}, at::TensorOptions().dtype(target.scalar_type()));
  if (target.scalar_type() == at::kLong) std::copy(cm.begin(), cm.end(), out.data_ptr<int64_t>());
  else
    for (int64_t i = 0; i < C * C; ++i) out.data_ptr<int32_t>()[i] = static_cast<int32_t>(cm[i]);
  return out;
}

}  // namespace

void tea_register_cpu_metrics(pybind11::module_& m) {
  m.def("cpu_binary_accuracy", &cpu_binary_accuracy, "host fast path of binary_accuracy for small CPU batches",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("threshold"));
  m.def("cpu_binary_accuracy_update", &cpu_binary_accuracy_update,
        "host fast path of BinaryAccuracy.update: counts added into the 0-d float32 states", pybind11::arg("input"),
        pybind11::arg("target"), pybind11::arg("threshold"), pybind11::arg("correct"), pybind11::arg("total"));
  m.def("cpu_binary_prf", &cpu_binary_prf,
        "host fast path of binary_precision / binary_recall / binary_f1_score (integer / bool targets)",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("threshold"), pybind11::arg("kind"));
  m.def("cpu_binary_prf_update", &cpu_binary_prf_update,
        "host fast path of BinaryPrecision / BinaryRecall / BinaryF1Score.update (0-d float32 states)",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("threshold"), pybind11::arg("kind"),
        pybind11::arg("a"), pybind11::arg("b"), pybind11::arg("c") = pybind11::none());
  m.def("cpu_r2", &cpu_r2, "host fast path of the functional r2_score for small CPU batches", pybind11::arg("x"),
        pybind11::arg("t"), pybind11::arg("mode"), pybind11::arg("num_regressors"));
  m.def("cpu_mse", &cpu_mse, "host fast path of the functional mean_squared_error for small CPU batches",
        pybind11::arg("x"), pybind11::arg("t"), pybind11::arg("w") = pybind11::none(), pybind11::arg("raw_values") = false);
  m.def("cpu_binary_auc", &cpu_binary_auc, "host twin of the K3 AUROC / AUPRC rows for small CPU batches",
        pybind11::arg("x"), pybind11::arg("t"), pybind11::arg("w") = pybind11::none());
  m.def("cpu_binned_counts", &cpu_binned_counts, "host twin of binned_counts for small CPU batches");
  m.def("cpu_labels_valid", &cpu_labels_valid, "all targets / label predictions in [0, num_classes)");
  m.def("cpu_cls_counts", &cpu_cls_counts, "host twin of cls_counts for small CPU batches");
  m.def("cpu_micro_accuracy_update", &cpu_micro_accuracy_update,
        "host fast path of MulticlassAccuracy.update (micro): counts added into the states",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("k"), pybind11::arg("correct"),
        pybind11::arg("total"));
  m.def("cpu_moments_update", &cpu_moments_update,
        "host fast path of MeanSquaredError / R2Score.update: FP64 batch sums added into float32 states",
        pybind11::arg("x"), pybind11::arg("t"), pybind11::arg("w"), pybind11::arg("sse"), pybind11::arg("st"),
        pybind11::arg("stt"), pybind11::arg("sw"), pybind11::arg("count"));
  m.def("cpu_class_average", &cpu_class_average,
        "macro / weighted accuracy, F1, precision, recall of float32 per-class counts (small CPU states)",
        pybind11::arg("kind"), pybind11::arg("average"), pybind11::arg("a"), pybind11::arg("b"),
        pybind11::arg("c") = pybind11::none());
  m.def("cpu_class_metric", &cpu_class_metric,
        "macro / weighted multiclass accuracy, F1, precision, recall of a small CPU batch in one call",
        pybind11::arg("kind"), pybind11::arg("average"), pybind11::arg("input"), pybind11::arg("target"),
        pybind11::arg("num_classes"), pybind11::arg("k") = 1);
  m.def("cpu_confusion", &cpu_confusion, "host fast path of the confusion-matrix functionals for small CPU batches",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("num_classes"), pybind11::arg("threshold"),
        pybind11::arg("binary"));
  m.def("cpu_micro_accuracy", &cpu_micro_accuracy,
        "host fast path: fused argmax / top-k test + micro accuracy for small CPU batches",
        pybind11::arg("input"), pybind11::arg("target"), pybind11::arg("k") = 1);
}
