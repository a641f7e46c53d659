// Pointer-level cores of the host (CPU) twins in csrc/runtime/cpu_metrics.cpp: no torch, no HIP,
// so tests/test_sanitizers.py can drive them under -fsanitize=address,undefined against naive
// formulas (csrc/tests/cpu_core_sanitize.cpp).  The ATen-facing wrappers validate shapes and
// dtypes and pass raw pointers + element strides here.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

namespace tea_cpu {

// element i of a 1-D int64 / int32 label vector
struct Labels {
  const void* p = nullptr;
  bool i64 = true;
  int64_t stride = 1;
  int64_t at(int64_t i) const {
    return i64 ? static_cast<const int64_t*>(p)[i * stride] : static_cast<int64_t>(static_cast<const int32_t*>(p)[i * stride]);
  }
};

// element (i, j) of a 2-D numeric tensor widened to double (targets / weights of any dtype)
enum class Num { f32, f64, i64, i32, i16, i8, u8, b8 };
struct Doubles {
  const void* p = nullptr;
  Num dt = Num::f64;
  int64_t s0 = 0, s1 = 0;
  double at(int64_t i, int64_t j = 0) const {
    const int64_t o = i * s0 + j * s1;
    switch (dt) {
      case Num::f32: return static_cast<const float*>(p)[o];
      case Num::f64: return static_cast<const double*>(p)[o];
      case Num::i64: return static_cast<double>(static_cast<const int64_t*>(p)[o]);
      case Num::i32: return static_cast<const int32_t*>(p)[o];
      case Num::i16: return static_cast<const int16_t*>(p)[o];
      case Num::i8: return static_cast<const int8_t*>(p)[o];
      case Num::u8: return static_cast<const uint8_t*>(p)[o];
      case Num::b8: return static_cast<const uint8_t*>(p)[o] != 0 ? 1.0 : 0.0;
    }
    return 0.0;
  }
};

// torch.argmax of one row: first index of the max, NaN counts as the max
template <typename T>
int64_t row_argmax(const T* row, int64_t c) {
  int64_t best = 0;
  T bv = row[0];
  if (std::isnan(static_cast<double>(bv))) return 0;
  for (int64_t j = 1; j < c; ++j) {
    const T v = row[j];
    if (std::isnan(static_cast<double>(v))) return j;
    if (v > bv) {
      bv = v;
      best = j;
    }
  }
  return best;
}

// micro-accuracy count over [n, c] rows (row stride ld): k == 1 argmax == target, else the
// rank-of-target test (strictly larger scores < k).  *bad_target: the index of the first row whose
// target is out of [0, c) in the k > 1 test (the caller raises the reference's index error), or -1.
template <typename T>
int64_t count_correct(const T* x, int64_t n, int64_t c, int64_t ld, const int64_t* t, int64_t ts, int64_t k,
                      int64_t* bad_target) {
  int64_t correct = 0;
  *bad_target = -1;
  for (int64_t i = 0; i < n; ++i) {
    const T* row = x + i * ld;
    const int64_t y = t[i * ts];
    if (k == 1) {
      correct += (row_argmax(row, c) == y);
    } else {
      if (y < 0 || y >= c) {
        *bad_target = i;
        return correct;
      }
      const T ty = row[y];
      int64_t above = 0;
      for (int64_t j = 0; j < c; ++j) above += (row[j] > ty);
      correct += (above < k);
    }
  }
  return correct;
}

// class-count outputs (float32, accumulated; null = not requested)
struct ClsOut {
  float *mc = nullptr, *mt = nullptr, *mi = nullptr, *mt2 = nullptr;  // micro correct / total / incorrect / total2
  float *cc = nullptr, *cl = nullptr, *cp = nullptr, *cf = nullptr;   // per class correct / label / pred / fp
  float* cm = nullptr;                                                // [C, C] confusion (target, pred)
  int* err = nullptr;                                                 // bit 0 bad target, bit 1 bad prediction
};

// The host twin of K1's contract: per row the prediction (argmax of scores [n, C] with row
// stride ld, or a label when scores is null) or, for k > 1, the rank-of-target test; then the
// micro counts and the class histograms.  Rows with an out-of-range label are skipped and flagged.
template <typename S>
void cls_counts(const S* scores, int64_t ld, const Labels& pred_labels, const Labels& target, int64_t n, int64_t C,
                int64_t k, const ClsOut& o) {
  int64_t correct_rows = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t t = target.at(i);
    const bool t_ok = t >= 0 && t < C;
    int64_t pred = -1;
    bool correct;
    if (!scores) {
      pred = pred_labels.at(i);
      correct = pred == t;
    } else if (k == 1) {
      pred = row_argmax(scores + i * ld, C);
      correct = pred == t;
    } else {
      int64_t above = 0;
      if (t_ok) {
        const S* row = scores + i * ld;
        for (int64_t j = 0; j < C; ++j) above += row[j] > row[t];
      }
      correct = t_ok && above < k;
    }
    correct_rows += correct;
    const bool p_ok = pred >= 0 && pred < C;
    if (o.err) {
      if (!t_ok) *o.err |= 1;
      if (!p_ok && (o.cp || o.cm || (o.cf && !correct))) *o.err |= 2;
    }
    if (t_ok) {
      if (o.cc && correct) o.cc[t] += 1.f;
      if (o.cl) o.cl[t] += 1.f;
    }
    if (p_ok && o.cp) o.cp[pred] += 1.f;
    if (p_ok && o.cf && !correct) o.cf[pred] += 1.f;
    if (t_ok && p_ok && o.cm) o.cm[t * C + pred] += 1.f;
  }
  if (o.mc) *o.mc += static_cast<float>(correct_rows);
  if (o.mi) *o.mi += static_cast<float>(n - correct_rows);
  if (o.mt) *o.mt += static_cast<float>(n);
  if (o.mt2) *o.mt2 += static_cast<float>(n);
}

// binned histogram [T + 1][C][neg, pos] of scores [n, C] (strides s0, s1) against ascending
// thresholds th[T] (in the score dtype); mode 1: labels (positive where label == class), mode 0:
// 0/1 targets [n, C]
template <typename S>
void binned_hist(const S* x, int64_t s0, int64_t s1, int64_t n, int64_t C, const std::vector<S>& th, int64_t mode,
                 const Doubles& target, std::vector<int64_t>& hist) {
  const int64_t T = static_cast<int64_t>(th.size());
  hist.assign((T + 1) * C * 2, 0);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t lab = mode == 1 ? static_cast<int64_t>(target.at(i)) : 0;
    for (int64_t c = 0; c < C; ++c) {
      const S v = x[i * s0 + c * s1];
      // searchsorted(thr, v, right=True): thresholds <= v; NaN sorts past every threshold
      int64_t b = T;
      if (!std::isnan(static_cast<double>(v))) b = std::upper_bound(th.begin(), th.end(), v) - th.begin();
      const bool pos = mode == 1 ? lab == c : target.at(i, c) == 1.0;
      ++hist[(b * C + c) * 2 + (pos ? 1 : 0)];
    }
  }
}

// tp / fp / fn [T, C] (float32, strides ts0 / ts1 shared) += the suffix counts of `hist`
inline void binned_suffix(const std::vector<int64_t>& hist, int64_t T, int64_t C, float* tp, float* fp, float* fn,
                          int64_t ts0, int64_t ts1) {
  for (int64_t c = 0; c < C; ++c) {
    int64_t pos_all = 0;
    for (int64_t b = 0; b <= T; ++b) pos_all += hist[(b * C + c) * 2 + 1];
    int64_t sp = 0, sn = 0;  // suffix sums over bins > k
    for (int64_t k = T - 1; k >= 0; --k) {
      sp += hist[((k + 1) * C + c) * 2 + 1];
      sn += hist[((k + 1) * C + c) * 2];
      tp[k * ts0 + c * ts1] += static_cast<float>(sp);
      fp[k * ts0 + c * ts1] += static_cast<float>(sn);
      fn[k * ts0 + c * ts1] += static_cast<float>(pos_all - sp);
    }
  }
}

// tie-aware binary AUROC / AUPRC of one row (x strided by sx, targets t, optional weights w)
template <typename S>
void auc_row(const S* x, int64_t n, int64_t sx, const std::vector<double>& t, const std::vector<double>* w,
             std::vector<int64_t>& idx, double& roc_out, double& pr_out) {
  idx.resize(n);
  for (int64_t i = 0; i < n; ++i) idx[i] = i;
  // torch.sort(descending=True) order: NaN above everything; ties in any order (only the
  // tie-group ends are used)
  std::sort(idx.begin(), idx.end(), [&](int64_t i, int64_t j) {
    const S a = x[i * sx], b = x[j * sx];
    if (std::isnan(static_cast<double>(a))) return !std::isnan(static_cast<double>(b));
    if (std::isnan(static_cast<double>(b))) return false;
    return a > b;
  });
  double tp = 0.0, fp = 0.0, tp0 = 0.0, fp0 = 0.0, roc = 0.0, pr = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const int64_t i = idx[k];
    const double wi = w ? (*w)[i] : 1.0;
    tp += wi * t[i];
    fp += wi * (1.0 - t[i]);
    // a group ends where the next sorted score differs (NaN != NaN: every NaN ends its own)
    if (k + 1 < n && x[idx[k + 1] * sx] == x[i * sx]) continue;
    roc += (fp - fp0) * (tp + tp0);
    const double den = tp + fp;
    pr += (tp - tp0) * (den > 0 ? tp / den : 0.0);
    tp0 = tp;
    fp0 = fp;
  }
  roc /= 2;
  roc_out = tp * fp == 0.0 ? 0.5 : roc / (tp * fp);
  pr_out = tp == 0.0 ? 0.0 : pr / tp;
}

// binary accuracy count: torch.where(x < thr, 0, 1) == t (NaN predicts 1)
template <typename S>
int64_t count_binary_correct(const S* x, int64_t n, int64_t sx, const Doubles& t, S thr) {
  int64_t correct = 0;
  for (int64_t i = 0; i < n; ++i) correct += ((x[i * sx] < thr ? 0.0 : 1.0) == t.at(i));
  return correct;
}

// (sum(pred * t), sum(pred & t), sum(t), sum(pred)) of thresholded predictions vs integer targets
template <typename S>
void prf_sums(const S* x, int64_t n, int64_t sx, S thr, const std::vector<int64_t>& t, int64_t* sums) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t pred = x[i * sx] < thr ? 0 : 1;  // torch.where(input < threshold, 0, 1)
    sums[0] += pred * t[i];
    sums[1] += pred & t[i];
    sums[2] += t[i];
    sums[3] += pred;
  }
}

// FP64 column sums of (weighted) squared errors of x, t [n, d] (strides (s0, s1) each; d = 1
// with s1 = 0 for 1-D), weights w [n] (stride ws0) or null; sw = total weight (n without weights)
template <typename S>
void mse_sums(const S* x, int64_t xs0, int64_t xs1, const S* t, int64_t ts0, int64_t ts1, const S* w, int64_t ws0,
              int64_t n, int64_t d, std::vector<double>& sse, double& sw) {
  sse.assign(d, 0.0);
  sw = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const double wi = w ? static_cast<double>(w[i * ws0]) : 1.0;
    sw += wi;
    for (int64_t c = 0; c < d; ++c) {
      const double e = static_cast<double>(t[i * ts0 + c * ts1]) - static_cast<double>(x[i * xs0 + c * xs1]);
      sse[c] += wi * e * e;
    }
  }
}

// FP64 column sums of R2: sum t^2, sum t, sum (t - x)^2
template <typename S>
void r2_sums(const S* x, int64_t xs0, int64_t xs1, const S* t, int64_t ts0, int64_t ts1, int64_t n, int64_t d,
             std::vector<double>& sso, std::vector<double>& so, std::vector<double>& rss) {
  sso.assign(d, 0.0);
  so.assign(d, 0.0);
  rss.assign(d, 0.0);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t c = 0; c < d; ++c) {
      const double tv = static_cast<double>(t[i * ts0 + c * ts1]);
      const double e = tv - static_cast<double>(x[i * xs0 + c * xs1]);
      sso[c] += tv * tv;
      so[c] += tv;
      rss[c] += e * e;
    }
}

// FP64 column sums for the class-API regression updates: sse = sum w (t - x)^2, st = sum w t,
// stt = sum w t^2 (null = not requested), sw = sum w (n without weights)
template <typename S>
void moment_sums(const S* x, int64_t xs0, int64_t xs1, const S* t, int64_t ts0, int64_t ts1, const S* w, int64_t ws0,
                 int64_t n, int64_t d, double* sse, double* st, double* stt, double& sw) {
  for (int64_t c = 0; c < d; ++c) {
    if (sse) sse[c] = 0.0;
    if (st) st[c] = 0.0;
    if (stt) stt[c] = 0.0;
  }
  sw = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const double wi = w ? static_cast<double>(w[i * ws0]) : 1.0;
    sw += wi;
    for (int64_t c = 0; c < d; ++c) {
      const double tv = static_cast<double>(t[i * ts0 + c * ts1]);
      if (sse) {
        const double e = tv - static_cast<double>(x[i * xs0 + c * xs1]);
        sse[c] += wi * e * e;
      }
      if (st) st[c] += wi * tv;
      if (stt) stt[c] += wi * tv * tv;
    }
  }
}

// torch.nan_to_num of a float32: NaN -> 0, +-inf -> +-FLT_MAX
inline float nan_to_num(float v) {
  if (std::isnan(v)) return 0.f;
  if (std::isinf(v)) return v > 0 ? 3.4028234663852886e38f : -3.4028234663852886e38f;
  return v;
}

// Macro / weighted class averages of float32 per-class counts [C], element-wise in float32 as the
// reference's tensor expressions are (the final mean / weighted sum accumulates in FP64):
//   kind 0 accuracy  (a correct, b total):      mean over total != 0 of a / b
//   kind 1 F1        (a tp, b label, c pred):    over label | pred != 0, nan_to_num(2 p r / (p + r))
//   kind 2 precision (a tp, b fp, c label):      over label | tp + fp != 0, nan_to_num(tp / (tp + fp))
//   kind 3 recall    (a tp, b label, c pred):    over label | pred != 0, tp / label (NaNs -> 0)
// avg 0 macro, 1 weighted (by label / sum(label) over all classes).  *label_zero: some class has
// no label (the F1 warning); nan_idx: recall's NaN positions within the masked vector.
inline float class_average(int kind, int avg, const float* a, const float* b, const float* c, int64_t C,
                           bool* label_zero, std::vector<int64_t>* nan_idx) {
  const float* label = kind == 2 ? c : b;
  double lsum_d = 0.0;
  for (int64_t i = 0; i < C; ++i) lsum_d += label[i];
  const float lsum = static_cast<float>(lsum_d);
  std::vector<float> vals, wts;
  vals.reserve(C);
  wts.reserve(C);
  for (int64_t i = 0; i < C; ++i) {
    float v;
    if (kind == 0) {
      if (b[i] == 0.f) continue;
      v = a[i] / b[i];
    } else if (kind == 1) {
      if (b[i] == 0.f && label_zero) *label_zero = true;
      if (b[i] == 0.f && c[i] == 0.f) continue;
      const float p = a[i] / c[i], r = a[i] / b[i];
      v = nan_to_num(2.f * p * r / (p + r));
    } else if (kind == 2) {
      if (c[i] == 0.f && a[i] + b[i] == 0.f) continue;
      v = nan_to_num(a[i] / (a[i] + b[i]));
    } else {
      if (b[i] == 0.f && c[i] == 0.f) continue;
      v = a[i] / b[i];
    }
    vals.push_back(v);
    wts.push_back(label[i] / lsum);
  }
  if (kind == 3) {  // torch.nan_to_num only runs when some class is NaN
    bool any = false;
    for (size_t j = 0; j < vals.size(); ++j)
      if (std::isnan(vals[j])) {
        any = true;
        if (nan_idx) nan_idx->push_back(static_cast<int64_t>(j));
      }
    if (any)
      for (float& v : vals) v = nan_to_num(v);
  }
  double acc = 0.0;
  if (avg == 0) {
    for (float v : vals) acc += v;
    return static_cast<float>(acc / static_cast<double>(vals.size()));  // empty: NaN, as mean([])
  }
  for (size_t j = 0; j < vals.size(); ++j) acc += static_cast<double>(vals[j] * wts[j]);
  return static_cast<float>(acc);
}

// confusion matrix [C, C] (target, prediction) counts of a small batch: prediction = argmax of
// scores [n, C] (row stride ld), a label, or (binary) score >= threshold.  False when some label is
// outside [0, C) (the caller's checking path raises the reference's error).
template <typename S>
bool confusion_counts(const S* scores, int64_t ld, const Labels& pred_labels, bool binary, double threshold,
                      const Labels& target, int64_t n, int64_t C, int64_t* cm) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t t = target.at(i);
    int64_t p;
    if (binary) p = scores[i * ld] < static_cast<S>(threshold) ? 0 : 1;  // torch.where(x < thr, 0, 1)
    else if (scores) p = row_argmax(scores + i * ld, C);
    else p = pred_labels.at(i);
    if (t < 0 || t >= C || p < 0 || p >= C) return false;
    cm[t * C + p] += 1;
  }
  return true;
}

}  // namespace tea_cpu
