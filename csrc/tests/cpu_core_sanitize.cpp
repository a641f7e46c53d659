// Host sanitizer driver for the CPU twins: the pointer-level cores of
// csrc/runtime/cpu_metrics.cpp (tea_cpu_core.h) and the K5b host twin (csrc/runtime/
// rowsums_host.cpp), built with -fsanitize=address,undefined by tests/test_sanitizers.py and run
// on randomized shapes (0, 1, odd, large), strides, NaN / inf values, weights and int / bool
// targets, each result checked against a naive formula written independently here.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <random>
#include <vector>

#include "tea_cpu_core.h"
#include "tea_kernels.h"

namespace {

int g_fail = 0;
#define CHECK(cond, ...)                          \
  do {                                            \
    if (!(cond)) {                                \
      ++g_fail;                                   \
      if (g_fail < 20) {                          \
        std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
        std::printf(__VA_ARGS__);                 \
        std::printf("\n");                        \
      }                                           \
    }                                             \
  } while (0)

std::mt19937 rng(20260);
int64_t rint(int64_t lo, int64_t hi) { return std::uniform_int_distribution<int64_t>(lo, hi)(rng); }
double runif() { return std::uniform_real_distribution<double>(0.0, 1.0)(rng); }
int64_t rsize() {  // 0, 1, small odd, large
  const int k = static_cast<int>(rint(0, 9));
  return k == 0 ? 0 : k == 1 ? 1 : k < 7 ? rint(2, 33) : rint(100, 2000);
}

template <typename T>
std::vector<T> rvec(int64_t n, double nan_p = 0.0, bool ties = false) {
  std::vector<T> v(n);
  for (auto& e : v) {
    double x = runif() * 4 - 2;
    if (ties) x = static_cast<int>(x * 2) / 2.0;
    if (runif() < nan_p) x = std::numeric_limits<double>::quiet_NaN();
    else if (runif() < nan_p / 2) x = std::numeric_limits<double>::infinity();
    e = static_cast<T>(x);
  }
  return v;
}

bool close(double a, double b, double tol) {
  if (a == b) return true;  // equal infinities included
  if (std::isnan(a) || std::isnan(b)) return std::isnan(a) && std::isnan(b);
  return std::fabs(a - b) <= tol * (1.0 + std::fabs(b));
}

// ---------------------------------------------------------------- classification counts
template <typename T>
void test_counts() {
  for (int it = 0; it < 400; ++it) {
    const int64_t n = rsize(), C = rint(1, 40), pad = rint(0, 3), ld = C + pad;
    std::vector<T> x = rvec<T>(n * ld + 1, 0.03, it % 2 == 0);
    std::vector<int64_t> t(n);
    for (auto& y : t) y = rint(0, C - 1);
    const int64_t k = it % 3 == 0 ? rint(2, 5) : 1;
    int64_t bad = 0;
    const int64_t got = tea_cpu::count_correct(x.data(), n, C, ld, t.data(), 1, k, &bad);
    int64_t want = 0;
    for (int64_t i = 0; i < n; ++i) {
      const T* row = x.data() + i * ld;
      if (k == 1) {  // first index of the max; NaN is the max
        int64_t best = 0;
        for (int64_t j = 0; j < C; ++j) {
          const bool nj = std::isnan(static_cast<double>(row[j])), nb = std::isnan(static_cast<double>(row[best]));
          if (nb) break;
          if (nj || row[j] > row[best]) best = j;
          if (nj) break;
        }
        want += best == t[i];
      } else {
        int64_t above = 0;
        for (int64_t j = 0; j < C; ++j) above += row[j] > row[t[i]];
        want += above < k;
      }
    }
    CHECK(bad == -1 && got == want, "count_correct n=%lld C=%lld k=%lld got %lld want %lld", (long long)n,
          (long long)C, (long long)k, (long long)got, (long long)want);
    // out-of-range target: reported, not read
    if (n > 0 && k > 1) {
      t[n - 1] = C + 3;
      tea_cpu::count_correct(x.data(), n, C, ld, t.data(), 1, k, &bad);
      CHECK(bad == n - 1, "bad target not reported");
    }
    // class histograms: labels (int32) and scores, incl. out-of-range labels flagged, skipped
    std::vector<int32_t> t32(n), p32(n);
    for (int64_t i = 0; i < n; ++i) {
      t32[i] = static_cast<int32_t>(it % 5 == 0 && i == 0 ? -1 : rint(0, C - 1));
      p32[i] = static_cast<int32_t>(it % 7 == 0 && i == 0 ? C : rint(0, C - 1));
    }
    std::vector<float> cc(C, 0), cl(C, 0), cp(C, 0), cf(C, 0), cm(C * C, 0), wc(C, 0), wl(C, 0), wp(C, 0), wf(C, 0),
        wm(C * C, 0);
    float mc = 0, mt = 0;
    int err = 0, werr = 0;
    tea_cpu::ClsOut o;
    o.mc = &mc;
    o.mt = &mt;
    o.cc = cc.data();
    o.cl = cl.data();
    o.cp = cp.data();
    o.cf = cf.data();
    o.cm = cm.data();
    o.err = &err;
    tea_cpu::Labels tl{t32.data(), false, 1}, pl{p32.data(), false, 1};
    tea_cpu::cls_counts<float>(nullptr, 0, pl, tl, n, C, 1, o);
    int64_t wcorrect = 0;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t y = t32[i], p = p32[i];
      const bool yok = y >= 0 && y < C, pok = p >= 0 && p < C, ok = p == y;
      wcorrect += ok;
      if (!yok) werr |= 1;
      if (!pok) werr |= 2;
      if (yok) {
        wl[y] += 1;
        if (ok) wc[y] += 1;
      }
      if (pok) {
        wp[p] += 1;
        if (!ok) wf[p] += 1;
      }
      if (yok && pok) wm[y * C + p] += 1;
    }
    CHECK(mc == static_cast<float>(wcorrect) && mt == static_cast<float>(n) && err == werr, "cls_counts micro / err");
    CHECK(cc == wc && cl == wl && cp == wp && cf == wf && cm == wm, "cls_counts histograms");
  }
}

// ---------------------------------------------------------------- binned histogram
template <typename S>
void test_binned() {
  for (int it = 0; it < 200; ++it) {
    const int64_t n = rsize(), C = rint(1, 12), T = rint(1, 30);
    std::vector<S> th = rvec<S>(T, 0.0, it % 2 == 1);
    for (auto& v : th) v = static_cast<S>((static_cast<double>(v) + 2) / 4);
    std::sort(th.begin(), th.end());
    std::vector<S> x = rvec<S>(n * C, 0.05, true);
    for (auto& v : x) v = std::isnan(static_cast<double>(v)) ? v : static_cast<S>((static_cast<double>(v) + 2) / 4);
    const int64_t mode = it % 2;
    std::vector<int64_t> lab(n);
    std::vector<uint8_t> tb(n * C);
    for (auto& l : lab) l = rint(0, C - 1);
    for (auto& b : tb) b = static_cast<uint8_t>(rint(0, 1));
    tea_cpu::Doubles tgt;
    if (mode == 1) tgt = {lab.data(), tea_cpu::Num::i64, 1, 0};
    else tgt = {tb.data(), tea_cpu::Num::b8, C, 1};
    std::vector<int64_t> hist;
    tea_cpu::binned_hist(x.data(), C, 1, n, C, th, mode, tgt, hist);
    std::vector<float> tp(T * C, 0), fp(T * C, 0), fn(T * C, 0);
    tea_cpu::binned_suffix(hist, T, C, tp.data(), fp.data(), fn.data(), C, 1);
    for (int64_t k = 0; k < T; ++k)
      for (int64_t c = 0; c < C; ++c) {
        int64_t wtp = 0, wfp = 0, wfn = 0;
        for (int64_t i = 0; i < n; ++i) {
          const S v = x[i * C + c];
          const bool pos = mode == 1 ? lab[i] == c : tb[i * C + c] == 1;
          // searchsorted(right=True) puts NaN past every threshold (the ATen form, ops/binned.py)
          const bool ge = std::isnan(static_cast<double>(v)) || v >= th[k];
          if (pos && ge) ++wtp;
          if (!pos && ge) ++wfp;
          if (pos && !ge) ++wfn;
        }
        CHECK(tp[k * C + c] == wtp && fp[k * C + c] == wfp && fn[k * C + c] == wfn, "binned k=%lld c=%lld",
              (long long)k, (long long)c);
      }
  }
}

// ---------------------------------------------------------------- AUROC / AUPRC rows
void test_auc() {
  for (int it = 0; it < 300; ++it) {
    const int64_t n = rsize();
    std::vector<float> x = rvec<float>(n, 0.03, it % 2 == 0);
    std::vector<double> t(n), w(n);
    for (auto& v : t) v = static_cast<double>(rint(0, 1));
    for (auto& v : w) v = runif();
    std::vector<int64_t> idx;
    double roc, pr;
    const bool weighted = it % 3 == 0;
    tea_cpu::auc_row(x.data(), n, 1, t, weighted ? &w : nullptr, idx, roc, pr);
    // naive AUROC: pairwise (pos, neg) with ties half, NaN highest (and tied only with itself)
    auto key = [&](int64_t i) { return std::isnan(static_cast<double>(x[i])) ? std::numeric_limits<double>::infinity() : x[i]; };
    double P = 0, N = 0, num = 0;
    for (int64_t i = 0; i < n; ++i) {
      const double wi = weighted ? w[i] : 1.0;
      P += wi * t[i];
      N += wi * (1 - t[i]);
    }
    for (int64_t i = 0; i < n; ++i)
      for (int64_t j = 0; j < n; ++j) {
        const double wp = (weighted ? w[i] : 1.0) * t[i], wn = (weighted ? w[j] : 1.0) * (1 - t[j]);
        if (wp == 0 || wn == 0) continue;
        const bool ni = std::isnan(static_cast<double>(x[i])), nj = std::isnan(static_cast<double>(x[j]));
        // NaN groups are singletons in the sorted scan: the earlier NaN counts as higher
        if (ni && nj) num += wp * wn * (i == j ? 0.5 : 0.5);
        else if (key(i) > key(j)) num += wp * wn;
        else if (key(i) == key(j)) num += 0.5 * wp * wn;
      }
    const double want = P * N == 0 ? 0.5 : num / (P * N);
    // NaN-vs-NaN pairs depend on the sort order; compare only NaN-free rows exactly
    bool has_nan = false;
    for (auto v : x) has_nan |= std::isnan(static_cast<double>(v));
    if (!has_nan) CHECK(close(roc, want, 1e-9), "auc_row roc %g want %g n=%lld", roc, want, (long long)n);
    CHECK(pr >= 0.0 && pr <= 1.0 + 1e-12, "auc_row pr %g out of [0, 1]", pr);
  }
}

// ---------------------------------------------------------------- binary accuracy / P / R
void test_binary() {
  for (int it = 0; it < 300; ++it) {
    const int64_t n = rsize(), sx = rint(1, 3);
    std::vector<double> x = rvec<double>(n * sx + 1, 0.05);
    std::vector<uint8_t> tb(n);
    std::vector<int64_t> ti(n);
    for (int64_t i = 0; i < n; ++i) ti[i] = tb[i] = static_cast<uint8_t>(rint(0, 1));
    const double thr = runif() - 0.5;
    const int64_t got = tea_cpu::count_binary_correct(x.data(), n, sx, tea_cpu::Doubles{tb.data(), tea_cpu::Num::b8, 1, 0}, thr);
    int64_t want = 0, s[4] = {0, 0, 0, 0}, w[4] = {0, 0, 0, 0};
    for (int64_t i = 0; i < n; ++i) {
      const int64_t p = x[i * sx] < thr ? 0 : 1;  // NaN < thr is false: predicts 1
      want += p == tb[i];
      w[0] += p * ti[i];
      w[1] += p & ti[i];
      w[2] += ti[i];
      w[3] += p;
    }
    tea_cpu::prf_sums(x.data(), n, sx, thr, ti, s);
    CHECK(got == want, "binary correct");
    CHECK(s[0] == w[0] && s[1] == w[1] && s[2] == w[2] && s[3] == w[3], "prf sums");
  }
}

// ---------------------------------------------------------------- MSE / R2 column sums
template <typename S>
void test_regression() {
  for (int it = 0; it < 300; ++it) {
    const int64_t n = rsize(), d = rint(1, 9), pad = rint(0, 2);
    const int64_t ld = d + pad;
    std::vector<S> x = rvec<S>(n * ld + 1, 0.02), t = rvec<S>(n * ld + 1, 0.02), w = rvec<S>(n + 1);
    const bool weighted = it % 2 == 0;
    std::vector<double> sse, sso, so, rss;
    double sw = 0;
    tea_cpu::mse_sums(x.data(), ld, 1, t.data(), ld, 1, weighted ? w.data() : nullptr, 1, n, d, sse, sw);
    tea_cpu::r2_sums(x.data(), ld, 1, t.data(), ld, 1, n, d, sso, so, rss);
    double wsw = 0;
    for (int64_t i = 0; i < n; ++i) wsw += weighted ? static_cast<double>(w[i]) : 1.0;
    CHECK(close(sw, wsw, 1e-12), "mse sw");
    for (int64_t c = 0; c < d; ++c) {
      double a = 0, b = 0, e2 = 0, e2w = 0;
      for (int64_t i = 0; i < n; ++i) {
        const double tv = t[i * ld + c], e = tv - static_cast<double>(x[i * ld + c]);
        a += tv * tv;
        b += tv;
        e2 += e * e;
        e2w += (weighted ? static_cast<double>(w[i]) : 1.0) * e * e;
      }
      CHECK(close(sse[c], e2w, 1e-9) && close(sso[c], a, 1e-9) && close(so[c], b, 1e-9) && close(rss[c], e2, 1e-9),
            "regression sums c=%lld", (long long)c);
    }
  }
}

// ---------------------------------------------------------------- class-API moment sums
template <typename S>
void test_moments() {
  for (int it = 0; it < 300; ++it) {
    const int64_t n = rsize(), d = rint(1, 9), pad = rint(0, 2);
    const int64_t ld = d + pad;
    std::vector<S> x = rvec<S>(n * ld + 1, 0.02), t = rvec<S>(n * ld + 1, 0.02), w = rvec<S>(n + 1);
    const bool weighted = it % 2 == 0, want_st = it % 3 != 0;
    std::vector<double> sse(d, -7), st(d, -7), stt(d, -7);  // overwritten, not accumulated
    double sw = -7;
    tea_cpu::moment_sums(x.data(), ld, 1, t.data(), ld, 1, weighted ? w.data() : nullptr, 1, n, d, sse.data(),
                         want_st ? st.data() : nullptr, stt.data(), sw);
    double wsw = 0;
    for (int64_t i = 0; i < n; ++i) wsw += weighted ? static_cast<double>(w[i]) : 1.0;
    CHECK(close(sw, wsw, 1e-12), "moments sw");
    for (int64_t c = 0; c < d; ++c) {
      double a = 0, b = 0, e2 = 0;
      for (int64_t i = 0; i < n; ++i) {
        const double wi = weighted ? static_cast<double>(w[i]) : 1.0;
        const double tv = t[i * ld + c], e = tv - static_cast<double>(x[i * ld + c]);
        a += wi * e * e;
        b += wi * tv;
        e2 += wi * tv * tv;
      }
      CHECK(close(sse[c], a, 1e-9) && close(stt[c], e2, 1e-9), "moments sse / stt c=%lld", (long long)c);
      CHECK(want_st ? close(st[c], b, 1e-9) : st[c] == -7, "moments st c=%lld", (long long)c);
    }
  }
}

// ---------------------------------------------------------------- class averages
void test_class_average() {
  for (int it = 0; it < 600; ++it) {
    const int64_t C = rint(1, 40);
    const int kind = static_cast<int>(rint(0, 3)), avg = kind == 0 ? 0 : static_cast<int>(rint(0, 1));
    std::vector<float> a(C), b(C), c(C);
    for (int64_t i = 0; i < C; ++i) {  // counts with zeros: absent classes, empty predictions
      b[i] = static_cast<float>(rint(0, 3) == 0 ? 0 : rint(0, 20));
      c[i] = static_cast<float>(rint(0, 3) == 0 ? 0 : rint(0, 20));
      a[i] = static_cast<float>(rint(0, static_cast<int64_t>(std::min(b[i], c[i]))));
    }
    bool zero = false;
    std::vector<int64_t> nan_idx;
    const float got = tea_cpu::class_average(kind, avg, a.data(), b.data(), c.data(), C, &zero, &nan_idx);
    // naive: the reference's masked expressions, element-wise in float32
    const std::vector<float>& label = kind == 2 ? c : b;
    double lsum = 0;
    for (float v : label) lsum += v;
    double num = 0;
    int64_t cnt = 0;
    bool any_zero = false;
    std::vector<int64_t> want_nan;
    for (int64_t i = 0; i < C; ++i) {
      any_zero |= b[i] == 0;
      bool keep;
      float v;
      if (kind == 0) { keep = b[i] != 0; v = a[i] / b[i]; }
      else if (kind == 1) { keep = b[i] != 0 || c[i] != 0; const float p = a[i] / c[i], r = a[i] / b[i]; v = tea_cpu::nan_to_num(2.f * p * r / (p + r)); }
      else if (kind == 2) { keep = c[i] != 0 || a[i] + b[i] != 0; v = tea_cpu::nan_to_num(a[i] / (a[i] + b[i])); }
      else { keep = b[i] != 0 || c[i] != 0; v = a[i] / b[i]; if (keep && std::isnan(v)) { want_nan.push_back(cnt); v = 0; } }
      if (!keep) continue;
      num += avg == 0 ? static_cast<double>(v) : static_cast<double>(v * (label[i] / static_cast<float>(lsum)));
      ++cnt;
    }
    const double want = avg == 0 ? num / static_cast<double>(cnt) : num;
    CHECK(close(got, static_cast<float>(want), 1e-6), "class_average kind %d avg %d C %lld: %g vs %g", kind, avg,
          (long long)C, static_cast<double>(got), want);
    if (kind == 1) CHECK(zero == any_zero, "class_average label-zero flag");
    if (kind == 3) CHECK(nan_idx == want_nan, "class_average recall NaN positions");
  }
}

// ---------------------------------------------------------------- confusion counts
template <typename S>
void test_confusion() {
  for (int it = 0; it < 300; ++it) {
    const int64_t n = rsize(), C = rint(2, 12), ld = C + rint(0, 2);
    const bool binary = it % 3 == 0, labels_in = !binary && it % 3 == 1;
    const int64_t Ce = binary ? 2 : C;
    std::vector<S> x = rvec<S>(n * ld + 1, 0.05, true);
    std::vector<int64_t> t(n), p(n);
    const bool bad = it % 11 == 0 && n > 0;
    for (int64_t i = 0; i < n; ++i) {
      t[i] = rint(0, Ce - 1);
      p[i] = rint(0, Ce - 1);
    }
    if (bad) t[rint(0, n - 1)] = Ce;
    tea_cpu::Labels tl{t.data(), true, 1}, pl{p.data(), true, 1};
    std::vector<int64_t> cm(Ce * Ce, 0);
    const bool ok = labels_in ? tea_cpu::confusion_counts<S>(nullptr, 0, pl, false, 0.0, tl, n, Ce, cm.data())
                              : tea_cpu::confusion_counts(x.data(), binary ? 1 : ld, tea_cpu::Labels{}, binary, 0.25,
                                                          tl, n, Ce, cm.data());
    CHECK(ok == !bad, "confusion validity");
    if (!ok) continue;
    std::vector<int64_t> want(Ce * Ce, 0);
    for (int64_t i = 0; i < n; ++i) {
      int64_t q;
      if (labels_in) q = p[i];
      else if (binary) q = x[i] < static_cast<S>(0.25) ? 0 : 1;
      else q = tea_cpu::row_argmax(x.data() + i * ld, C);
      ++want[t[i] * Ce + q];
    }
    CHECK(cm == want, "confusion counts n=%lld C=%lld binary=%d", (long long)n, (long long)Ce, binary);
  }
}

// ---------------------------------------------------------------- K5b host twin
void test_rowsums() {
  using namespace tea;
  for (int it = 0; it < 300; ++it) {
    const int64_t rows = rint(1, 5), n = rsize(), pad = rint(0, 3), rs = n + pad;
    std::vector<float> x = rvec<float>(rows * rs + 1, 0.02), t = rvec<float>(rows * rs + 1, 0.02),
                       w = rvec<float>(rows * rs + 1);
    std::vector<double> x64(x.begin(), x.end());
    const bool f64x = it % 4 == 1, weighted = it % 3 == 0;
    RowSumsArgs a;
    a.rows = rows;
    a.n = n;
    a.x = f64x ? static_cast<const void*>(x64.data()) : x.data();
    a.x_dt = f64x ? DType::f64 : DType::f32;
    a.x_rs = rs;
    a.x_cs = 1;
    a.t = t.data();
    a.t_dt = DType::f32;
    a.t_rs = rs;
    a.t_cs = 1;
    if (weighted) {
      a.w = w.data();
      a.w_dt = DType::f32;
      a.w_rs = rs;
      a.w_cs = 1;
    }
    a.w_scalar = weighted ? 1.0 : runif() * 3;
    // outputs: WX (f64 add), W (f32 add), WSSE (f64 set), TMIN (f32 min), TMAX (f64 max), COUNT
    // (f32 add, row 0 only), RANGE (f64 set)
    std::vector<double> o_wx(rows, 1.0), o_wsse(rows, 0.0), o_tmax(rows, -1e300), o_range(rows, 0.0);
    std::vector<float> o_w(rows, 2.f), o_tmin(rows, 1e30f), o_cnt(1, 0.f);
    struct Spec {
      void* p;
      DType dt;
      int stat, op, first;
    } specs[] = {{o_wx.data(), DType::f64, kWX, kAdd, 0},       {o_w.data(), DType::f32, kW, kAdd, 0},
                 {o_wsse.data(), DType::f64, kWSSE, kSet, 0},   {o_tmin.data(), DType::f32, kTMIN, kMin, 0},
                 {o_tmax.data(), DType::f64, kTMAX, kMax, 0},   {o_cnt.data(), DType::f32, kCOUNT, kAdd, 1},
                 {o_range.data(), DType::f64, kRANGE, kSet, 0}};
    a.nout = 7;
    int need = 0;
    for (int k = 0; k < 7; ++k) {
      a.out[k].p = specs[k].p;
      a.out[k].dt = specs[k].dt;
      a.out[k].stride = specs[k].first ? 0 : 1;
      a.out[k].stat = specs[k].stat;
      a.out[k].op = specs[k].op;
      a.out[k].first_row_only = specs[k].first;
      if (specs[k].stat < kCOUNT) need |= 1 << specs[k].stat;
    }
    a.need = need | (1 << kTMIN) | (1 << kTMAX);
    row_sums_host(a);
    for (int64_t r = 0; r < rows; ++r) {
      double wx = 0, ww = 0, wsse = 0, tmin = std::numeric_limits<double>::infinity(), tmax = -tmin;
      bool tnan = false;
      for (int64_t i = 0; i < n; ++i) {
        const double xv = x[r * rs + i], tv = t[r * rs + i], wv = weighted ? w[r * rs + i] : a.w_scalar;
        wx += wv * xv;
        ww += wv;
        wsse += wv * (xv - tv) * (xv - tv);
        tnan |= std::isnan(tv);
        tmin = std::fmin(tmin, tv);
        tmax = std::fmax(tmax, tv);
      }
      if (tnan) tmin = tmax = std::numeric_limits<double>::quiet_NaN();
      const double mmin = std::isnan(tmin) ? tmin : std::fmin(1e30f, static_cast<float>(tmin));
      const double mmax = std::isnan(tmax) ? tmax : std::fmax(-1e300, tmax);
      CHECK(close(o_wx[r], 1.0 + wx, 1e-9), "rowsums wx r=%lld n=%lld", (long long)r, (long long)n);
      CHECK(close(o_w[r], 2.0 + static_cast<float>(ww), 1e-5), "rowsums w");
      CHECK(close(o_wsse[r], wsse, 1e-9), "rowsums wsse");
      CHECK(close(o_tmin[r], mmin, 1e-6), "rowsums tmin %g vs %g", static_cast<double>(o_tmin[r]), mmin);
      CHECK(close(o_tmax[r], mmax, 1e-12), "rowsums tmax");
      CHECK(close(o_range[r], static_cast<double>(mmax) - static_cast<double>(static_cast<float>(mmin)), 1e-6) ||
                (std::isnan(o_range[r]) && (std::isnan(mmin) || std::isnan(mmax))),
            "rowsums range");
    }
    CHECK(o_cnt[0] == static_cast<float>(n), "rowsums count (row 0 only)");
  }
}

}  // namespace

int main() {
  test_counts<float>();
  test_counts<double>();
  test_binned<float>();
  test_binned<double>();
  test_auc();
  test_binary();
  test_regression<float>();
  test_regression<double>();
  test_moments<float>();
  test_moments<double>();
  test_class_average();
  test_confusion<float>();
  test_confusion<double>();
  test_rowsums();
  if (g_fail) {
    std::printf("cpu_core_sanitize: %d failures\n", g_fail);
    return 1;
  }
  std::printf("cpu_core_sanitize: ok\n");
  return 0;
}
