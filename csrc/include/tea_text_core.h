// Pure C++ core of the text-metric runtime (no Python / pybind dependency), shared by the
// extension (csrc/runtime/text.cpp) and the sanitizer driver (csrc/tests/text_core_sanitize.cpp).
#pragma once

#include <algorithm>
#include <cstdint>
#include <climits>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

namespace tea_text {

using Tokens = std::vector<std::string>;

struct Interner {
  std::unordered_map<std::string, int> ids;
  int get(const std::string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const int id = static_cast<int>(ids.size());
    ids.emplace(s, id);
    return id;
  }
  std::vector<int> map(const Tokens& t) {
    std::vector<int> out;
    out.reserve(t.size());
    for (const auto& s : t) out.push_back(get(s));
    return out;
  }
};

inline int64_t levenshtein(const std::vector<int>& a, const std::vector<int>& b) {
  const size_t n = a.size(), m = b.size();
  std::vector<int64_t> prev(m + 1), cur(m + 1);
  for (size_t j = 0; j <= m; ++j) prev[j] = static_cast<int64_t>(j);
  for (size_t i = 1; i <= n; ++i) {
    cur[0] = static_cast<int64_t>(i);
    for (size_t j = 1; j <= m; ++j) {
      if (a[i - 1] == b[j - 1]) {
        cur[j] = prev[j - 1];
      } else {
        cur[j] = std::min({prev[j], cur[j - 1], prev[j - 1]}) + 1;
      }
    }
    std::swap(prev, cur);
  }
  return prev[m];
}

// errors, max_total, target_total, input_total (the reference's _get_errors_and_totals)
inline std::tuple<double, double, double, double> errors_and_totals(const std::vector<Tokens>& inputs,
                                                             const std::vector<Tokens>& targets) {
  double errors = 0, max_total = 0, target_total = 0, input_total = 0;
  const size_t n = std::min(inputs.size(), targets.size());
  {
    for (size_t p = 0; p < n; ++p) {
      Interner in;
      const auto a = in.map(inputs[p]);
      const auto b = in.map(targets[p]);
      errors += static_cast<double>(levenshtein(a, b));
      target_total += static_cast<double>(b.size());
      input_total += static_cast<double>(a.size());
      max_total += static_cast<double>(std::max(a.size(), b.size()));
    }
  }
  return {errors, max_total, target_total, input_total};
}

struct VecHash {
  size_t operator()(const std::vector<int>& v) const {
    uint64_t h = 1469598103934665603ull;
    for (int x : v) {
      h ^= static_cast<uint64_t>(x) + 0x9e3779b97f4a7c15ull;
      h *= 1099511628211ull;
    }
    return static_cast<size_t>(h);
  }
};

using NgramCounts = std::unordered_map<std::vector<int>, int64_t, VecHash>;

inline NgramCounts ngrams(const std::vector<int>& s, int n_gram) {
  NgramCounts c;
  for (int n = 1; n <= n_gram; ++n) {
    for (int64_t i = 0; i + n <= static_cast<int64_t>(s.size()); ++i) {
      c[std::vector<int>(s.begin() + i, s.begin() + i + n)] += 1;
    }
  }
  return c;
}

// input_len, target_len, matches_by_order[n_gram], possible_matches_by_order[n_gram]
inline std::tuple<int64_t, int64_t, std::vector<double>, std::vector<double>> bleu_counts(
    const std::vector<Tokens>& candidates, const std::vector<std::vector<Tokens>>& references,
    int n_gram) {
  int64_t input_len = 0, target_len = 0;
  std::vector<double> matches(n_gram, 0.0), possible(n_gram, 0.0);
  {
    Interner in;
    for (size_t p = 0; p < candidates.size() && p < references.size(); ++p) {
      const auto cand = in.map(candidates[p]);
      const int64_t lc = static_cast<int64_t>(cand.size());
      int64_t lr = INT64_MAX;
      NgramCounts refmax;
      for (const auto& r : references[p]) {
        const auto ref = in.map(r);
        lr = std::min<int64_t>(lr, static_cast<int64_t>(ref.size()));
        for (const auto& kv : ngrams(ref, n_gram)) {
          auto& slot = refmax[kv.first];
          slot = std::max(slot, kv.second);
        }
      }
      if (lr == INT64_MAX) lr = 0;
      input_len += lc;
      target_len += lr;
      for (const auto& kv : ngrams(cand, n_gram)) {
        auto it = refmax.find(kv.first);
        if (it != refmax.end()) {
          matches[kv.first.size() - 1] += static_cast<double>(std::min(kv.second, it->second));
        }
      }
      for (int i = 0; i < n_gram; ++i)
        if (lc - i > 0) possible[i] += static_cast<double>(lc - i);
    }
  }
  return {input_len, target_len, matches, possible};
}


}  // namespace tea_text
