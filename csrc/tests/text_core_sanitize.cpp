// Host sanitizer driver for the C++ text runtime: built with
// -fsanitize=address,undefined by tests/test_sanitizers.py and run on randomized inputs.
// Checks the O(n*m) two-row Levenshtein against a full-matrix DP, and BLEU count invariants.
#include <cstdio>
#include <cstdlib>
#include <random>

#include "tea_text_core.h"

namespace {

int64_t full_dp(const std::vector<int>& a, const std::vector<int>& b) {
  std::vector<std::vector<int64_t>> d(a.size() + 1, std::vector<int64_t>(b.size() + 1, 0));
  for (size_t i = 0; i <= a.size(); ++i) d[i][0] = static_cast<int64_t>(i);
  for (size_t j = 0; j <= b.size(); ++j) d[0][j] = static_cast<int64_t>(j);
  for (size_t i = 1; i <= a.size(); ++i)
    for (size_t j = 1; j <= b.size(); ++j)
      d[i][j] = std::min({d[i - 1][j] + 1, d[i][j - 1] + 1, d[i - 1][j - 1] + (a[i - 1] != b[j - 1])});
  return d[a.size()][b.size()];
}

tea_text::Tokens random_sentence(std::mt19937& rng, int max_len, int vocab) {
  std::uniform_int_distribution<int> len(0, max_len), word(0, vocab - 1);
  tea_text::Tokens t(len(rng));
  for (auto& w : t) w = "w" + std::to_string(word(rng));
  return t;
}

}  // namespace

int main() {
  std::mt19937 rng(1234);
  int failures = 0;
  for (int it = 0; it < 3000; ++it) {
    const auto a = random_sentence(rng, 24, 6), b = random_sentence(rng, 24, 6);
    tea_text::Interner in;
    const auto ia = in.map(a), ib = in.map(b);
    if (tea_text::levenshtein(ia, ib) != full_dp(ia, ib)) ++failures;
  }
  for (int it = 0; it < 300; ++it) {
    std::vector<tea_text::Tokens> cands;
    std::vector<std::vector<tea_text::Tokens>> refs;
    for (int p = 0; p < 4; ++p) {
      cands.push_back(random_sentence(rng, 12, 5));
      refs.push_back({random_sentence(rng, 12, 5), random_sentence(rng, 12, 5)});
    }
    const int n_gram = 1 + it % 4;
    const auto res = tea_text::bleu_counts(cands, refs, n_gram);
    const auto& matches = std::get<2>(res);
    const auto& possible = std::get<3>(res);
    for (int i = 0; i < n_gram; ++i)
      if (matches[i] < 0 || matches[i] > possible[i]) ++failures;
    const auto et = tea_text::errors_and_totals(cands, std::vector<tea_text::Tokens>(cands.rbegin(), cands.rend()));
    if (std::get<0>(et) > std::get<1>(et)) ++failures;  // edit distance <= max length
  }
  std::printf("text_core_sanitize: %s (%d failures)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
