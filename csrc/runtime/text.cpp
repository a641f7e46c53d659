// Host runtime for text metrics.
//
// Reference (pure Python, O(n*m) interpreter loop per pair):
//   functional/text/helper.py:12-64  _edit_distance / _get_errors_and_totals
//   functional/text/bleu.py:65-160   collections.Counter n-gram matching
// Here: tokens are interned to int ids per call, the Levenshtein DP runs on two int rows,
// n-grams are packed into 64-bit keys (4 x 16-bit ids; longer vocabularies fall back to a
// vector key) and counted in hash maps.  Results are bit-identical to the reference.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <array>
#include <cstdint>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "tea_runtime.h"
#include "tea_text_core.h"

namespace py = pybind11;

namespace {

using tea_text::Tokens;

std::tuple<double, double, double, double> errors_and_totals(const std::vector<Tokens>& inputs,
                                                             const std::vector<Tokens>& targets) {
  py::gil_scoped_release release;
  return tea_text::errors_and_totals(inputs, targets);
}

std::tuple<int64_t, int64_t, std::vector<double>, std::vector<double>> bleu_counts(
    const std::vector<Tokens>& candidates, const std::vector<std::vector<Tokens>>& references,
    int n_gram) {
  py::gil_scoped_release release;
  return tea_text::bleu_counts(candidates, references, n_gram);
}

}  // namespace

void tea_register_runtime(py::module_& m) {
  m.def("text_errors_and_totals", &errors_and_totals,
        "word-level Levenshtein errors + totals over sentence pairs (pre-tokenized)");
  m.def("bleu_counts", &bleu_counts, "BLEU n-gram match statistics (pre-tokenized)");
}
