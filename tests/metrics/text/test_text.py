"""Text metrics: reference-pinned values + independent oracles
(parity: tests/metrics/text/*, functional/text/test_bleu.py)."""

import math

import pytest
import torch

from torcheval_amd.metrics import (
    BLEUScore,
    Perplexity,
    WordErrorRate,
    WordInformationLost,
    WordInformationPreserved,
)
from torcheval_amd.metrics.functional import (
    bleu_score,
    perplexity,
    word_error_rate,
    word_information_lost,
    word_information_preserved,
)
from torcheval_amd.utils.test_utils import MetricClassTester

F64 = torch.float64


def _lev(a, b) -> int:
    d = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        prev, d[0] = d[0], i
        for j, y in enumerate(b, 1):
            prev, d[j] = d[j], min(d[j] + 1, d[j - 1] + 1, prev + (x != y))
    return d[len(b)]


def _wer_oracle(inp, tgt):
    e = sum(_lev(i.split(), t.split()) for i, t in zip(inp, tgt))
    return e / sum(len(t.split()) for t in tgt)


def _wip_oracle(inp, tgt):
    e = sum(_lev(i.split(), t.split()) for i, t in zip(inp, tgt))
    ti, tt = sum(len(i.split()) for i in inp), sum(len(t.split()) for t in tgt)
    mx = sum(max(len(i.split()), len(t.split())) for i, t in zip(inp, tgt))
    hits = mx - e
    return (hits / tt) * (hits / ti)


PRED = [["hello world", "welcome to the facebook"]] * 4
REF = [["hello metaverse", "welcome to meta"]] * 4


class TestWordMetrics(MetricClassTester):
    def test_wer_class(self) -> None:
        self.run_class_implementation_tests(
            metric=WordErrorRate(), state_names={"errors", "total"},
            update_kwargs={"input": PRED, "target": REF}, compute_result=torch.tensor(0.6), num_total_updates=4,
        )

    def test_wil_wip_class(self) -> None:
        self.run_class_implementation_tests(
            metric=WordInformationLost(), state_names={"correct_total", "target_total", "preds_total"},
            update_kwargs={"input": PRED, "target": REF}, compute_result=torch.tensor(0.7, dtype=F64),
            num_total_updates=4,
        )
        self.run_class_implementation_tests(
            metric=WordInformationPreserved(), state_names={"correct_total", "input_total", "target_total"},
            update_kwargs={"input": PRED, "target": REF}, compute_result=torch.tensor(0.3, dtype=F64),
            num_total_updates=4,
        )

    def test_functional_vs_oracle(self) -> None:
        import random

        rnd = random.Random(0)
        vocab = "a b c d e f g".split()
        inp = [" ".join(rnd.choice(vocab) for _ in range(rnd.randint(1, 9))) for _ in range(40)]
        tgt = [" ".join(rnd.choice(vocab) for _ in range(rnd.randint(1, 9))) for _ in range(40)]
        assert float(word_error_rate(inp, tgt)) == pytest.approx(_wer_oracle(inp, tgt), rel=1e-6)
        assert float(word_information_preserved(inp, tgt)) == pytest.approx(_wip_oracle(inp, tgt), rel=1e-6)
        assert float(word_information_lost(inp, tgt)) == pytest.approx(1 - _wip_oracle(inp, tgt), rel=1e-6)
        assert float(word_error_rate("hello world", "hello world")) == 0.0

    def test_invalid(self) -> None:
        with pytest.raises(ValueError, match="same type"):
            word_error_rate(["hello metaverse", "welcome to meta"], "hello world")
        with pytest.raises(ValueError, match="same length"):
            word_error_rate(["hello metaverse", "welcome to meta"], ["welcome to meta"])


class TestBLEU(MetricClassTester):
    def test_single(self) -> None:
        m = BLEUScore(n_gram=4)
        m.update(["the squirrel is eating the nut"], [["a squirrel is eating a nut", "the squirrel is eating a tasty nut"]])
        assert m.compute().item() == pytest.approx(0.53728497, abs=1e-7)

    def test_multiple_updates(self) -> None:
        self.run_class_implementation_tests(
            metric=BLEUScore(n_gram=4),
            state_names={"input_len", "target_len", "matches_by_order", "possible_matches_by_order"},
            update_kwargs={
                "input": [["the squirrel is eating the nut"], ["the cat is on the mat"]],
                "target": [
                    [["a squirrel is eating a nut", "the squirrel is eating a tasty nut"]],
                    [["there is a cat on the mat", "a cat is on the mat"]],
                ],
            },
            compute_result=torch.tensor(0.65341892, dtype=F64),
            num_total_updates=2,
            num_processes=2,
        )

    def test_multiple_examples_per_update(self) -> None:
        self.run_class_implementation_tests(
            metric=BLEUScore(n_gram=4),
            state_names={"input_len", "target_len", "matches_by_order", "possible_matches_by_order"},
            update_kwargs={
                "input": [["the squirrel is eating the nut", "the cat is on the mat"], ["i like ice cream and apple pie"]],
                "target": [
                    [["a squirrel is eating a nut", "the squirrel is eating a tasty nut"],
                     ["there is a cat on the mat", "a cat is on the mat"]],
                    [["i like apple pie with ice cream on top", "i like ice cream with my apple pie",
                      "i enjoy my apple pie with ice cream"]],
                ],
            },
            compute_result=torch.tensor(0.56377503, dtype=F64),
            num_total_updates=2,
            num_processes=2,
        )

    def test_functional_and_invalid(self) -> None:
        v = bleu_score(["the cat is on the mat"], [["there is a cat on the mat", "a cat is on the mat"]], n_gram=2)
        # unigram 5/6 clipped matches, bigram 3/5 (the cat, is on, on the, the mat -> "cat is","is on","on the","the mat" = 4/5)
        assert 0.0 < float(v) <= 1.0
        with pytest.raises(ValueError, match="n_gram should be 1, 2, 3, or 4"):
            BLEUScore(n_gram=5)
        with pytest.raises(ValueError):
            BLEUScore(n_gram=4, weights=torch.tensor([0.3, 0.3, 0.4]))


_PPL_IN = torch.tensor(
    [
        [[[0.3659, 0.7025, 0.3104]], [[0.5555, 0.5435, 0.7654]]],
        [[[0.0097, 0.6577, 0.1947]], [[0.5342, 0.6234, 0.8764]]],
        [[[0.4343, 0.0001, 0.9231]], [[0.6544, 0.0343, 0.0432]]],
        [[[0.2222, 0.0432, 0.3543]], [[0.9433, 0.8687, 0.5324]]],
    ]
)
_PPL_T = torch.tensor([[[2], [1]], [[1], [0]], [[2], [0]], [[1], [1]]])


def _ppl_oracle(x: torch.Tensor, t: torch.Tensor, ignore=None) -> float:
    lp = torch.log_softmax(x.double(), -1).reshape(-1, x.shape[-1])
    tt = t.reshape(-1)
    keep = tt != ignore if ignore is not None else torch.ones_like(tt, dtype=torch.bool)
    nll = -lp[keep].gather(1, tt[keep, None]).sum()
    return math.exp(float(nll) / int(keep.sum()))


class TestPerplexity(MetricClassTester):
    def test_pinned(self) -> None:
        self.run_class_implementation_tests(
            metric=Perplexity(), state_names={"sum_log_probs", "num_total"},
            update_kwargs={"input": _PPL_IN, "target": _PPL_T},
            compute_result=torch.tensor(2.784602403641, dtype=F64), num_total_updates=4, num_processes=2,
        )
        self.run_class_implementation_tests(
            metric=Perplexity(ignore_index=2), state_names={"sum_log_probs", "num_total"},
            update_kwargs={"input": _PPL_IN, "target": _PPL_T},
            compute_result=torch.tensor(2.824995994568, dtype=F64), num_total_updates=4, num_processes=2,
        )

    def test_functional_vs_log_softmax(self) -> None:
        torch.manual_seed(0)
        x = torch.randn(4, 16, 100) * 3
        t = torch.randint(0, 100, (4, 16))
        assert float(perplexity(x, t)) == pytest.approx(_ppl_oracle(x, t), rel=1e-5)
        assert float(perplexity(x, t, ignore_index=7)) == pytest.approx(_ppl_oracle(x, t, 7), rel=1e-5)

    def test_invalid(self) -> None:
        with pytest.raises(ValueError, match="target should be a two-dimensional tensor"):
            perplexity(torch.rand(3, 2, 3), torch.tensor([1, 2]))
        with pytest.raises(ValueError, match="input should be a three-dimensional tensor"):
            perplexity(torch.rand(3, 2), torch.tensor([[1, 2], [0, 0]]))
        with pytest.raises(ValueError, match="cannot be larger than vocab_size minus one"):
            perplexity(torch.rand(3, 2, 3), torch.tensor([[4, 2], [1, 0], [0, 0]]))
        with pytest.raises(ValueError, match="cannot be larger than vocab_size minus one"):
            Perplexity().update(torch.rand(3, 2, 3), torch.tensor([[4, 2], [1, 0], [0, 0]]))
