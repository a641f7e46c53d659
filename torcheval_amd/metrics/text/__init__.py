"""Text metrics, class API (parity: metrics/text/*.py).  All states are additive
(``merge="sum"``): one RCCL all-reduce syncs any collection of them."""

from typing import Iterable, List, Optional, Sequence, Union

import torch

from torcheval_amd.metrics.functional.text import (
    _bleu_score_compute,
    _bleu_score_update,
    _perplexity_compute,
    _perplexity_label_check,
    _perplexity_update,
    _wil_compute,
    _wil_update,
    _word_error_rate_compute,
    _word_error_rate_update,
    _word_information_preserved_compute,
    _word_information_preserved_update,
)
from torcheval_amd.metrics.metric import Metric

__all__ = ["BLEUScore", "Perplexity", "WordErrorRate", "WordInformationLost", "WordInformationPreserved"]
__doc_name__ = "Text Metrics"


class _SumStates(Metric[torch.Tensor]):
    _names: tuple = ()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["_SumStates"]):
        for metric in metrics:
            for n in self._names:
                getattr(self, n).add_(getattr(metric, n).to(self.device))
        return self


class BLEUScore(_SumStates):
    """Corpus BLEU with up to 4-gram precision (native C++ n-gram counting)."""

    _names = ("input_len", "target_len", "matches_by_order", "possible_matches_by_order")

    def __init__(self, *, n_gram: int, weights: Optional[torch.Tensor] = None, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        if n_gram not in [1, 2, 3, 4]:
            raise ValueError(f"n_gram should be 1, 2, 3, or 4, got {n_gram}.")
        if weights is not None and n_gram != len(weights):
            raise ValueError(
                f"the length of weights should equal n_gram, got len(weights)={len(weights)}, n_gram={n_gram}"
            )
        self.weights = weights
        self.n_gram = n_gram
        f64 = torch.float64
        self._add_state("input_len", torch.tensor(0.0, dtype=f64, device=self.device), merge="sum")
        self._add_state("target_len", torch.tensor(0.0, dtype=f64, device=self.device), merge="sum")
        self._add_state("matches_by_order", torch.zeros(n_gram, dtype=f64, device=self.device), merge="sum")
        self._add_state("possible_matches_by_order", torch.zeros(n_gram, dtype=f64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: Union[str, Sequence[str]], target: Sequence[Union[str, Sequence[str]]]) -> "BLEUScore":
        il, tl, m, p = _bleu_score_update(input, target, self.n_gram, self.device)
        self.input_len += il
        self.target_len += tl
        self.matches_by_order += m
        self.possible_matches_by_order += p
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        if torch.sum(self.matches_by_order) == 0:
            return torch.tensor(0.0, dtype=torch.float64, device=self.device)
        return _bleu_score_compute(
            self.input_len, self.target_len, self.matches_by_order, self.possible_matches_by_order,
            self.n_gram, self.weights,
        )


class Perplexity(_SumStates):
    """Perplexity of token logits (fused K7 kernel on ROCm; label check deferred to compute)."""

    _names = ("sum_log_probs", "num_total")

    def __init__(self, ignore_index: Optional[int] = None, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self.ignore_index = ignore_index
        self._err: Optional[torch.Tensor] = None
        self._add_state("sum_log_probs", torch.tensor(0.0, dtype=torch.float64, device=self.device), merge="sum")
        self._add_state("num_total", torch.tensor(0.0, dtype=torch.float64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: torch.Tensor, target: torch.Tensor) -> "Perplexity":
        if input.is_cuda and self._err is None:
            self._err = torch.zeros(1, dtype=torch.int32, device=input.device)
        s, n = _perplexity_update(input, target, self.ignore_index, err=self._err if input.is_cuda else None)
        self.sum_log_probs += s
        self.num_total += n
        return self

    def _check_device_errors(self) -> None:
        if self._err is not None and int(self._err.item()) != 0:
            self._err.zero_()
            raise ValueError(
                "Class labels in `target` tensor cannot be larger than vocab_size minus one "
                "(detected on device in an earlier update())."
            )

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        self._check_device_errors()
        if self.num_total == 0.0:
            return torch.empty(0)
        return _perplexity_compute(self.sum_log_probs, self.num_total)


class WordErrorRate(_SumStates):
    """Word error rate (native C++ edit distance)."""

    _names = ("errors", "total")

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        self._add_state("errors", torch.tensor(0, dtype=torch.float, device=self.device), merge="sum")
        self._add_state("total", torch.tensor(0, dtype=torch.float, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: Union[str, List[str]], target: Union[str, List[str]]) -> "WordErrorRate":
        errors, total = _word_error_rate_update(input, target)
        self.errors += errors.to(self.device)
        self.total += total.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _word_error_rate_compute(self.errors, self.total)


class WordInformationLost(_SumStates):
    """Word information lost (native C++ edit distance)."""

    _names = ("correct_total", "target_total", "preds_total")

    def __init__(self, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        for n in self._names:
            self._add_state(n, torch.tensor(0.0, dtype=torch.float64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: Union[str, List[str]], target: Union[str, List[str]]) -> "WordInformationLost":
        c, t, p = _wil_update(input, target)
        self.correct_total += c.to(self.device)
        self.target_total += t.to(self.device)
        self.preds_total += p.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _wil_compute(self.correct_total, self.target_total, self.preds_total)


class WordInformationPreserved(_SumStates):
    """Word information preserved (native C++ edit distance)."""

    _names = ("correct_total", "input_total", "target_total")

    def __init__(self, *, device: Optional[torch.device] = None) -> None:
        super().__init__(device=device)
        for n in self._names:
            self._add_state(n, torch.tensor(0, dtype=torch.float64, device=self.device), merge="sum")

    @torch.inference_mode()
    def update(self, input: Union[str, List[str]], target: Union[str, List[str]]) -> "WordInformationPreserved":
        c, t, i = _word_information_preserved_update(input, target)
        self.correct_total += c.to(self.device)
        self.target_total += t.to(self.device)
        self.input_total += i.to(self.device)
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        return _word_information_preserved_compute(self.correct_total, self.target_total, self.input_total)
