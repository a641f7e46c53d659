"""Word information preserved, functional API (parity: functional/text/word_information_preserved.py)."""

from typing import List, Tuple, Union

import torch

from torcheval_amd.metrics.functional.text.helper import _get_errors_and_totals, _text_pair_check

__all__ = ["word_information_preserved"]


@torch.inference_mode()
def word_information_preserved(input: Union[str, List[str]], target: Union[str, List[str]]) -> torch.Tensor:
    """Word information preserved.  Class: ``WordInformationPreserved``."""
    return _word_information_preserved_compute(*_word_information_preserved_update(input, target))


def _word_information_preserved_update(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    _text_pair_check(input, target)
    errors, max_total, target_total, input_total = _get_errors_and_totals(input, target)
    return max_total - errors, target_total, input_total


def _word_information_preserved_compute(
    correct_total: torch.Tensor, target_total: torch.Tensor, input_total: torch.Tensor
) -> torch.Tensor:
    return correct_total / target_total * (correct_total / input_total)
