"""Word information lost, functional API (parity: functional/text/word_information_lost.py)."""

from typing import List, Tuple, Union

import torch

from torcheval_amd.metrics.functional.text.helper import _get_errors_and_totals

__all__ = ["word_information_lost"]


def _wil_update(
    input: Union[str, List[str]], target: Union[str, List[str]]
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if isinstance(input, str):
        input = [input]
    if isinstance(target, str):
        target = [target]
    assert len(input) == len(target), (
        "Arguments must contain the same number of strings, "
        f"but got len(input)={len(input)} and len(target)={len(target)}"
    )
    errors, max_total, target_total, input_total = _get_errors_and_totals(input, target)
    # (errors - max_total) is the NEGATED number of hits; the square in compute hides the sign
    return errors - max_total, target_total, input_total


def _wil_compute(correct_total: torch.Tensor, target_total: torch.Tensor, preds_total: torch.Tensor) -> torch.Tensor:
    return 1 - correct_total / target_total * (correct_total / preds_total)


@torch.inference_mode()
def word_information_lost(input: Union[str, List[str]], target: Union[str, List[str]]) -> torch.Tensor:
    """Word information lost.  Class: ``WordInformationLost``."""
    return _wil_compute(*_wil_update(input, target))
