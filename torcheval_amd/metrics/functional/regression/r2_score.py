"""R^2 score, functional API (parity: functional/regression/r2_score.py)."""

from typing import Tuple

import torch

from torcheval_amd.metrics.functional.regression._common import _native
from torcheval_amd.ops import compiling, native, native_loaded

__all__ = ["r2_score"]


@torch.inference_mode()
def r2_score(
    input: torch.Tensor,
    target: torch.Tensor,
    *,
    multioutput: str = "uniform_average",
    num_regressors: int = 0,
) -> torch.Tensor:
    """Coefficient of determination; ``multioutput`` in uniform_average | raw_values |
    variance_weighted; ``num_regressors`` > 0 gives adjusted R2.  Class: ``R2Score``."""
    _r2_score_param_check(multioutput, num_regressors)
    cpu_twin = _cpu_r2_ok(input, target)
    if _native(input, target) or cpu_twin:
        # the sample count is known on the host: the reference's checks need no device sync
        _r2_score_update_input_check(input, target)
        n = target.size(0)
        if n < 2:
            raise ValueError(
                "There is no enough data for computing. Needs at least two samples to calculate r2 score."
            )
        if num_regressors >= n - 1:
            raise ValueError(
                "The `num_regressors` must be smaller than n_samples - 1, "
                f"got num_regressors={num_regressors}, n_samples={torch.tensor(n)}."
            )
        if cpu_twin:  # small CPU batches: one C++ call instead of ~12 ATen dispatches
            return native().cpu_r2(input, target, _R2_MODES[multioutput], num_regressors)
        from torcheval_amd.ops.reductions import r2_fused

        return r2_fused(input, target, multioutput, num_regressors)
    stats = _r2_score_update(input, target)
    return _r2_score_compute(*stats, multioutput, num_regressors)


_R2_MODES = {"raw_values": 0, "uniform_average": 1, "variance_weighted": 2}


def _cpu_r2_ok(input: torch.Tensor, target: torch.Tensor) -> bool:
    return (
        input.device.type == "cpu"
        and target.device.type == "cpu"
        and input.dtype in (torch.float32, torch.float64)
        and target.dtype == input.dtype
        and input.shape == target.shape
        and input.dim() in (1, 2)
        and input.numel() <= (1 << 16)
        and not input.requires_grad
        and not compiling()
        and native_loaded()
    )


def _r2_score_update(
    input: torch.Tensor, target: torch.Tensor
) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]:
    _r2_score_update_input_check(input, target)
    if _native(input, target):
        from torcheval_amd.ops.reductions import column_moments

        d = input.shape[1] if input.ndim == 2 else 1
        buf = torch.zeros(3 * d + 1, dtype=torch.float32, device=input.device)
        column_moments(input, target, None, stt=buf[:d], st=buf[d : 2 * d], sse=buf[2 * d : 3 * d],
                       sw=buf[3 * d :])
        # the count is known on the host: a CPU int64 scalar as in the reference (r2_score.py:109)
        n = torch.tensor(target.size(0))
        if input.ndim == 2:
            return buf[:d], buf[d : 2 * d], buf[2 * d : 3 * d], n
        return buf[0], buf[1], buf[2], n
    return (
        torch.sum(torch.square(target), dim=0),
        torch.sum(target, dim=0),
        torch.sum(torch.square(target - input), dim=0),
        torch.tensor(target.size(0)),
    )


def _r2_score_compute(
    sum_squared_obs: torch.Tensor,
    sum_obs: torch.Tensor,
    rss: torch.Tensor,
    num_obs: torch.Tensor,
    multioutput: str,
    num_regressors: int,
) -> torch.Tensor:
    if num_obs < 2:
        raise ValueError(
            "There is no enough data for computing. Needs at least two samples to calculate r2 score."
        )
    if num_regressors >= num_obs - 1:
        raise ValueError(
            "The `num_regressors` must be smaller than n_samples - 1, "
            f"got num_regressors={num_regressors}, n_samples={num_obs}."
        )
    tss = sum_squared_obs - torch.square(sum_obs) / num_obs
    r_squared = 1 - rss / tss
    if multioutput == "uniform_average":
        r_squared = torch.mean(r_squared)
    elif multioutput == "variance_weighted":
        r_squared = torch.sum(r_squared * tss / torch.sum(tss))
    if num_regressors != 0:
        r_squared = 1 - (1 - r_squared) * (num_obs - 1) / (num_obs - num_regressors - 1)
    return r_squared


def _r2_score_param_check(multioutput: str, num_regressors: int) -> None:
    if multioutput not in ("raw_values", "uniform_average", "variance_weighted"):
        raise ValueError(
            "The `multioutput` must be either `raw_values` or `uniform_average` or `variance_weighted`, "
            f"got multioutput={multioutput}."
        )
    if not isinstance(num_regressors, int) or num_regressors < 0:
        raise ValueError(
            "The `num_regressors` must an integer larger or equal to zero, "
            f"got num_regressors={num_regressors}."
        )


def _r2_score_update_input_check(input: torch.Tensor, target: torch.Tensor) -> None:
    if input.ndim >= 3 or target.ndim >= 3:
        raise ValueError(
            "The dimension `input` and `target` should be 1D or 2D, "
            f"got shapes {input.shape} and {target.shape}."
        )
    if input.size() != target.size():
        raise ValueError(
            "The `input` and `target` should have the same size, "
            f"got shapes {input.shape} and {target.shape}."
        )
