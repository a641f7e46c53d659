"""Device helpers (owned replacement of torchtnt.utils.copy_data_to_device)."""

import dataclasses
from collections import defaultdict
from typing import Any

import torch


def copy_data_to_device(data: Any, device: torch.device, *args: Any, **kwargs: Any) -> Any:
    """Recursively move every tensor inside ``data`` (lists, tuples, dicts, dataclasses) to
    ``device``.  Metrics are moved with ``Metric.to``."""
    from torcheval_amd.metrics.metric import Metric

    if isinstance(data, torch.Tensor):
        return data.to(device, *args, **kwargs)
    if isinstance(data, Metric):
        return data.to(device)
    if isinstance(data, defaultdict):
        return type(data)(
            data.default_factory,
            {k: copy_data_to_device(v, device, *args, **kwargs) for k, v in data.items()},
        )
    if isinstance(data, dict):
        return type(data)({k: copy_data_to_device(v, device, *args, **kwargs) for k, v in data.items()})
    if isinstance(data, tuple) and hasattr(data, "_fields"):  # namedtuple
        return type(data)(*(copy_data_to_device(v, device, *args, **kwargs) for v in data))
    if isinstance(data, (list, tuple)):
        return type(data)(copy_data_to_device(v, device, *args, **kwargs) for v in data)
    if dataclasses.is_dataclass(data) and not isinstance(data, type):
        values = {
            f.name: copy_data_to_device(getattr(data, f.name), device, *args, **kwargs)
            for f in dataclasses.fields(data)
            if f.init
        }
        new = type(data)(**values)
        for f in dataclasses.fields(data):
            if not f.init:
                setattr(new, f.name, getattr(data, f.name))
        return new
    return data
