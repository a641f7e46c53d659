"""Metric base class and state registry.

Behavioural parity with the reference ``Metric`` ABC (torcheval/metrics/metric.py:21-256):
``_add_state`` / ``update`` / ``compute`` / ``merge_state`` / ``_prepare_for_merge_state`` /
``reset`` / ``state_dict`` / ``load_state_dict`` / ``to`` / ``device``, the allowed state
types (``TState``, metric.py:18) and the exact error strings.

MI355X-first differences (documented decisions):

* every state carries a *merge kind* (``"sum" | "max" | "min" | "cat" | None``).  The
  distributed toolkit (``torcheval_amd.parallel.state_sync``) uses it to sync additive /
  extremal states with ONE bucketed RCCL ``all_reduce`` per (dtype, op) instead of the
  reference's pickled ``all_gather_object`` of whole metric objects.  States that declare
  nothing are still synced correctly: their tensors travel through a device-resident
  all-gather-v and the metric's own ``merge_state`` is called, exactly as in the reference.
* additive / extremal tensor states live as views into ONE contiguous device buffer per metric
  (``torcheval_amd.parallel.state_buffer``), so ``sync_and_compute`` sends
  one bucket and ``reset()`` is one copy.
* ``reset()`` also restores ``int`` / ``float`` states (the reference leaves them stale,
  metric.py:126-146).
* dict states use a picklable zero-tensor factory instead of a lambda, so every metric is
  picklable (the reference's lambda-defaultdict metrics are not).
"""

import functools
from abc import ABC, abstractmethod
from collections import defaultdict
from copy import deepcopy
from typing import Any, Callable, Dict, Generic, Iterable, List, Optional, TypeVar, Union

import torch

from torcheval_amd.config import config as _cfg

TSelf = TypeVar("TSelf", bound="Metric")
TComputeReturn = TypeVar("TComputeReturn")
TState = Union[torch.Tensor, List[torch.Tensor], Dict[Any, torch.Tensor], int, float]

__doc_name__ = "Metric Base"

MERGE_KINDS = ("sum", "max", "min", "cat", None)


class _ZeroTensor:
    """Picklable default factory for dict states (replaces the reference's lambda)."""

    __slots__ = ("device",)

    def __init__(self, device: torch.device) -> None:
        self.device = device

    def __call__(self) -> torch.Tensor:
        return torch.tensor(0.0, device=self.device)

    def __reduce__(self):
        return (_ZeroTensor, (self.device,))


def _as_device(device: Optional[Union[str, torch.device]]) -> torch.device:
    if device is None:
        return torch.device("cpu")
    return torch.device(device) if not isinstance(device, torch.device) else device


def _instrument(fn: Callable, label: str, check_after: bool) -> Callable:
    """Wrap a metric method: ``record_function`` range when tracing; after ``update`` in
    validate mode, raise any device-recorded input error immediately."""
    if getattr(fn, "__tea_instrumented__", False):
        return fn

    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        if _cfg.trace:
            with torch.profiler.record_function(f"{type(self).__name__}.{label}"):
                out = fn(self, *args, **kwargs)
        else:
            out = fn(self, *args, **kwargs)
        if check_after and _cfg.validate:
            with torch.inference_mode():  # error flags are created inside inference-mode updates
                self._check_device_errors()
        return out

    wrapper.__tea_instrumented__ = True  # type: ignore[attr-defined]
    return wrapper


def inference_update(fn: Callable) -> Callable:
    """``torch.inference_mode()`` for eager ``update()`` calls; a plain call while torch.compile
    traces (states never require grad, and inference-mode views inside a compiled region break
    inductor's storage bookkeeping)."""

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        # compiling first (dynamo cannot trace is_inference_mode_enabled); already inside (a
        # subclass update calling super().update): no second ~2 us context
        if torch.compiler.is_compiling() or torch.is_inference_mode_enabled():
            return fn(*args, **kwargs)
        with torch.inference_mode():
            return fn(*args, **kwargs)

    return wrapper


class Metric(Generic[TComputeReturn], ABC):
    """
    Base class for all metrics present in the Metrics API.

    Implement ``__init__()``, ``update()``, ``compute()`` and ``merge_state()`` to implement
    your own metric (reference: torcheval/metrics/metric.py:21-47).
    """

    def __init_subclass__(cls, **kwargs: Any) -> None:
        super().__init_subclass__(**kwargs)
        for label in ("update", "compute", "merge_state"):
            fn = cls.__dict__.get(label)
            if fn is not None and callable(fn):
                setattr(cls, label, _instrument(fn, label, check_after=label == "update"))

    # How a device error flag (``self._err``, when a metric has one) merges across ranks in the
    # distributed sync: "max" (elementwise; codes and largest offending labels) or "first"
    # (the lowest flagged rank's whole record, for multi-word records).
    _err_merge: str = "max"
    # Words of the device error flag, when every instance's flag has the same size: the sync
    # then sizes a receiving rank's flag without reading the gathered record on the host.
    _err_words: Optional[int] = None

    def _check_device_errors(self) -> None:
        """Raise input-validation errors that native kernels recorded on the device.

        Metrics whose GPU update validates inputs asynchronously (a device error flag instead
        of a host sync) override this; ``compute()`` calls it, and so does every ``update()``
        when ``torcheval_amd.config.validate`` is set."""

    def __init__(self: TSelf, *, device: Optional[torch.device] = None) -> None:
        torch._C._log_api_usage_once(f"torcheval_amd.metrics.{self.__class__.__name__}")
        self._state_name_to_default: Dict[str, TState] = {}
        self._state_merge_kind: Dict[str, Optional[str]] = {}
        self._device: torch.device = _as_device(device)
        # contiguous device buffer of the sum / max / min states (built lazily by the sync
        # engine, torcheval_amd.parallel.state_buffer); None until then
        self._tea_sb = None

    # ------------------------------------------------------------------ state registry
    def _add_state(
        self: TSelf, name: str, default: TState, *, merge: Optional[str] = None
    ) -> None:
        """
        Used in subclass ``__init__()`` to add a metric state variable.

        Args:
            name: The name of the state variable. The variable can be accessed with
                ``self.name``.
            default: Default value of the state. It should be a type of TState. The state
                will be reset to this value when ``self.reset()`` is called.
            merge: How the state combines across metric instances / ranks: ``"sum"``,
                ``"max"``, ``"min"`` (elementwise, shape fixed at construction), ``"cat"``
                (list of tensors concatenated) or ``None`` (custom ``merge_state``).
                Declared reductions let the distributed toolkit use RCCL all-reduce.
        Raises:
            TypeError: If ``default`` is not a type of TState.
        """
        _check_state_variable_type(name, default)
        if merge not in MERGE_KINDS:
            raise ValueError(f"merge kind must be one of {MERGE_KINDS}, got {merge}.")
        if isinstance(default, defaultdict):
            default = defaultdict(_ZeroTensor(self.device), default)
        setattr(self, name, deepcopy(default))
        self._state_name_to_default[name] = deepcopy(default)
        self._state_merge_kind[name] = merge

    # ------------------------------------------------------------------ abstract API
    @abstractmethod
    def update(self: TSelf, *_: Any, **__: Any) -> TSelf:
        """Update the state variables of the metric with a new batch."""

    @abstractmethod
    def compute(self: TSelf) -> TComputeReturn:
        """Compute and return the metric value from the state variables."""

    @abstractmethod
    def merge_state(self: TSelf, metrics: Iterable[TSelf]) -> TSelf:
        """
        Merge the states of ``metrics`` into this metric.  Input metrics stay unchanged.
        Used by the distributed toolkit for states that declare no merge kind.
        """

    def _prepare_for_merge_state(self: TSelf) -> None:
        """Hook called before syncing (e.g. collapse list states into one tensor)."""
        pass

    # ------------------------------------------------------------------ lifecycle
    def reset(self: TSelf) -> TSelf:
        """
        Reset the metric state variables to their default value.  Tensors in the default
        values are moved to the device of the last ``self.to(device)`` call.
        """
        sb = getattr(self, "_tea_sb", None)
        if sb is not None and sb.valid(self) and sb.device == self.device and sb.reset():
            return self  # one copy of the default image into the state buffer (views kept)
        device = self.device
        for state_name, default in self._state_name_to_default.items():
            if isinstance(default, torch.Tensor):
                setattr(self, state_name, default.clone().to(device))
            elif isinstance(default, list):
                setattr(self, state_name, [t.clone().to(device) for t in default])
            elif isinstance(default, dict):
                setattr(
                    self,
                    state_name,
                    defaultdict(
                        _ZeroTensor(device),
                        {k: t.clone().to(device) for k, t in default.items()},
                    ),
                )
            else:  # int / float: restored too (fixes reference metric.py:126-146)
                setattr(self, state_name, deepcopy(default))
        return self

    def state_dict(self: TSelf) -> Dict[str, TState]:
        """Save metric state variables in a state_dict (detached clones)."""
        state_dict: Dict[str, TState] = {}
        for state_name in self._state_name_to_default:
            value = getattr(self, state_name)
            _check_state_variable_type(state_name, value)
            if isinstance(value, torch.Tensor):
                state_dict[state_name] = value.detach().clone()
            elif isinstance(value, list):
                state_dict[state_name] = [t.detach().clone() for t in value]
            elif isinstance(value, dict):
                state_dict[state_name] = {k: t.detach().clone() for k, t in value.items()}
            else:
                state_dict[state_name] = value
        return state_dict

    def load_state_dict(self: TSelf, state_dict: Dict[str, Any], strict: bool = True) -> None:
        """
        Loads metric state variables from state_dict.

        Raises:
            RuntimeError: If ``strict`` is ``True`` and keys in state_dict does not match
                all names of the metric states.
            TypeError: If a value is not a type of TState.
        """
        state_dict = deepcopy(state_dict)
        metric_state_names = set(self._state_name_to_default.keys())
        for state_name in metric_state_names:
            if state_name in state_dict:
                value = state_dict[state_name]
                _check_state_variable_type(state_name, value)
                if isinstance(value, dict) and not isinstance(value, defaultdict):
                    if isinstance(self._state_name_to_default[state_name], defaultdict):
                        value = defaultdict(_ZeroTensor(self.device), value)
                setattr(self, state_name, value)
        if strict:
            state_dict_keys = set(state_dict.keys())
            unexpected_keys = state_dict_keys.difference(metric_state_names)
            missing_keys = metric_state_names.difference(state_dict_keys)
            if missing_keys or unexpected_keys:
                raise RuntimeError(
                    f"Error(s) in loading state_dict for {self.__class__.__name__}. "
                    f"Encountered missing keys: {missing_keys} and unexpected "
                    f"keys: {unexpected_keys}."
                )

    def to(self: TSelf, device: Union[str, torch.device], *args: Any, **kwargs: Any) -> TSelf:
        """Move tensors in metric state variables to ``device``."""
        device = torch.device(device) if isinstance(device, str) else device
        for state_name in self._state_name_to_default:
            value = getattr(self, state_name)
            _check_state_variable_type(state_name, value)
            if isinstance(value, torch.Tensor):
                setattr(self, state_name, value.to(device))
            elif isinstance(value, list):
                setattr(self, state_name, [t.to(device, *args, **kwargs) for t in value])
            elif isinstance(value, dict):
                setattr(
                    self,
                    state_name,
                    defaultdict(
                        _ZeroTensor(device),
                        {k: t.to(device, *args, **kwargs) for k, t in value.items()},
                    ),
                )
        self._device = device
        return self

    @property
    def device(self: TSelf) -> torch.device:
        """The last input device of ``Metric.to()`` (default ``cpu``)."""
        return self._device

    # ------------------------------------------------------------------ sync helpers
    def _state_merge_kinds(self) -> Dict[str, Optional[str]]:
        kinds = getattr(self, "_state_merge_kind", None)
        if kinds is None:  # user metric built without our __init__ bookkeeping
            return {n: None for n in self._state_name_to_default}
        return {n: kinds.get(n) for n in self._state_name_to_default}


def _check_state_variable_type(name: str, value: Any) -> None:
    """Check the type of a state variable value.  It should be a type of TState."""
    if (
        not isinstance(value, torch.Tensor)
        and not (isinstance(value, list) and all(isinstance(x, torch.Tensor) for x in value))
        and not (
            isinstance(value, dict) and all(isinstance(x, torch.Tensor) for x in value.values())
        )
        and not isinstance(value, int)
        and not isinstance(value, float)
    ):
        raise TypeError(
            "The value of state variable must be a ``torch.Tensor``, a list of ``torch.Tensor``, "
            f"a dictionary with ``torch.Tensor``, int, or float as values."
            f"Get {name}={value} instead."
        )
