"""Module summaries: parameters, bytes, FLOPs, activation shapes, forward time
(parity: tools/module_summary.py:63-759).

Differences from the reference, by design:
* forward time is measured with HIP events on GPU modules (host timers only measure launch
  latency there) and reported in real milliseconds (the reference divides seconds by 1000);
* the tree is built in one pass over ``named_modules`` bookkeeping instead of recursive
  re-traversal per summary;
* no dependency on torchtnt.
"""

import copy
import math
import time
import warnings
from collections import defaultdict
from typing import Any, Dict, List, MutableMapping, Optional, Tuple, Union

import torch
from torch.nn.parameter import UninitializedParameter
from torch.utils._pytree import tree_flatten

__all__ = ["ModuleSummary", "get_module_summary", "get_summary_table", "prune_module_summary"]

_UNKNOWN = "?"

_COLUMNS = {
    "module_name": "Name",
    "module_type": "Type",
    "num_parameters": "# Parameters",
    "num_trainable_parameters": "# Trainable Parameters",
    "size_bytes": "Size (bytes)",
    "has_uninitialized_param": "Contains Uninitialized Parameters?",
    "flops_forward": "Forward FLOPs",
    "flops_backward": "Backward FLOPs",
    "in_size": "In size",
    "out_size": "Out size",
    "forward_elapsed_time_ms": "Forward Elapsed Times (ms)",
}
_OPTIONAL = ("flops_forward", "flops_backward", "in_size", "out_size", "forward_elapsed_time_ms")
_FLOP_COLS = ("flops_forward", "flops_backward")
_NUM_UNITS = [" ", "K", "M", "B", "T"]
_FLOP_UNITS = [" ", "k", "M", "G", "T", "P", "E", "Z", "Y"]


def _warn_uninit(what: str) -> None:
    warnings.warn(
        "A layer with UninitializedParameter was found. "
        f"Thus, the total {what} detected may be inaccurate."
    )


class ModuleSummary:
    """Summary of a module and (recursively) its submodules.  ``"?"`` marks values that were
    not measured (no example inputs given)."""

    def __init__(self) -> None:
        self._module_name = ""
        self._module_type = ""
        self._num_parameters = 0
        self._num_trainable_parameters = 0
        self._size_bytes = 0
        self._submodule_summaries: Dict[str, "ModuleSummary"] = {}
        self._has_uninitialized_param = False
        self._flops_forward: Union[str, int] = _UNKNOWN
        self._flops_backward: Union[str, int] = _UNKNOWN
        self._flops_forward_detail: Dict[str, int] = {}
        self._flops_backward_detail: Dict[str, int] = {}
        self._in_size: Union[str, List[Any]] = _UNKNOWN
        self._out_size: Union[str, List[Any]] = _UNKNOWN
        self._forward_time_elapsed_ms: Union[str, float] = _UNKNOWN

    @property
    def submodule_summaries(self) -> Dict[str, "ModuleSummary"]:
        return self._submodule_summaries

    @property
    def module_name(self) -> str:
        return self._module_name

    @property
    def module_type(self) -> str:
        return self._module_type

    @property
    def num_parameters(self) -> int:
        if self._has_uninitialized_param:
            _warn_uninit("number of parameters")
        return self._num_parameters

    @property
    def num_trainable_parameters(self) -> int:
        if self._has_uninitialized_param:
            _warn_uninit("number of parameters")
        return self._num_trainable_parameters

    @property
    def flops_forward(self) -> Union[int, str]:
        if self._has_uninitialized_param:
            _warn_uninit("number of FLOPs")
        return self._flops_forward

    @property
    def flops_backward(self) -> Union[int, str]:
        if self._has_uninitialized_param:
            _warn_uninit("number of FLOPs")
        return self._flops_backward

    @property
    def in_size(self) -> Union[str, List[Any]]:
        return self._in_size

    @property
    def out_size(self) -> Union[str, List[Any]]:
        return self._out_size

    @property
    def forward_elapsed_time_ms(self) -> Union[str, float]:
        return self._forward_time_elapsed_ms

    @property
    def size_bytes(self) -> int:
        if self._has_uninitialized_param:
            _warn_uninit("byte sizes")
        return self._size_bytes

    @property
    def has_uninitialized_param(self) -> bool:
        return self._has_uninitialized_param

    def __repr__(self) -> str:
        return str(self)

    def __str__(self) -> str:
        return get_summary_table(self)


# ----------------------------------------------------------------------------- profiling run
class _Probe:
    """Forward hooks recording activation shapes and per-module forward time."""

    def __init__(self, module: torch.nn.Module) -> None:
        self.shapes: Dict[str, Tuple[Any, Any]] = {}
        self.starts: Dict[str, Any] = {}
        self.times_ms: Dict[str, List[Any]] = defaultdict(list)
        self.handles: List[Any] = []
        for name, mod in module.named_modules():
            if isinstance(mod, torch.jit.ScriptModule):
                warnings.warn("Registering hooks on torch.jit.ScriptModule is not supported.")
                continue
            self.handles.append(mod.register_forward_pre_hook(self._start(name, mod)))
            self.handles.append(mod.register_forward_hook(self._stop(name)))

    @staticmethod
    def _on_gpu(mod: torch.nn.Module) -> bool:
        for p in mod.parameters():
            return p.is_cuda
        for b in mod.buffers():
            return b.is_cuda
        return torch.cuda.is_available() and torch.cuda.is_initialized()

    def _start(self, name: str, mod: torch.nn.Module):
        def hook(_m, _inp) -> None:
            if self._on_gpu(mod):
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self.starts[name] = ev
            else:
                self.starts[name] = time.perf_counter()

        return hook

    def _stop(self, name: str):
        def hook(_m, inp, out) -> None:
            start = self.starts.pop(name, None)
            if isinstance(start, torch.cuda.Event):
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self.times_ms[name].append((start, ev))
            elif start is not None:
                self.times_ms[name].append((time.perf_counter() - start) * 1000.0)
            x = inp[0] if len(inp) == 1 else inp
            self.shapes[name] = (_shape_of(x), _shape_of(out))  # last call wins (reference)

        return hook

    def finish(self) -> Dict[str, float]:
        for h in self.handles:
            h.remove()
        if any(isinstance(e, tuple) for v in self.times_ms.values() for e in v):
            torch.cuda.synchronize()
        # a module called several times reports its total forward time
        return {
            k: float(sum(e[0].elapsed_time(e[1]) if isinstance(e, tuple) else e for e in v))
            for k, v in self.times_ms.items()
        }


def _shape_of(x: Any) -> Any:
    if hasattr(x, "shape"):
        return list(x.shape)
    if isinstance(x, (list, tuple)):
        return [_shape_of(e) for e in x]
    return _UNKNOWN


def _profile(module: torch.nn.Module, args: Tuple[Any, ...], kwargs: MutableMapping[str, Any]):
    from torcheval_amd.tools.flops import FlopTensorDispatchMode

    probe = _Probe(module)
    module.zero_grad()
    fwd = bwd = None
    try:
        with FlopTensorDispatchMode(module) as ftdm:
            res = module(*args, **kwargs)
            times = probe.finish()
            fwd = copy.deepcopy(ftdm.flop_counts)
            if isinstance(res, torch.Tensor):
                ftdm.reset()
                if res.requires_grad:
                    res.mean().backward()
                bwd = copy.deepcopy(ftdm.flop_counts)
            else:
                warnings.warn("Backward FLOPs are only computed if module foward returns a tensor.")
    finally:
        for h in probe.handles:
            h.remove()
    module.zero_grad()
    return fwd, bwd, probe.shapes, times


def _has_tensor(obj: Any) -> bool:
    leaves, _ = tree_flatten(obj)
    return any(isinstance(e, torch.Tensor) for e in leaves)


def get_module_summary(
    module: torch.nn.Module,
    module_args: Optional[Tuple[Any, ...]] = None,
    module_kwargs: Optional[MutableMapping[str, Any]] = None,
) -> ModuleSummary:
    """Summarise ``module``; with example ``module_args`` also FLOPs (forward of the call,
    backward of ``out.mean()``), activation shapes and forward time.  Lazy (uninitialised)
    modules are summarised without running them."""
    fwd = bwd = None
    shapes: Dict[str, Tuple[Any, Any]] = {}
    times: Dict[str, float] = {}
    uninit = any(isinstance(p, UninitializedParameter) for p in module.parameters())
    if not uninit:
        in_args, in_kwargs = _has_tensor(module_args), _has_tensor(module_kwargs)
        if in_kwargs:
            warnings.warn(
                "A tensor in module_kwargs was found. This may lead to an inaccurately computed "
                "activation size, as keyword arguments are not passed into forward hooks for modules. "
                "For best results, please input tensors though module_args."
            )
        if in_args or in_kwargs:
            fwd, bwd, shapes, times = _profile(module, tuple(module_args or ()), dict(module_kwargs or {}))
    return _build(module, "", fwd, bwd, shapes, times)


def _build(module, name, fwd, bwd, shapes, times) -> ModuleSummary:
    s = ModuleSummary()
    s._module_name = name
    s._module_type = type(module).__name__
    for child_name, child in module.named_children():
        full = f"{name}.{child_name}" if name else child_name
        sub = _build(child, full, fwd, bwd, shapes, times)
        s._submodule_summaries[full] = sub
        s._has_uninitialized_param |= sub._has_uninitialized_param
        s._num_parameters += sub._num_parameters
        s._num_trainable_parameters += sub._num_trainable_parameters
        s._size_bytes += sub._size_bytes
    for p in module.parameters(recurse=False):
        if isinstance(p, UninitializedParameter):
            s._has_uninitialized_param = True
            continue
        s._num_parameters += p.numel()
        s._size_bytes += p.numel() * p.element_size()
        if p.requires_grad:
            s._num_trainable_parameters += p.numel()
    for b in module.buffers(recurse=False):
        s._size_bytes += b.numel() * b.element_size()
    if fwd is not None:
        s._flops_forward_detail = dict(fwd.get(name, {}))
        s._flops_forward = sum(s._flops_forward_detail.values())
    if bwd is not None:
        s._flops_backward_detail = dict(bwd.get(name, {}))
        s._flops_backward = sum(s._flops_backward_detail.values())
    if name in shapes:
        s._in_size, s._out_size = shapes[name]
    if name in times:
        s._forward_time_elapsed_ms = times[name]
    return s


# ----------------------------------------------------------------------------- rendering
def _get_human_readable_count(number: int, labels: Optional[List[str]] = None) -> str:
    """123 -> '123  ', 1234 -> '1.2 K', 2e6 -> '2.0 M', 5e15 -> '5,000 T' (last unit caps)."""
    if not isinstance(number, int):
        raise TypeError(f"Input type must be int, but received {type(number)}")
    if number < 0:
        raise ValueError(f"Input value must be greater than 0, received {number}")
    labels = labels or _NUM_UNITS
    if len(labels) <= 0:
        raise ValueError(f"Input labels must be a list with at least one string, received {labels}")
    digits = int(math.floor(math.log10(number)) + 1) if number > 0 else 1
    groups = min(int(math.ceil(digits / 3)), len(labels))
    scaled = number * 10 ** (-3 * (groups - 1))
    idx = groups - 1
    if idx < 1 or scaled >= 100:
        return f"{int(scaled):,d} {labels[idx]}"
    return f"{scaled:,.1f} {labels[idx]}"


def _cell(attr: str, value: Any, human: bool) -> str:
    if isinstance(value, bool):
        return "Yes" if value else "No"
    if isinstance(value, int):
        if attr in _FLOP_COLS:
            if value < 0:
                return ""
            return _get_human_readable_count(value, labels=_FLOP_UNITS) if human else str(value)
        return _get_human_readable_count(value) if human else str(value)
    if isinstance(value, float):
        return f"{value:.10f}"
    if isinstance(value, list):
        return str(value)
    if value is None:
        return ""
    return str(value)


def _rows(summary: ModuleSummary, cols: List[str], human: bool, out: List[List[str]]) -> None:
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        out.append([_cell(c, getattr(summary, c), human) for c in cols])
    for sub in summary.submodule_summaries.values():
        _rows(sub, cols, human, out)


def get_summary_table(module_summary: ModuleSummary, human_readable_nums: bool = True) -> str:
    """Render ``module_summary`` (and its submodules, depth-first) as a text table; columns
    that were not measured on the root are dropped."""
    cols = [c for c in _COLUMNS if not (c in _OPTIONAL and getattr(module_summary, c) == _UNKNOWN)]
    rows: List[List[str]] = []
    _rows(module_summary, cols, human_readable_nums, rows)
    widths = [max([len(_COLUMNS[c])] + [len(r[i]) for r in rows]) for i, c in enumerate(cols)]
    fmt = lambda vals: " | ".join(f"{v:{w}}" for v, w in zip(vals, widths))  # noqa: E731
    lines = [fmt([_COLUMNS[c] for c in cols]), "-" * (sum(widths) + 3 * (len(cols) - 1))]
    lines += [fmt(r) for r in rows]
    table = "\n".join(lines) + "\n"
    if "flops_forward" in cols or "flops_backward" in cols:
        from torcheval_amd.tools.flops import flop_mapping

        ops = "|".join(
            f"`{op.__name__}`" for op in flop_mapping if not op.__name__.endswith(".default")
        )
        table += (
            f"Remark for FLOPs calculation: (1) Only operators {ops} are included. "
            "To add more operators supported in FLOPs calculation, use "
            "torcheval_amd.tools.flops.register_flop_formula. "
            "(2) The calculation related to additional loss function is not included. "
            "For forward, we calculated FLOPs based on `loss = model(input_data).mean()`. "
            "For backward, we calculated FLOPs based on `loss.backward()`. \n"
        )
    return table


def prune_module_summary(module_summary: ModuleSummary, *, max_depth: int) -> None:
    """Drop submodule summaries deeper than ``max_depth`` (in place; root depth = 1)."""
    if max_depth < 1:
        raise ValueError(f"`max_depth` must be an int greater than 0. Got {max_depth}.")
    if max_depth == 1:
        module_summary._submodule_summaries = {}
        return
    for sub in module_summary._submodule_summaries.values():
        prune_module_summary(sub, max_depth=max_depth - 1)
