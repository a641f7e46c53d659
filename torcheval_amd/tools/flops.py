"""FLOP counting by op interception (parity: tools/flops.py:30-335).

``FlopTensorDispatchMode(module)`` is a ``TorchDispatchMode``: every ATen op the module runs
(forward and backward, any device) passes through ``__torch_dispatch__``; ops with a formula
in ``flop_mapping`` add their count to every enclosing module scope.  Counts are
multiply-accumulates, as in the reference (Linear(10, 70) on one row = 700).

Module scopes are tracked differently from the reference: the scope stack is *derived from
the module's dotted name* (``"layer1.0.conv1"`` -> ``["", "layer1", "layer1.0",
"layer1.0.conv1"]``) instead of push/pop pairs, and backward scopes are switched by tensor
gradient hooks on module outputs (entering a module's backward) and inputs (leaving it) rather
than by identity autograd Functions that clone every activation.  A hook that never fires
(e.g. the first layer's input does not require grad) therefore cannot leave the stack
unbalanced, and no activation is copied.
"""

import logging
from collections import defaultdict
from functools import reduce
from operator import mul
from typing import Any, Callable, DefaultDict, Dict, List, Sequence, Tuple

import torch
from torch.utils._python_dispatch import TorchDispatchMode
from torch.utils._pytree import tree_flatten

aten = torch.ops.aten

__all__ = ["FlopTensorDispatchMode", "flop_mapping", "register_flop_formula"]


def _prod(xs: Sequence[int]) -> int:
    return reduce(mul, xs, 1)


def _mm_flops(inputs: Tuple[Any, ...], outputs: Tuple[Any, ...]) -> int:
    a, b = inputs[0], inputs[1]
    assert a.shape[-1] == b.shape[-2], (a.shape, b.shape)
    return a.numel() * b.shape[-1]


def _addmm_flops(inputs: Tuple[Any, ...], outputs: Tuple[Any, ...]) -> int:
    m1, m2 = inputs[1], inputs[2]
    assert m1.dim() == 2 and m2.dim() == 2, (m1.shape, m2.shape)
    return m1.shape[0] * m1.shape[1] * m2.shape[1]


def _bmm_flops(inputs: Tuple[Any, ...], outputs: Tuple[Any, ...]) -> int:
    assert len(inputs) == 2, len(inputs)
    n, c, t = inputs[0].shape
    return n * c * t * inputs[1].shape[-1]


def _conv_macs(batch: int, w_shape: Sequence[int], spatial: Sequence[int]) -> int:
    # one MAC per (sample, weight element, output position); bias/additions not counted
    return batch * _prod(w_shape) * _prod(spatial)


def _conv_flops(inputs: Tuple[Any, ...], outputs: Tuple[Any, ...]) -> int:
    x, w, transposed = inputs[0], inputs[1], bool(inputs[6])
    spatial = (x.shape if transposed else outputs[0].shape)[2:]
    return _conv_macs(x.shape[0], w.shape, spatial)


def _conv_backward_flops(inputs: Tuple[Any, ...], outputs: Tuple[Any, ...]) -> int:
    """dgrad and wgrad each cost exactly the forward convolution's MACs
    (N * |w| * output positions; input positions for a transposed conv).  For ordinary
    convolutions this equals the reference's per-gradient formulas; for transposed ones the
    reference's wgrad formula multiplies by the wrong spatial extent and is not reproduced."""
    grad_out, x, w = inputs[0], inputs[1], inputs[2]
    transposed, mask = bool(inputs[7]), inputs[-1]
    fwd = _conv_macs(x.shape[0], w.shape, (x.shape if transposed else grad_out.shape)[2:])
    return fwd * (int(bool(mask[0])) + int(bool(mask[1])))


flop_mapping: Dict[Any, Callable[[Tuple[Any, ...], Tuple[Any, ...]], int]] = {}


def register_flop_formula(ops: Sequence[Any], fn: Callable[[Tuple[Any, ...], Tuple[Any, ...]], int]) -> None:
    """Register ``fn(args, outputs) -> MACs`` for ATen op packets and their ``.default``."""
    for op in ops:
        flop_mapping[op] = fn
        default = getattr(op, "default", None)
        if default is not None:
            flop_mapping[default] = fn


register_flop_formula([aten.mm, aten.matmul], _mm_flops)
register_flop_formula([aten.addmm], _addmm_flops)
register_flop_formula([aten.bmm], _bmm_flops)
register_flop_formula([aten.convolution, aten._convolution], _conv_flops)
register_flop_formula([aten.convolution_backward], _conv_backward_flops)


def _scope_of(name: str) -> List[str]:
    """``"a.b.c"`` -> ``["", "a", "a.b", "a.b.c"]``; ``""`` -> ``[""]``."""
    if not name:
        return [""]
    parts = name.split(".")
    return [""] + [".".join(parts[: i + 1]) for i in range(len(parts))]


def _parent(name: str) -> str:
    return name.rsplit(".", 1)[0] if "." in name else ""


class FlopTensorDispatchMode(TorchDispatchMode):
    """
    Context manager counting FLOPs (MACs) of ``module`` per submodule and per ATen op.

    ``flop_counts[module_name][op_name]`` accumulates across forward and backward until
    ``reset()``; the root module is ``""``.

    Example::

        with FlopTensorDispatchMode(model) as ftdm:
            out = model(x).mean()
            fwd = copy.deepcopy(ftdm.flop_counts)
            ftdm.reset()
            out.backward()
            bwd = copy.deepcopy(ftdm.flop_counts)
    """

    def __init__(self, module: torch.nn.Module) -> None:
        super().__init__()
        self._all_hooks: List[torch.utils.hooks.RemovableHandle] = []
        self.flop_counts: DefaultDict[str, DefaultDict[str, int]] = defaultdict(lambda: defaultdict(int))
        self._parents: List[str] = [""]
        self._instrument(module, "")

    def __exit__(self, exc_type, exc_val, exc_tb):
        for h in self._all_hooks:
            h.remove()
        self._all_hooks.clear()
        return super().__exit__(exc_type, exc_val, exc_tb)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        fn = flop_mapping.get(func)
        if fn is None:
            logging.debug("%s is not yet supported in FLOPs calculation.", func)
            return out
        count = fn(args, out if isinstance(out, tuple) else (out,))
        key = func.__name__
        for scope in self._parents:
            self.flop_counts[scope][key] += count
        return out

    # ------------------------------------------------------------------ scoping
    def _set_scope(self, name: str) -> None:
        self._parents = _scope_of(name)

    def _tag(self, t: torch.Tensor, name: str, is_output: bool) -> None:
        """Attach one gradient hook per tensor; when its gradient is ready the scope switches
        to the module whose backward runs next.  A module *output* tag (the innermost
        producer - its post-hook runs first) wins over any *input* tag (consumer's parent)."""
        tags = t.__dict__.setdefault("_tea_flop_scope", {})
        cur = tags.get(id(self))
        if cur is None:
            tags[id(self)] = [name, is_output]
            t.register_hook(lambda _g, tags=tags, key=id(self): self._set_scope(tags[key][0]))
        elif is_output and not cur[1]:
            cur[0], cur[1] = name, True

    def _hook_tensors(self, obj: Any, name: str, is_output: bool) -> None:
        leaves, _ = tree_flatten(obj)
        for t in leaves:
            if isinstance(t, torch.Tensor) and t.requires_grad:
                self._tag(t, name, is_output)

    def _pre(self, name: str) -> Callable[..., None]:
        def f(_module: torch.nn.Module, inputs: Tuple[Any, ...]) -> None:
            self._set_scope(name)
            if torch.is_grad_enabled():
                # grad w.r.t. the module's inputs = its backward is done -> back to the parent
                self._hook_tensors(inputs, _parent(name), False)

        return f

    def _post(self, name: str) -> Callable[..., None]:
        def f(_module: torch.nn.Module, _inputs: Tuple[Any, ...], outputs: Any) -> None:
            self._set_scope(_parent(name))
            if torch.is_grad_enabled():
                # grad w.r.t. the module's outputs = its backward starts
                self._hook_tensors(outputs, name, True)

        return f

    def _instrument(self, mod: torch.nn.Module, prefix: str) -> None:
        for child_name, child in mod.named_children():
            name = f"{prefix}.{child_name}" if prefix else child_name
            self._all_hooks.append(child.register_forward_pre_hook(self._pre(name)))
            self._all_hooks.append(child.register_forward_hook(self._post(name)))
            self._instrument(child, name)

    def reset(self) -> None:
        """Clear all counts and return to the root scope."""
        self._parents = [""]
        self.flop_counts.clear()
