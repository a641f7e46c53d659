"""Deferred fold of device partial sums into metric states (K5 deferred mode).

A streaming reduction over many blocks needs a cross-block combine.  Done inside the update's
launch it sits on the launch's tail (a write-through hand-off + ticket + the last block's fold:
~3.5 us of a 15 us MeanSquaredError update at 8192 x 1000, profiles/k5_v2_ab_r5.jsonl); done as
a second launch it costs a kernel boundary.  Deferred mode does neither: each block ADDS its
FP64 partials to a slot it owns in a per-metric pending buffer, the update's launch ends with
its last load, and the states fold the slots in only when they are next READ (compute, sync,
state_dict, merge, copies) - the pattern of K1's pending micro-accuracy cells, generalised.

``pending_states(*names)`` turns the named states of a metric class into properties:

* get: fold first if updates are pending (one small launch), then return the tensor;
* set: fold first (other pending states keep their contributions), then store;
* ``reset()`` drops the pending sums, ``to()`` / pickling fold them and detach the buffer,
  ``_mark_updated()`` (HIP-graph replays, utils/graphs.py) marks them pending again.

The pending sums are FP64 across updates and round to the float32 states once per fold, so a
folded state is at least as accurate as the reference's per-update float32 ``+=``
(mean_squared_error.py:82-97, r2_score.py:97-106).
"""

from typing import Dict, NamedTuple, Optional, Tuple

import torch

from torcheval_amd.ops import compiling, native

PEND_SLOTS = 64  # csrc/include/tea_kernels.h kMomentsPendSlots
ROWSUMS_PEND_STATS = 9  # kRowPendStats: six sums, COUNT, target min / max
ROWSUMS_PEND_BLOCKS = 2048  # kRowPendBlocks
ROWSUMS_PEND_MIN = 32768  # rowsums.hip kSingle: shorter rows are one block, folded in-launch


class RowSumsSpec(NamedTuple):
    """The K5b outputs a deferred update accumulates: state names, packed codes, rows."""

    names: Tuple[str, ...]
    codes: Tuple[int, ...]
    rows: int


def _prop(name: str) -> property:
    key = "_pv_" + name

    def fget(self):
        d = self.__dict__
        if d.get("_pend_dirty"):
            self._fold_pending()
        return d[key]

    def fset(self, value) -> None:
        d = self.__dict__
        if d.get("_pend_dirty"):
            self._fold_pending()
        d[key] = value

    return property(fget, fset, doc=f"metric state ``{name}`` (folds pending device sums on read)")


def pending_states(*names: str):
    """Class decorator: ``names`` become deferred-fold states (see the module docstring)."""

    def deco(cls):
        cls._pend_states = tuple(names)
        for n in names:
            setattr(cls, n, _prop(n))
        return cls

    return deco


class PendingMixin:
    """Fold / drop / buffer management of the deferred states (with ``pending_states``)."""

    _pend_states: tuple = ()

    def _raw_state(self, name: str) -> torch.Tensor:
        """The state tensor without folding (for the update that adds to the pending sums, and
        for HIP-graph replays' state-pointer checks)."""
        t = self.__dict__.get("_pv_" + name)
        return getattr(self, name) if t is None else t

    def _pend_buffer(self, numel: int, device: torch.device, spec=None) -> torch.Tensor:
        """The pending buffer for an update that will add ``spec``'s sums (pending sums of a
        different spec are folded first)."""
        d = self.__dict__
        if d.get("_pend_dirty") and spec is not None and d.get("_pend_spec") != spec:
            self._fold_pending()
        buf: Optional[torch.Tensor] = d.get("_pend")
        if buf is None or buf.numel() < numel or buf.device != device or d.get("_pend_id") != id(self):
            if d.get("_pend_dirty"):
                self._fold_pending()
            buf = torch.zeros(numel, dtype=torch.float64, device=device)
            d["_pend"] = buf
            d["_pend_id"] = id(self)
            d["_pend_r"] = 0
        return buf

    def _pend_mark(self, slots: int, spec: Dict[str, str]) -> None:
        d = self.__dict__
        d["_pend_spec"] = spec
        d["_pend_r"] = max(d.get("_pend_r", 0), slots)
        d["_pend_dirty"] = True

    def _fold_pending(self) -> None:
        d = self.__dict__
        d["_pend_dirty"] = False  # first: the state reads below must not recurse
        spec = d.get("_pend_spec") or {}
        if isinstance(spec, RowSumsSpec):  # K5b: outputs and codes of the deferred updates
            native().row_sums_fold(d["_pend"], d.get("_pend_r", 0), [d["_pv_" + n] for n in spec.names],
                                   list(spec.codes), spec.rows)
        else:  # K5 column moments: {statistic: state name}
            st = {k: d["_pv_" + n] for k, n in spec.items()}
            native().column_moments_fold(d["_pend"], d.get("_pend_r", 0), st.get("sse"), st.get("st"),
                                         st.get("stt"), st.get("sx"), st.get("sw"))
        d["_pend_r"] = 0

    def _rowsums_deferred(self, x: torch.Tensor, w, w_scalar: float, spec: "RowSumsSpec", t=None) -> bool:
        """K5b deferred update of ``spec``'s states from a long ROCm batch (``spec.rows`` rows;
        one for Sum / Mean / PSNR, the tasks for CTR / WC), with an optional target operand:
        True when the launch ran (the states now have pending sums)."""
        if not x.is_cuda or x.numel() <= ROWSUMS_PEND_MIN * spec.rows or compiling():
            return False
        pend = self._pend_buffer(spec.rows * ROWSUMS_PEND_STATS * ROWSUMS_PEND_BLOCKS, x.device, spec)
        used = native().row_sums_pend(x, t, w, w_scalar, [self.__dict__["_pv_" + n] for n in spec.names],
                                      list(spec.codes), spec.rows, pend)
        if not used:
            return False
        self._pend_mark(used, spec)
        return True

    def _drop_pending(self) -> None:
        d = self.__dict__
        if d.get("_pend_dirty"):
            d["_pend"].zero_()
            d["_pend_dirty"] = False
            d["_pend_r"] = 0

    def _pend_capture(self):
        """Right after a HIP-graph capture of ``update``: what every replay adds to, as
        ``(buffer, spec, slots)`` (None when the captured update did not run deferred).  A replay
        launches the captured kernels only - no Python - so ``_mark_updated`` must restore the
        spec and slot count the fold needs (a fold resets ``_pend_r`` to 0)."""
        d = self.__dict__
        if not d.get("_pend_dirty") or d.get("_pend") is None:
            return None
        return (d["_pend"], d.get("_pend_spec"), d.get("_pend_r", 0))

    def _pend_prepare(self, captured) -> None:
        """Before a replay: the captured launches add ``captured``'s sums into ``captured``'s
        buffer, so pending sums of another spec (an eager update in between) are folded first,
        and a buffer replaced since the capture (``to()``, a larger eager batch) is refused."""
        if captured is None:
            return
        d = self.__dict__
        if d.get("_pend") is not captured[0]:
            raise RuntimeError(
                f"{type(self).__name__}: the deferred-sum buffer was replaced after graph capture "
                "(to() or a larger eager update); re-create the GraphedUpdate"
            )
        if d.get("_pend_dirty") and d.get("_pend_spec") != captured[1]:
            self._fold_pending()

    def _mark_updated(self, captured=None) -> None:
        """Called after a HIP-graph replay of ``update`` (torcheval_amd.utils.graphs) with the
        ``_pend_capture()`` of the captured update: its sums are pending again, over its slots."""
        d = self.__dict__
        if captured is not None:
            d["_pend_spec"] = captured[1]
            d["_pend_r"] = max(d.get("_pend_r", 0), captured[2])
            d["_pend_dirty"] = True
        elif d.get("_pend") is not None and d.get("_pend_spec"):
            d["_pend_dirty"] = True

    def reset(self):
        self._drop_pending()  # the pending sums belong to the states being reset
        return super().reset()

    def to(self, device, *args, **kwargs):
        out = super().to(device, *args, **kwargs)  # reads (so folds) every state first
        self.__dict__["_pend"] = None
        return out

    def __getstate__(self):
        # copies (copy / deepcopy / pickle) carry folded states and no pending buffer
        d = self.__dict__
        if d.get("_pend_dirty"):
            self._fold_pending()
        state = dict(d)
        state["_pend"] = None
        state["_pend_dirty"] = False
        state["_pend_r"] = 0
        return state

    def __setstate__(self, state) -> None:
        self.__dict__.update(state)
