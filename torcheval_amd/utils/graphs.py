"""HIP-graph capture of metric ``update`` calls (EXPERIMENTAL: no measured case is faster than
direct calls yet - replay 11.2-17.8 us vs 5.5-12.6 us direct on every metric the GPU tests graph).

``GraphedUpdate`` records ``metric.update(*static_inputs)`` once into a HIP graph
(``torch.cuda.CUDAGraph`` on ROCm) and then replays it: per call, the new inputs are copied into
the static input buffers and the captured launches run as one graph launch.

Measured cost, not a free speed-up: on this runtime (ROCm 7 / MI355X) a graph launch costs
~27 us of wall time, while a direct one-kernel update (K1, K2, K5, K7 write straight into the
states) costs ~5 us (``profiles/bench_suite_r4b.json``: the "HIP-graph replay" rows, 27.3 vs
5.0 us at bs=8).  So a graph pays only for a step that chains many launches (a user's forward
plus several metric updates, or an ATen-path update of ~10 ops), never for a one-kernel update.
The constructor times both (``check_speed=True``) and warns when the replay is the slower one.

Requirements (checked): the update must write its states in place (the native kernels do;
an update that rebinds a state attribute, e.g. ``self.x = self.x + y``, would replay against
stale tensors and is rejected), must not synchronise with the host, and every replay must
use inputs of the captured shapes / dtypes.

The metric's contiguous state buffer (``parallel/state_buffer.py``) is built right before capture,
so a later ``sync_and_compute`` / ``reset`` finds it valid and never rebinds the states the
graph writes.  Anything else that rebinds a state after capture (``load_state_dict``,
``to()``) is caught at the next replay, which raises instead of writing into freed memory.

Several metrics fed the same inputs can share one graph (``GraphedUpdate([m1, m2, ...], x, y)``):
one replay then stands for all their update calls, which is where a graph pays - each direct
update costs its Python dispatch and launch, the replay one launch for the whole step.
"""

import time
import warnings
from typing import Any, Dict, List, Sequence, Tuple, Union

import torch

from torcheval_amd.metrics.metric import Metric

__all__ = ["GraphedUpdate"]


def _raw(metric: Metric, name: str) -> torch.Tensor:
    """A state tensor without folding pending device sums (the pointer check runs per replay;
    a fold per replay would add a launch and reset the slot count the replays add to)."""
    raw = getattr(metric, "_raw_state", None)
    return raw(name) if raw is not None else getattr(metric, name)


def _state_ptrs(metric: Metric) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for name in metric._state_name_to_default:
        v = _raw(metric, name)
        if isinstance(v, torch.Tensor):
            out[name] = v.data_ptr()
        elif isinstance(v, list):
            out[name] = ("list", len(v))
        else:
            out[name] = ("obj", v)
    return out


class GraphedUpdate:
    """Replayable HIP graph of ``metric.update(*example_args)`` - or of the updates of several
    metrics fed the same inputs.

    Example::

        acc = MulticlassAccuracy(device="cuda")
        step = GraphedUpdate(acc, logits_example, target_example)
        for logits, target in loader:
            step(logits, target)        # == acc.update(logits, target), one graph launch
        acc.compute()

        ms = [MulticlassAccuracy(device="cuda"), MulticlassPrecision(device="cuda"), ...]
        step = GraphedUpdate(ms, logits_example, target_example)   # one launch for all updates
    """

    def __init__(
        self,
        metric: Union[Metric, Sequence[Metric]],
        *example_args: torch.Tensor,
        warmup: int = 2,
        check_speed: bool = True,
    ) -> None:
        if not all(isinstance(a, torch.Tensor) and a.is_cuda for a in example_args):
            raise ValueError("GraphedUpdate needs ROCm-device tensor inputs")
        self.metric = metric
        self._metrics: List[Metric] = list(metric) if isinstance(metric, (list, tuple)) else [metric]
        if not self._metrics:
            raise ValueError("GraphedUpdate needs at least one metric")
        self._static: List[torch.Tensor] = [a.detach().clone() for a in example_args]
        befores = [
            {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in m.state_dict().items()}
            for m in self._metrics
        ]
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            for _ in range(warmup):  # workspaces / lazy buffers are created outside capture
                self._direct()
        torch.cuda.current_stream().wait_stream(stream)
        # the states (and error flags the warm-up created) move into their final contiguous
        # buffer now, not at the first sync, which would rebind what the graph writes
        from torcheval_amd.parallel.state_buffer import buffer_of

        for m in self._metrics:
            buffer_of(m)
        stream.wait_stream(torch.cuda.current_stream())
        ptrs = [_state_ptrs(m) for m in self._metrics]
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph, stream=stream):
                self._direct()
        except Exception as e:  # host syncs / H2D copies / allocations that cannot be recorded
            torch.cuda.synchronize()
            names = ", ".join(type(m).__name__ for m in self._metrics)
            raise RuntimeError(f"{names}.update cannot be captured into a HIP graph: {e}") from e
        # deferred-fold metrics (metrics/_pending.py): the buffer / spec / slots every replay adds
        # to, taken before anything reads (and so folds) the states
        self._pend_caps = []
        for m in self._metrics:
            cap = getattr(m, "_pend_capture", None)
            self._pend_caps.append(cap() if cap is not None else None)
        for m, p in zip(self._metrics, ptrs):
            if _state_ptrs(m) != p:
                raise RuntimeError(f"{type(m).__name__}.update rebinds its states; it cannot be replayed from a graph")
        torch.cuda.current_stream().wait_stream(stream)
        self.direct_us = self.replay_us = None
        if check_speed:
            self.direct_us, self.replay_us = self._time()
            if self.replay_us > self.direct_us:
                names = ", ".join(type(m).__name__ for m in self._metrics)
                warnings.warn(
                    f"GraphedUpdate({names}): a graph replay costs {self.replay_us:.1f} us against "
                    f"{self.direct_us:.1f} us for the direct update(s) on this runtime; call update directly "
                    "(graphs pay only for steps that chain many launches)",
                    RuntimeWarning,
                    stacklevel=2,
                )
        # undo the warm-up / timing updates in place (the graph holds these exact tensors)
        with torch.no_grad():
            for m, before in zip(self._metrics, befores):
                for name, v in before.items():
                    cur = getattr(m, name)
                    if isinstance(cur, torch.Tensor):
                        cur.copy_(v)
                    else:
                        setattr(m, name, v)
        torch.cuda.current_stream().wait_stream(stream)
        self._names = [tuple(n for n, q in p.items() if isinstance(q, int)) for p in ptrs]
        self._ptrs = [tuple(p[n] for n in names) for p, names in zip(ptrs, self._names)]
        # per-replay rebinding check, fast form: the captured state objects, compared by identity
        # in the metric's __dict__ (the pointer check of every state cost ~2 us per metric a
        # replay); anything else falls back to the pointer check
        self._objs = [self._locate(m, names) for m, names in zip(self._metrics, self._names)]
        self._hooks = [
            (getattr(m, "_pend_prepare", None), getattr(m, "_mark_updated", None), cap)
            for m, cap in zip(self._metrics, self._pend_caps)
        ]

    def _direct(self) -> None:
        for m in self._metrics:
            m.update(*self._static)

    def _time(self, n: int = 10) -> Tuple[float, float]:
        """Wall time per call (us) of ``n`` direct steps and of ``n`` replays, each run to
        completion: what the caller's loop pays per step either way."""
        out = []
        for replay in (False, True):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n):
                if replay:
                    self._replay()
                else:
                    self._direct()
            torch.cuda.synchronize()
            out.append((time.perf_counter() - t0) / n * 1e6)
        return out[0], out[1]

    def _replay(self) -> None:
        hooks = getattr(self, "_hooks", None)
        if hooks is None:  # the timing runs at construction
            hooks = [
                (getattr(m, "_pend_prepare", None), getattr(m, "_mark_updated", None), cap)
                for m, cap in zip(self._metrics, self._pend_caps)
            ]
        for prep, _, cap in hooks:
            if prep is not None:
                prep(cap)
        self.graph.replay()
        for _, mark, cap in hooks:
            if mark is not None:  # deferred folds (K1 micro's pending cells, K5 / K5b pending slots)
                mark(cap)

    @staticmethod
    def _locate(m: Metric, names: Tuple[str, ...]) -> Tuple[Tuple[Any, torch.Tensor], ...]:
        """(the metric ``__dict__`` key holding each raw state object, the object); key None where
        the object lives elsewhere (then only the pointer check applies)."""
        out = []
        for n in names:
            o = _raw(m, n)
            key = next((k for k, v in m.__dict__.items() if v is o), None)
            out.append((key, o))
        return tuple(out)

    @staticmethod
    def _same_objects(m: Metric, objs: Tuple[Tuple[Any, torch.Tensor], ...]) -> bool:
        d = m.__dict__
        for key, o in objs:
            if key is None or d.get(key) is not o:
                return False
        return True

    @property
    def static_inputs(self) -> Tuple[torch.Tensor, ...]:
        return tuple(self._static)

    def __call__(self, *args: torch.Tensor) -> Union[Metric, Sequence[Metric]]:
        if len(args) != len(self._static):
            raise ValueError(f"expected {len(self._static)} inputs, got {len(args)}")
        for dst, src in zip(self._static, args):
            if src.shape != dst.shape or src.dtype != dst.dtype:
                raise ValueError(
                    f"graph captured for {tuple(dst.shape)}/{dst.dtype}, got {tuple(src.shape)}/{src.dtype}"
                )
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        for i, (m, names, ptrs) in enumerate(zip(self._metrics, self._names, self._ptrs)):
            if self._same_objects(m, self._objs[i]):
                continue
            if tuple(_raw(m, n).data_ptr() for n in names) != ptrs:
                raise RuntimeError(
                    f"{type(m).__name__}: a state was rebound after graph capture (load_state_dict / to()); "
                    "re-create the GraphedUpdate"
                )
            self._objs[i] = self._locate(m, names)  # rebound onto the same memory
        self._replay()
        return self.metric
