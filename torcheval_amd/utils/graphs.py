"""HIP-graph capture of metric ``update`` calls.

A metric update on the native path is a handful of launches (often one: K1, K2, K5, K7 write
straight into the state tensors), so for small batches the step is launch- and Python-bound
rather than HBM-bound.  ``GraphedUpdate`` records ``metric.update(*static_inputs)`` once into a
HIP graph (``torch.cuda.CUDAGraph`` on ROCm) and then replays it: per call, the new inputs are
copied into the static input buffers and the whole update is one graph launch.

Requirements (checked): the update must write its states in place (the native kernels do;
an update that rebinds a state attribute, e.g. ``self.x = self.x + y``, would replay against
stale tensors and is rejected), must not synchronise with the host, and every replay must
use inputs of the captured shapes / dtypes.

The metric's contiguous state buffer (``parallel/state_buffer.py``) is built right before capture,
so a later ``sync_and_compute`` / ``reset`` finds it valid and never rebinds the states the
graph writes.  Anything else that rebinds a state after capture (``load_state_dict``,
``to()``) is caught at the next replay, which raises instead of writing into freed memory.
"""

from typing import Any, Dict, List, Tuple

import torch

from torcheval_amd.metrics.metric import Metric

__all__ = ["GraphedUpdate"]


def _state_ptrs(metric: Metric) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for name in metric._state_name_to_default:
        v = getattr(metric, name)
        if isinstance(v, torch.Tensor):
            out[name] = v.data_ptr()
        elif isinstance(v, list):
            out[name] = ("list", len(v))
        else:
            out[name] = ("obj", v)
    return out


class GraphedUpdate:
    """Replayable HIP graph of ``metric.update(*example_args)``.

    Example::

        acc = MulticlassAccuracy(device="cuda")
        step = GraphedUpdate(acc, logits_example, target_example)
        for logits, target in loader:
            step(logits, target)        # == acc.update(logits, target), one graph launch
        acc.compute()
    """

    def __init__(self, metric: Metric, *example_args: torch.Tensor, warmup: int = 2) -> None:
        if not all(isinstance(a, torch.Tensor) and a.is_cuda for a in example_args):
            raise ValueError("GraphedUpdate needs ROCm-device tensor inputs")
        self.metric = metric
        self._static: List[torch.Tensor] = [a.detach().clone() for a in example_args]
        before = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in metric.state_dict().items()}
        stream = torch.cuda.Stream()
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            for _ in range(warmup):  # workspaces / lazy buffers are created outside capture
                metric.update(*self._static)
        torch.cuda.current_stream().wait_stream(stream)
        # the states (and error flags the warm-up created) move into their final contiguous
        # buffer now, not at the first sync, which would rebind what the graph writes
        from torcheval_amd.parallel.state_buffer import buffer_of

        buffer_of(metric)
        stream.wait_stream(torch.cuda.current_stream())
        ptrs = _state_ptrs(metric)
        self.graph = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(self.graph, stream=stream):
                metric.update(*self._static)
        except Exception as e:  # host syncs / H2D copies / allocations that cannot be recorded
            torch.cuda.synchronize()
            raise RuntimeError(
                f"{type(metric).__name__}.update cannot be captured into a HIP graph: {e}"
            ) from e
        if _state_ptrs(metric) != ptrs:
            raise RuntimeError(
                f"{type(metric).__name__}.update rebinds its states; it cannot be replayed from a graph"
            )
        # undo the warm-up updates in place (the graph holds these exact tensors)
        with torch.no_grad():
            for name, v in before.items():
                cur = getattr(metric, name)
                if isinstance(cur, torch.Tensor):
                    cur.copy_(v)
                else:
                    setattr(metric, name, v)
        torch.cuda.current_stream().wait_stream(stream)
        self._names = tuple(n for n, p in ptrs.items() if isinstance(p, int))
        self._ptrs = tuple(ptrs[n] for n in self._names)

    @property
    def static_inputs(self) -> Tuple[torch.Tensor, ...]:
        return tuple(self._static)

    def __call__(self, *args: torch.Tensor) -> Metric:
        if len(args) != len(self._static):
            raise ValueError(f"expected {len(self._static)} inputs, got {len(args)}")
        for dst, src in zip(self._static, args):
            if src.shape != dst.shape or src.dtype != dst.dtype:
                raise ValueError(
                    f"graph captured for {tuple(dst.shape)}/{dst.dtype}, got {tuple(src.shape)}/{src.dtype}"
                )
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        m = self.metric
        if tuple(getattr(m, n).data_ptr() for n in self._names) != self._ptrs:
            raise RuntimeError(
                f"{type(m).__name__}: a state was rebound after graph capture (load_state_dict / to()); "
                "re-create the GraphedUpdate"
            )
        self.graph.replay()
        mark = getattr(self.metric, "_mark_updated", None)
        if mark is not None:  # metrics with deferred folds (K1 micro's pending cells)
            mark()
        return self.metric
