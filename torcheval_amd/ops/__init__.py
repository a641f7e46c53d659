"""Native op layer: loader for ``torcheval_amd/_C.so`` (HIP/CDNA4 kernels + C++ runtime).

Dispatch rule used by every metric: tensors on a ROCm device run the hand-written HIP
kernels; CPU tensors run the ATen reference path (which is also the numerics oracle in the
tests).  On a GPU the native path is mandatory: if the extension is missing or was built
without the needed op, ``use_native`` raises instead of silently falling back, unless the
user explicitly opts out with ``TORCHEVAL_AMD_DISABLE_HIP=1``.

Environment flags:
  TORCHEVAL_AMD_DISABLE_HIP=1   force the ATen path on GPU tensors (debug / A-B only)
  TORCHEVAL_AMD_MAX_BLOCKS=N    override the streaming-kernel grid cap (tuning)
"""

import os
from typing import Any, Optional

import torch

_C: Optional[Any] = None
_LOAD_ERROR: Optional[BaseException] = None

try:  # the extension is built in-tree by torcheval_amd.ops.build / __graft_entry__.build()
    from torcheval_amd import _C as _C  # type: ignore[no-redef]
except ImportError as e:  # pragma: no cover - exercised only when unbuilt
    _C = None
    _LOAD_ERROR = e

DISABLE_HIP = os.environ.get("TORCHEVAL_AMD_DISABLE_HIP", "0") == "1"

# True while torch.compile (dynamo) traces a metric: hot paths then call the kernels through
# the dispatcher (``torch.ops.torcheval_amd.*``, with Meta kernels and mutation-annotated
# schemas, csrc/bindings.cpp) and CPU tensors take the ATen path instead of the pybind host
# twins, so compiled update loops trace into one graph.  Eager calls keep the pybind entry
# points, whose host cost per call is lower (benchmarks/host_overhead.py).
from torch.compiler import is_compiling as compiling  # noqa: E402
MAX_BLOCKS = int(os.environ.get("TORCHEVAL_AMD_MAX_BLOCKS", "0"))


def native_loaded() -> bool:
    return _C is not None


def native() -> Any:
    """Return the loaded extension module or raise a clear error."""
    if _C is None:
        raise RuntimeError(
            "torcheval_amd native extension (_C.so) is not built or failed to load: "
            f"{_LOAD_ERROR!r}. Build it with `python -m torcheval_amd.ops.build`."
        )
    return _C


def use_native(t: torch.Tensor) -> bool:
    """True when ``t`` lives on a ROCm device and the HIP path must be used."""
    if not t.is_cuda or DISABLE_HIP:
        return False
    native()  # raise loudly if missing on a GPU
    return True


def build(force: bool = False, verbose: bool = False) -> str:
    from torcheval_amd.ops.build import build as _build

    return _build(force=force, verbose=verbose)
