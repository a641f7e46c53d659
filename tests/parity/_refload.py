"""Load the read-only reference (Connor-Guo/torcheval) as a differential oracle.

The reference is pure Python over ATen; it imports two packages this image lacks
(``torchtnt`` helpers and ``torchvision`` for FID's default model).  Minimal import shims are
installed for exactly the symbols it touches at import time, then ``torcheval`` is imported
from ``/root/reference``.  Used only by ``gen_goldens.py`` (offline golden generation) and
the live differential tests, which skip when the reference is not mounted (e.g. on the GPU
box, where the committed goldens are used instead).
"""

import importlib.machinery
import os
import sys
import types

REFERENCE = os.environ.get("TORCHEVAL_REFERENCE", "/root/reference")


def available() -> bool:
    return os.path.isfile(os.path.join(REFERENCE, "torcheval", "metrics", "metric.py"))


def _module(name: str) -> types.ModuleType:
    m = types.ModuleType(name)
    m.__spec__ = importlib.machinery.ModuleSpec(name, None)
    sys.modules[name] = m
    return m


def _install_shims() -> None:
    import torch
    import torch.distributed as dist

    if "torchvision" not in sys.modules:
        tv = _module("torchvision")
        tv.models = _module("torchvision.models")
    if "torchtnt" in sys.modules:
        return
    _module("torchtnt")
    utils = _module("torchtnt.utils")

    class PGWrapper:
        def __init__(self, pg=None) -> None:
            self.pg = pg

        def get_world_size(self) -> int:
            return dist.get_world_size(self.pg) if dist.is_initialized() else 1

    class Timer:  # module_summary imports it; timing hooks are not exercised here
        pass

    utils.PGWrapper = PGWrapper
    utils.Timer = Timer
    utils.copy_data_to_device = lambda data, device: data
    utils.init_from_env = lambda *a, **k: torch.device("cpu")
    ver = _module("torchtnt.utils.version")
    ver.is_torch_version_geq_1_13 = lambda: True
    d = _module("torchtnt.utils.distributed")

    def all_gather_tensors(t, group=None):
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(group))]
        dist.all_gather(out, t, group=group)
        return out

    d.all_gather_tensors = all_gather_tensors


def load():
    """Return ``(reference_metrics_module, reference_functional_module)``."""
    if not available():
        raise RuntimeError(f"reference not mounted at {REFERENCE}")
    _install_shims()
    if REFERENCE not in sys.path:
        sys.path.append(REFERENCE)
    import torcheval.metrics as M  # noqa: E402
    import torcheval.metrics.functional as F  # noqa: E402

    return M, F
