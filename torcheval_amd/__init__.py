"""torcheval_amd — an MI355X-native (gfx950 / CDNA4) model-evaluation metrics engine.

Same capabilities and public API shape as torcheval: functional metrics
(``torcheval_amd.metrics.functional``), stateful ``Metric`` classes
(``torcheval_amd.metrics``), the distributed toolkit (``torcheval_amd.metrics.toolkit``),
and model tools (``torcheval_amd.tools``).  Hot reductions run as hand-written HIP kernels
(``torcheval_amd/_C.so``, built by ``python -m torcheval_amd.ops.build``); metric-state sync
rides RCCL over xGMI.
"""

from torcheval_amd.version import __version__

__all__ = ["__version__"]
