"""Distributed layer: one process per MI355X, RCCL (backend "nccl") over xGMI.

* ``distributed`` — process-group helpers (PGWrapper, init_from_env, transport device).
* ``collectives`` — bucketed all-reduce and packed all-gather-v of metric states.
* ``state_sync`` — typed metric-state sync engine used by ``metrics.toolkit``.
* ``class_shard`` — class-dimension reduce-scatter sync (row-sharded confusion matrix, binned AUPRC).
* ``dist_auc`` — sample-sharded exact AUROC / AUPRC (splitter all-to-all + K3 shard offsets).
"""

from torcheval_amd.parallel.collectives import (
    all_gather_tensors,
    allreduce_coalesced,
    allreduce_coalesced_async,
    packed_all_gather,
)
from torcheval_amd.parallel.distributed import (
    get_local_rank,
    get_rank,
    get_world_size,
    init_from_env,
    PGWrapper,
    transport_device,
)

__all__ = [
    "PGWrapper",
    "all_gather_tensors",
    "allreduce_coalesced",
    "allreduce_coalesced_async",
    "get_local_rank",
    "get_rank",
    "get_world_size",
    "init_from_env",
    "packed_all_gather",
    "transport_device",
    "distributed_binary_auroc",
    "distributed_binary_auprc",
    "distributed_binary_areas",
    "sharded_compute",
    "class_sharded_compute",
    "reduce_scatter_classes",
    "sharded_confusion_matrix",
]

_LAZY = {
    "distributed_binary_auroc": "dist_auc",
    "distributed_binary_auprc": "dist_auc",
    "distributed_binary_areas": "dist_auc",
    "sharded_compute": "dist_auc",
    "class_sharded_compute": "class_shard",
    "reduce_scatter_classes": "class_shard",
    "sharded_confusion_matrix": "class_shard",
}


def __getattr__(name):  # these modules import the metric layer, which imports this package
    if name in _LAZY:
        import importlib

        return getattr(importlib.import_module(f"torcheval_amd.parallel.{_LAZY[name]}"), name)
    raise AttributeError(name)
