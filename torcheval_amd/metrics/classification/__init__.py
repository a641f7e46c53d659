from torcheval_amd.metrics.classification.accuracy import (
    BinaryAccuracy,
    MulticlassAccuracy,
    MultilabelAccuracy,
    TopKMultilabelAccuracy,
)

__all__ = [
    "BinaryAccuracy",
    "MulticlassAccuracy",
    "MultilabelAccuracy",
    "TopKMultilabelAccuracy",
]
