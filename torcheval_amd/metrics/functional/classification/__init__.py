from torcheval_amd.metrics.functional.classification.accuracy import (
    binary_accuracy,
    multiclass_accuracy,
    multilabel_accuracy,
    topk_multilabel_accuracy,
)

__all__ = [
    "binary_accuracy",
    "multiclass_accuracy",
    "multilabel_accuracy",
    "topk_multilabel_accuracy",
]
