"""torch.compile(fullgraph=True) traces metric update loops on CPU tensors (dynamo with the
eager backend: no inductor build), so a graph break in the shared update wrappers
(metric.inference_update / _instrument) or the CPU fast paths is caught without a GPU.  (CPU
updates that validate labels on the host, e.g. the confusion matrix's ``max(target)`` check,
break the graph by design, as in the reference.)"""
import pytest
import torch

from torcheval_amd.metrics import (
    BinaryAccuracy,
    BinaryAUROC,
    BinaryBinnedAUPRC,
    MulticlassAccuracy,
    HitRate,
    Mean,
    MulticlassF1Score,
    MulticlassPrecision,
    PeakSignalNoiseRatio,
    R2Score,
)

CASES = {
    "multiclass_accuracy": (MulticlassAccuracy, lambda g: (torch.randn(64, 10, generator=g), torch.randint(0, 10, (64,), generator=g))),
    "binary_accuracy": (BinaryAccuracy, lambda g: (torch.rand(64, generator=g), torch.randint(0, 2, (64,), generator=g))),
    "binary_auroc": (BinaryAUROC, lambda g: (torch.rand(64, generator=g), torch.randint(0, 2, (64,), generator=g))),
    "binned_auprc": (lambda: BinaryBinnedAUPRC(threshold=20), lambda g: (torch.rand(64, generator=g), torch.randint(0, 2, (64,), generator=g))),
    "mean": (Mean, lambda g: (torch.rand(64, generator=g),)),
    "multiclass_precision_macro": (lambda: MulticlassPrecision(num_classes=5, average="macro"),
                                   lambda g: (torch.randn(64, 5, generator=g), torch.randint(0, 5, (64,), generator=g))),
    "multiclass_f1_macro": (lambda: MulticlassF1Score(num_classes=5, average="macro"),
                            lambda g: (torch.randn(64, 5, generator=g), torch.randint(0, 5, (64,), generator=g))),
    "psnr": (PeakSignalNoiseRatio, lambda g: (torch.rand(2, 3, 4, 4, generator=g), torch.rand(2, 3, 4, 4, generator=g))),
    "r2": (R2Score, lambda g: (torch.rand(64, generator=g), torch.rand(64, generator=g))),
    "hit_rate": (lambda: HitRate(k=2), lambda g: (torch.randn(64, 5, generator=g), torch.randint(0, 5, (64,), generator=g))),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_update_traces_fullgraph_on_cpu(name):
    make, data = CASES[name]
    eager, comp = make(), make()
    torch._dynamo.reset()

    @torch.compile(fullgraph=True, backend="eager")
    def step(*args):
        comp.update(*args)

    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        args = data(g)
        eager.update(*args)
        step(*args)
    torch.testing.assert_close(comp.compute(), eager.compute())
