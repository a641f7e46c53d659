"""torch.compile(fullgraph=True) update loops run the native kernels through the dispatcher
(torch.ops.torcheval_amd.*) and match eager execution on the same data."""

import pytest
import torch

from torcheval_amd.metrics import (
    BinaryAccuracy,
    BinaryBinnedAUPRC,
    Mean,
    MeanSquaredError,
    MulticlassAccuracy,
    MulticlassConfusionMatrix,
    MultilabelAccuracy,
    R2Score,
)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _cls_data(i):
    g = torch.Generator(device=DEV).manual_seed(i)
    return torch.randn(2048, 100, device=DEV, generator=g), torch.randint(0, 100, (2048,), device=DEV, generator=g)


def _bin_data(i):
    g = torch.Generator(device=DEV).manual_seed(100 + i)
    return torch.rand(4096, device=DEV, generator=g), torch.randint(0, 2, (4096,), device=DEV, generator=g)


def _reg_data(i):
    g = torch.Generator(device=DEV).manual_seed(200 + i)
    return torch.randn(4096, 8, device=DEV, generator=g), torch.randn(4096, 8, device=DEV, generator=g)


def _ml_data(i):
    g = torch.Generator(device=DEV).manual_seed(300 + i)
    return torch.rand(1024, 50, device=DEV, generator=g), torch.randint(0, 2, (1024, 50), device=DEV, generator=g)


CASES = {
    "accuracy": (lambda: MulticlassAccuracy(device=DEV), _cls_data),
    "confusion": (lambda: MulticlassConfusionMatrix(100, device=DEV), _cls_data),
    "binned_auprc": (lambda: BinaryBinnedAUPRC(threshold=200, device=DEV), _bin_data),
    "binary_accuracy": (lambda: BinaryAccuracy(device=DEV), _bin_data),
    "mse": (lambda: MeanSquaredError(device=DEV), _reg_data),
    "r2": (lambda: R2Score(device=DEV), _reg_data),
    "multilabel_hamming": (lambda: MultilabelAccuracy(criteria="hamming", device=DEV), _ml_data),
    "mean": (lambda: Mean(device=DEV), lambda i: (_bin_data(i)[0],)),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_compiled_update_loop_matches_eager(name):
    make, data = CASES[name]
    eager, comp = make(), make()
    torch._dynamo.reset()

    @torch.compile(fullgraph=True)
    def step(*args):
        comp.update(*args)

    for i in range(4):
        args = data(i)
        eager.update(*args)
        step(*args)
    torch.testing.assert_close(comp.compute(), eager.compute())


def test_compiled_graph_holds_the_dispatcher_op():
    m = MulticlassAccuracy(device=DEV)
    seen = []

    def backend(gm, example_inputs):
        seen.extend(str(n.target) for n in gm.graph.nodes if n.op == "call_function")
        return gm

    torch._dynamo.reset()
    step = torch.compile(lambda x, y: m.update(x, y), backend=backend, fullgraph=True)
    x, y = _cls_data(0)
    step(x, y)
    assert any("torcheval_amd.micro_accuracy" in t for t in seen), seen
    torch.testing.assert_close(m.compute(), (x.argmax(1) == y).float().mean())
