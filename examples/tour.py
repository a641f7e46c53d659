"""A guided tour of torcheval_amd (counterpart of the reference's Introducing_TorchEval notebook).

Sections: functional metrics, class metrics (update / compute / merge_state / state_dict),
writing a custom metric (a two-sample Kolmogorov-Smirnov statistic with typed states),
distributed sync (2 gloo processes here; one process per MI355X over RCCL in production),
and the model tools (module summary + FLOP counter).

    python examples/tour.py [--device cuda]
"""

import argparse
import os
import sys
from typing import Iterable

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd.metrics import BinaryAUROC, Metric, MulticlassAccuracy  # noqa: E402
from torcheval_amd.metrics.functional import binary_auroc, multiclass_accuracy  # noqa: E402
from torcheval_amd.metrics.toolkit import sync_and_compute  # noqa: E402
from torcheval_amd.tools import FlopTensorDispatchMode, get_module_summary, prune_module_summary  # noqa: E402


def section(title: str) -> None:
    print(f"\n=== {title}")


class KSStatistic(Metric[torch.Tensor]):
    """Two-sample Kolmogorov-Smirnov statistic sup_x |F1(x) - F2(x)| over streamed samples.

    Samples are kept as ``cat`` states, so a distributed sync is one all-gather-v (typed path);
    ``compute`` sorts the union once."""

    def __init__(self, device=None) -> None:
        super().__init__(device=device)
        self._add_state("a", [], merge="cat")
        self._add_state("b", [], merge="cat")

    @torch.inference_mode()
    def update(self, a: torch.Tensor, b: torch.Tensor) -> "KSStatistic":
        self.a.append(a.to(self.device).flatten())
        self.b.append(b.to(self.device).flatten())
        return self

    @torch.inference_mode()
    def compute(self) -> torch.Tensor:
        a, b = torch.cat(self.a), torch.cat(self.b)
        grid = torch.cat([a, b]).sort().values
        fa = torch.searchsorted(a.sort().values, grid, right=True) / a.numel()
        fb = torch.searchsorted(b.sort().values, grid, right=True) / b.numel()
        return (fa - fb).abs().max()

    @torch.inference_mode()
    def merge_state(self, metrics: Iterable["KSStatistic"]) -> "KSStatistic":
        for m in metrics:
            self.a.extend(t.to(self.device) for t in m.a)
            self.b.extend(t.to(self.device) for t in m.b)
        return self


def _dist_worker(rank: int, ws: int) -> float:
    torch.manual_seed(rank)
    acc = MulticlassAccuracy()
    acc.update(torch.randn(100, 5), torch.randint(0, 5, (100,)))
    ks = KSStatistic().update(torch.randn(500), torch.randn(500) + 0.1 * rank)
    return float(sync_and_compute(acc)), float(sync_and_compute(ks))


def main(device: str = "cpu") -> None:
    dev = torch.device(device)
    torch.manual_seed(0)

    section("functional metrics: stateless, one call")
    logits, labels = torch.randn(64, 10, device=dev), torch.randint(0, 10, (64,), device=dev)
    print("multiclass_accuracy:", float(multiclass_accuracy(logits, labels)))
    print("binary_auroc:", float(binary_auroc(torch.rand(1000, device=dev), torch.randint(0, 2, (1000,), device=dev))))

    section("class metrics: accumulate over batches, compute once")
    acc = MulticlassAccuracy(average="macro", num_classes=10, device=dev)
    for _ in range(5):
        acc.update(torch.randn(64, 10, device=dev), torch.randint(0, 10, (64,), device=dev))
    print("macro accuracy:", float(acc.compute()))
    ckpt = acc.state_dict()  # checkpoint / resume
    fresh = MulticlassAccuracy(average="macro", num_classes=10, device=dev)
    fresh.load_state_dict(ckpt)
    print("restored == original:", bool(torch.equal(fresh.compute(), acc.compute())))

    section("merge_state: combine metrics computed on different shards")
    a, b = BinaryAUROC(device=dev), BinaryAUROC(device=dev)
    x, t = torch.rand(2000, device=dev), torch.randint(0, 2, (2000,), device=dev)
    a.update(x[:1000], t[:1000])
    b.update(x[1000:], t[1000:])
    print("merged:", float(a.merge_state([b]).compute()), " whole:", float(binary_auroc(x, t)))

    section("custom metric: two-sample KS statistic")
    ks = KSStatistic(device=dev)
    for _ in range(4):
        ks.update(torch.randn(1000, device=dev), torch.randn(1000, device=dev) + 0.2)
    print("KS(N(0,1), N(0.2,1)):", float(ks.compute()))

    section("distributed: sync_and_compute over 2 processes (gloo here; RCCL on MI355X)")
    from torcheval_amd.utils.test_utils.dist_pool import run_distributed

    for rank, (acc_v, ks_v) in enumerate(run_distributed(_dist_worker, 2)):
        print(f"rank {rank}: synced accuracy {acc_v:.4f}, synced KS {ks_v:.4f}")

    section("tools: module summary and FLOP counter")
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3), torch.nn.ReLU(), torch.nn.Flatten(), torch.nn.Linear(16 * 30 * 30, 10))
    ms = get_module_summary(model, module_args=(torch.randn(1, 3, 32, 32),))
    prune_module_summary(ms, max_depth=2)
    print(ms)
    with FlopTensorDispatchMode(model) as ftdm:
        model(torch.randn(1, 3, 32, 32)).sum().backward()
        print("forward+backward MACs per op:", dict(ftdm.flop_counts[""]))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    main(ap.parse_args().device)
