"""Single-process training loop with a streaming accuracy metric.

Mirrors the reference's examples/simple_example.py scenario (same seed, data recipe, model
shape and optimiser, so the printed numbers match its golden output), written against
``torcheval_amd``.  ``--device cuda`` keeps model, data and metric state on the MI355X: each
``update`` is then one K1 kernel launch and ``compute`` is the only host sync.

    python examples/simple_example.py [--device cuda]
"""

import argparse
import os
import sys

import torch
from torch import nn
from torch.utils.data import DataLoader, TensorDataset

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # run from a checkout
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402

EPOCHS, BATCHES, BATCH = 4, 16, 8
REPORT_EVERY = 4


def make_model() -> nn.Module:
    return nn.Sequential(
        nn.Sequential(nn.Linear(128, 64), nn.ReLU(), nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 2))
    )


def make_loader(device: torch.device) -> DataLoader:
    n = BATCHES * BATCH
    x = torch.randn(n, 128)
    y = torch.randint(low=0, high=2, size=(n,))
    return DataLoader(TensorDataset(x.to(device), y.to(device)), batch_size=BATCH)


def main(device: str = "cpu") -> str:
    dev = torch.device(device)
    torch.random.manual_seed(42)
    model = make_model().to(dev)
    opt = torch.optim.Adagrad(model.parameters(), lr=0.001)
    loader = make_loader(dev)
    loss_fn = nn.CrossEntropyLoss()
    acc = MulticlassAccuracy(device=dev)
    line = ""
    for epoch in range(EPOCHS):
        for step, (x, y) in enumerate(loader, start=1):
            logits = model(x)
            acc.update(logits, y)  # accumulate state; no sync
            loss = loss_fn(logits, y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            if step % REPORT_EVERY == 0:
                line = "Epoch {}/{}, Batch {}/{} --- loss: {:.4f}, acc: {:.4f}".format(
                    epoch + 1, EPOCHS, step, BATCHES, loss.item(), acc.compute()
                )
                print(line)
        acc.reset()  # per-epoch accuracy
    return line


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cpu")
    main(ap.parse_args().device)
