"""Data-parallel training with metrics synced over RCCL (or gloo on CPU).

One process per GPU (``torchrun --nproc-per-node N``); every rank updates its own metric
states on its own shard, and ``sync_and_compute`` merges them across ranks: states declared
``merge="sum"`` (accuracy counts, confusion matrix) travel in ONE bucketed all-reduce, while
``Throughput`` (custom merge) goes through the packed all-gather.  Scenario and printed
format follow the reference's examples/distributed_example.py.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/distributed_example.py
    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/distributed_example.py --device cpu
"""

import argparse
import os
import sys
import time

import torch
import torch.distributed as dist
from torch import nn
from torch.nn.parallel import DistributedDataParallel as DDP
from torch.utils.data import DataLoader, TensorDataset

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # run from a checkout
from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix, Throughput  # noqa: E402
from torcheval_amd.metrics.toolkit import sync_and_compute, sync_and_compute_collection  # noqa: E402
from torcheval_amd.parallel import init_from_env  # noqa: E402

EPOCHS, BATCHES, BATCH = 4, 16, 8
REPORT_EVERY = 4


def run(device_type: str) -> None:
    dev = init_from_env(device_type=device_type)
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(42)  # identical init on every rank (DDP also broadcasts rank 0's)
    model = DDP(
        nn.Sequential(nn.Linear(128, 64), nn.ReLU(), nn.Linear(64, 32), nn.ReLU(), nn.Linear(32, 2)).to(dev),
        device_ids=[dev.index] if dev.type == "cuda" else None,
    )
    opt = torch.optim.Adagrad(model.parameters(), lr=0.001)
    g = torch.Generator().manual_seed(1000 + rank)  # each rank sees its own data shard
    n = BATCHES * BATCH
    loader = DataLoader(
        TensorDataset(torch.randn(n, 128, generator=g).to(dev), torch.randint(0, 2, (n,), generator=g).to(dev)),
        batch_size=BATCH,
    )
    loss_fn = nn.CrossEntropyLoss()
    metrics = {
        "acc": MulticlassAccuracy(device=dev),
        "confusion": MulticlassConfusionMatrix(2, device=dev),
    }
    throughput = Throughput(device=dev)

    for epoch in range(EPOCHS):
        t0 = time.monotonic()
        for step, (x, y) in enumerate(loader, start=1):
            logits = model(x)
            loss = loss_fn(logits, y)
            opt.zero_grad()
            loss.backward()
            opt.step()
            for m in metrics.values():
                m.update(logits, y)
            if step % REPORT_EVERY == 0:
                # collective: every rank must call it; one all-reduce for both metrics
                res = sync_and_compute_collection(metrics)
                if rank == 0:
                    print(
                        "Epoch {}/{}, Batch {}/{} --- loss: {:.4f}, acc: {:.4f}".format(
                            epoch + 1, EPOCHS, step, BATCHES, loss.item(), res["acc"]
                        )
                    )
            throughput.update(step * BATCH, time.monotonic() - t0)
        for m in metrics.values():
            m.reset()

    global_tput = sync_and_compute(throughput)  # sum of items / slowest rank's time
    local_tput = throughput.compute()
    if rank == 0:
        print(f"Epoch{EPOCHS}/{EPOCHS} -- synced throughput:{global_tput}")
        print(
            f"Epoch{EPOCHS}/{EPOCHS} -- local throughput:{local_tput}, "
            f"approximate global throughput: {local_tput * world}"
        )
    dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    run(ap.parse_args().device)
