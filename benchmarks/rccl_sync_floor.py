"""Latency floor of the metric-state sync over RCCL on ONE MI355X (1-rank nccl group).

With ``collectives_at_world_size_1`` the full multi-rank sync engine runs (bucketed all-reduce,
packed all-gather-v with its header exchange, error-flag gather), so the numbers are the
fixed software + RCCL launch cost that every world size pays on top of the xGMI transfer time.
Cases: MulticlassConfusionMatrix(1000), FID D=2048 (2 x 2048^2 fp32 sums),
BinaryAUROC with 1M cached samples (cat states, all-gather-v), plus MulticlassAccuracy.

Prints one JSON object; ``--out`` also writes it to a file.
"""

import argparse
import json
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _time(fn, iters: int) -> float:
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from torcheval_amd.metrics import BinaryAUROC, MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.image.fid import FrechetInceptionDistance
    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1,
                            device_id=dev)
    g = torch.Generator(device=dev).manual_seed(0)

    acc = MulticlassAccuracy(device=dev)
    acc.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
    cm = MulticlassConfusionMatrix(1000, device=dev)
    cm.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
    fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=dev)
    fid.update_activations(torch.randn(4096, 2048, device=dev, generator=g), True)
    fid.update_activations(torch.randn(4096, 2048, device=dev, generator=g), False)
    au = BinaryAUROC(device=dev)
    for _ in range(8):
        au.update(torch.rand(131072, device=dev, generator=g), torch.randint(0, 2, (131072,), device=dev, generator=g))

    res = {"what": "1-rank RCCL sync latency floor (full multi-rank engine forced at ws=1)",
           "device": torch.cuda.get_device_name(0), "iters": args.iters, "ms": {}}
    with collectives_at_world_size_1():
        for name, m in (("MulticlassAccuracy", acc), ("MulticlassConfusionMatrix(1000)", cm),
                        ("FID_D2048", fid), ("BinaryAUROC_1M", au)):
            sync_ms = _time(lambda: get_synced_metric(m), args.iters)
            if name == "FID_D2048":
                snc_ms = None  # compute (eigvalsh) dominates and is timed elsewhere
            else:
                snc_ms = _time(lambda: sync_and_compute(m), args.iters)
            local_ms = _time(lambda: m.compute(), args.iters) if snc_ms is not None else None
            res["ms"][name] = {"get_synced_metric": round(sync_ms, 4),
                               "sync_and_compute": None if snc_ms is None else round(snc_ms, 4),
                               "local_compute": None if local_ms is None else round(local_ms, 4)}
    dist.destroy_process_group()
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
