"""Does the async metric sync overlap further update() calls?  

1-rank RCCL group on one MI355X with the multi-rank engine forced on.  The synced state is a
MulticlassConfusionMatrix(1000) (8 MB of int64 counts: the bucketed all-reduce path) plus a
BinaryAUROC holding 2M cached samples (the packed all-gather-v path); the overlapped work is
50 MulticlassAccuracy updates of 8192 x 1000 logits.

    serial   = blocking sync, then the 50 updates
    overlap  = sync_and_compute_async(...) ; 50 updates ; .wait()
Run under ``rocprofv3 --kernel-trace`` to see the RCCL kernels next to the K1 kernels.
Prints one JSON line (``--out`` also writes it).
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


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from torcheval_amd.metrics import BinaryAUROC, MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.toolkit import get_synced_metric_async, get_synced_metric_collection
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    cm = MulticlassConfusionMatrix(1000, device=dev)
    cm.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
    au = BinaryAUROC(device=dev)
    for _ in range(2):
        au.update(torch.rand(1_000_000, device=dev, generator=g), torch.randint(0, 2, (1_000_000,), device=dev, generator=g))
    coll = {"cm": cm, "au": au}
    acc = MulticlassAccuracy(device=dev)
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(8)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(8)]

    def updates():
        for i in range(50):
            acc.update(xs[i % 8], ys[i % 8])

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.reps * 1e3

    with collectives_at_world_size_1():
        t_upd = timed(updates)
        t_sync = timed(lambda: get_synced_metric_collection(coll))

        def serial():
            get_synced_metric_collection(coll)
            updates()

        def overlap():
            fut = get_synced_metric_async(coll)
            updates()
            fut.wait()

        t_serial = timed(serial)
        t_overlap = timed(overlap)
    dist.destroy_process_group()
    hidden = (t_serial - t_overlap) / max(min(t_sync, t_upd), 1e-9)
    res = {"what": "async metric sync overlapping 50 MulticlassAccuracy updates (1-rank RCCL, engine forced)",
           "ms": {"updates_alone": round(t_upd, 3), "sync_alone": round(t_sync, 3),
                  "serial": round(t_serial, 3), "overlapped": round(t_overlap, 3)},
           "fraction_of_shorter_phase_hidden": round(hidden, 3)}
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
