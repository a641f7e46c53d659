"""Async metric sync overlapping update() on the device, measured as kernels.

1-rank RCCL group on one MI355X with the multi-rank engine forced.  The synced metric is a
MulticlassConfusionMatrix(4096): 128 MB of int64 counts, one bucketed all_reduce on RCCL's
stream, with no host read on the way (its error flag rides the same all_reduce).  The
overlapped work is 64 MulticlassAccuracy K1 updates of 8192 x 1000 logits on the compute
stream.

    serial  = get_synced_metric(cm); 64 updates
    overlap = get_synced_metric_async(cm); 64 updates; .wait()

Run it under ``rocprofv3 --kernel-trace`` and pass the trace CSV to ``--trace`` in a second,
GPU-free invocation: it reports, per overlapped call, how many K1 kernels ran while the RCCL
kernel was running (their [start, end] intervals intersect).
"""

import argparse
import csv
import json
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(reps: int) -> dict:
    import torch
    import torch.distributed as dist

    from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.toolkit import get_synced_metric, get_synced_metric_async
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    cm = MulticlassConfusionMatrix(4096, device=dev)
    cm.update(torch.randn(8192, 4096, device=dev, generator=g), torch.randint(0, 4096, (8192,), device=dev, generator=g))
    acc = MulticlassAccuracy(device=dev)
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(8)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(8)]

    def updates():
        for i in range(64):
            acc.update(xs[i % 8], ys[i % 8])

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    with collectives_at_world_size_1():
        t_upd = timed(updates)
        t_sync = timed(lambda: get_synced_metric(cm))

        def serial():
            get_synced_metric(cm)
            updates()

        def overlap():
            fut = get_synced_metric_async(cm)
            updates()
            return fut.wait()

        t_serial = timed(serial)
        t_overlap = timed(overlap)
        synced = overlap()
        assert torch.equal(synced.confusion_matrix, cm.confusion_matrix)  # snapshot taken at the call
    dist.destroy_process_group()
    return {"updates_alone": round(t_upd, 3), "sync_alone": round(t_sync, 3),
            "serial": round(t_serial, 3), "overlapped": round(t_overlap, 3),
            "hidden_ms": round(t_serial - t_overlap, 3)}


def analyse(trace: str) -> dict:
    rows = list(csv.DictReader(open(trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")) for r in rows))
    rccl = [k for k in ks if "nccl" in k[2].lower() or "rccl" in k[2].lower()]
    k1 = [k for k in ks if "cls_micro_kernel" in k[2] or "cls_wide_kernel" in k[2]]
    per = []
    for s, e, name, q in rccl:
        inside = [k for k in k1 if k[0] < e and k[1] > s]
        per.append({"rccl_kernel": name[:60], "rccl_us": round((e - s) / 1e3, 2), "rccl_queue": q,
                    "k1_kernels_overlapping": len(inside),
                    "k1_queues": sorted({k[3] for k in inside})})
    busy = [p for p in per if p["k1_kernels_overlapping"] > 0]
    return {"rccl_kernels": len(per), "rccl_kernels_with_concurrent_k1": len(busy),
            "max_k1_kernels_inside_one_rccl_kernel": max([p["k1_kernels_overlapping"] for p in per], default=0),
            "examples": busy[:4]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--trace", default=None, help="rocprofv3 kernel_trace.csv of a previous run: analyse only")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    if args.trace:
        res = {"what": "kernel-trace overlap of the async CM(4096) sync with K1 updates", **analyse(args.trace)}
    else:
        res = {"what": "async CM(4096) sync (128 MB all_reduce, 1-rank RCCL, engine forced) vs 64 K1 updates",
               "ms": run(args.reps)}
    line = json.dumps(res)
    print(line)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
