"""North-star benchmark: MulticlassAccuracy metric-updates/sec on MI355X (BASELINE.json).

Config (BASELINE.json "metric"): MulticlassAccuracy, bs=8192 per GPU, num_classes=1000,
fp32 logits (the dtype of the reference measurement), synthetic data.  One step = one
``metric.update(logits, target)`` on a fresh batch.  Weak scaling: every rank updates its own
metric on its own batches; the timed region ends with ONE ``sync_and_compute`` (RCCL
all-reduce of the metric state) so the reported number includes the distributed merge.

Data: a pool of 8 distinct [8192, 1000] fp32 batches per GPU (262 MB, larger than the
256 MiB Infinity Cache), rotated every step, so updates stream from HBM.

Usage::

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (driver launches N > 1 this way)

Rank 0 prints ONE JSON line.

Timing: barrier + device synchronize, then ``t0``; K updates and the ``sync_and_compute``
(at N > 1 an RCCL all-gather of the metric's state buffer: no rank can leave it before every
rank has entered it, so it closes the region like a barrier would); device synchronize, then
the elapsed time, max-reduced over ranks.

Rehearsal switches (not used by the driver): ``BENCH_BACKEND=gloo`` runs the multi-rank path
over gloo, ``BENCH_DEVICE=cpu`` on CPU tensors (so the exact ``torchrun --nproc-per-node 8``
launch can be exercised without GPUs, tests/test_bench_rehearsal.py), ``BENCH_EXTRAS=0`` skips
the secondary sync timings, ``BENCH_EXTRAS=sync`` runs only the sync diagnostics (the headline's
own closing sync, its path, the direct-RCCL arm).
"""

import argparse
from datetime import timedelta
import gc
import json
import os
import time

import torch
import torch.distributed as dist

BATCH = 8192
NUM_CLASSES = 1000
POOL = 8
BASELINE_UPDATES_PER_S = 351.0  # reference MulticlassAccuracy.update bs=8192, C=1000


def _reference_eager_rate(x_pool, y_pool, iters: int) -> float:
    """The reference's update op chain (accuracy.py:250-278 + class :111-132) as eager ATen
    on the same GPU, for context: argmax -> eq -> long -> sum, torch.tensor(N), two adds."""
    dev = x_pool[0].device
    num_correct = torch.tensor(0.0, device=dev)
    num_total = torch.tensor(0.0, device=dev)

    @torch.inference_mode()
    def step(x, y):
        nonlocal num_correct, num_total
        x = x.to(dev)
        y = y.to(dev)
        pred = torch.argmax(x, dim=1)
        mask = (pred == y).long()
        c = mask.sum()
        t = torch.tensor(y.shape[0])
        num_correct += c
        num_total += t

    for i in range(20):
        step(x_pool[i % POOL], y_pool[i % POOL])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(iters):
        step(x_pool[i % POOL], y_pool[i % POOL])
    torch.cuda.synchronize()
    return iters / (time.perf_counter() - t0)


def _sync_path(metric) -> str:
    """Which engine the metric's last sync took: ``direct-rccl`` (the sync engine's own RCCL
    communicator, one grouped call) or ``c10d`` (torch.distributed collectives + seg_reduce)."""
    from torcheval_amd.parallel.state_buffer import buffer_of

    plans = list(buffer_of(metric).plans.values())
    if not plans:
        return "none"
    return "direct-rccl" if any(p.comm is not None for p in plans) else "c10d"


def _sync_extras(dev: torch.device, world: int, barrier, headline_metric) -> dict:
    """Diagnostics at N > 1, after the headline is final (max over ranks, ms per call):

    * the headline's own closing ``sync_and_compute(MulticlassAccuracy)`` and the path it took
      (``sync_path``: c10d by default at ws > 1, parallel/rccl_direct.py policy);
    * a direct-RCCL arm: ``TORCHEVAL_AMD_DIRECT_RCCL=1`` set identically on every rank, fresh
      metrics (new state buffers, so new plans), so the engine's bootstrap + self-check + MIN
      vote run here for the first time at this world size; the accuracy and CM(1000) syncs are
      timed again and ``sync_path`` says whether the vote kept the direct path or fell back;
    * BASELINE.json secondary configs: RCCL sync of a 1000x1000 confusion matrix, of
      BinaryAUROC's 1M samples per rank (all-gather-v + K3a sort of the union), and of FID's
      D=2048 states (one all-reduce of 2 x 16 MB + sums)."""
    from torcheval_amd.metrics import BinaryAUROC, MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.image.fid import FrechetInceptionDistance
    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute

    out = {}
    g = torch.Generator(device=dev).manual_seed(7 + dist.get_rank())
    only_sync = os.environ.get("BENCH_EXTRAS", "1") == "sync"  # the rehearsal's subset

    def dsync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def timed(name, fn, reps):
        try:
            fn()
            dsync()
            barrier()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            dsync()
            barrier()
            t = torch.tensor([(time.perf_counter() - t0) / reps * 1e3], dtype=torch.float64)
            if dist.get_backend() == "nccl":
                t = t.to(dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            out[name] = round(float(t), 3)
        except Exception as e:  # an extra must never cost the headline number
            out[name] = f"error: {type(e).__name__}: {e}"[:160]

    # the headline metric's own closing sync (its state: world * steps * 8192 counted samples)
    timed("accuracy_sync_and_compute", lambda: sync_and_compute(headline_metric), 20)
    out["sync_path"] = _sync_path(headline_metric)
    cm = MulticlassConfusionMatrix(1000, device=dev)
    cm.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
    timed("confusion_matrix_1000_sync_and_compute", lambda: sync_and_compute(cm), 20)

    # direct-RCCL arm (opt-in policy at ws > 1): same env on every rank, fresh state buffers
    prev = os.environ.get("TORCHEVAL_AMD_DIRECT_RCCL")
    os.environ["TORCHEVAL_AMD_DIRECT_RCCL"] = "1"
    try:
        acc_d = MulticlassAccuracy(device=dev)
        acc_d.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
        timed("direct_accuracy_sync_and_compute", lambda: sync_and_compute(acc_d), 20)
        cm_d = MulticlassConfusionMatrix(1000, device=dev)
        cm_d.update(torch.randn(8192, 1000, device=dev, generator=g), torch.randint(0, 1000, (8192,), device=dev, generator=g))
        timed("direct_confusion_matrix_1000_sync_and_compute", lambda: sync_and_compute(cm_d), 20)
        try:
            out["direct_sync_path"] = _sync_path(acc_d)
        except Exception as e:  # noqa: BLE001
            out["direct_sync_path"] = f"error: {type(e).__name__}: {e}"[:160]
    finally:
        if prev is None:
            os.environ.pop("TORCHEVAL_AMD_DIRECT_RCCL", None)
        else:
            os.environ["TORCHEVAL_AMD_DIRECT_RCCL"] = prev
    if only_sync:
        return out
    auroc = BinaryAUROC(device=dev)
    auroc.update(torch.rand(1_000_000, device=dev, generator=g), torch.randint(0, 2, (1_000_000,), device=dev, generator=g))
    timed("binary_auroc_1M_per_rank_sync_and_compute", lambda: sync_and_compute(auroc), 5)
    fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=dev)
    fid.update_activations(torch.randn(1000, 2048, device=dev, generator=g), True)
    fid.update_activations(torch.randn(1000, 2048, device=dev, generator=g), False)
    timed("fid_2048_state_sync", lambda: get_synced_metric(fid), 5)

    # sharded alternatives (torcheval_amd.parallel): same results, no full replication
    from torcheval_amd.metrics import MulticlassBinnedAUPRC
    from torcheval_amd.parallel import class_sharded_compute, sharded_compute, sharded_confusion_matrix
    from torcheval_amd.parallel.collectives import sync_timeout

    with sync_timeout(timedelta(seconds=120)):
        timed("binary_auroc_1M_per_rank_sample_sharded", lambda: sharded_compute(auroc), 5)
        timed("confusion_matrix_1000_row_sharded", lambda: sharded_confusion_matrix(cm), 20)
        ap = MulticlassBinnedAUPRC(num_classes=20000, threshold=200, average="macro", device=dev)
        for s_ in (ap.num_tp, ap.num_fp, ap.num_fn):
            s_.copy_(torch.randint(0, 1000, s_.shape, device=dev, generator=g).float())
        timed("binned_auprc_C20000_T200_sync_and_compute", lambda: sync_and_compute(ap), 5)
        timed("binned_auprc_C20000_T200_class_sharded", lambda: class_sharded_compute(ap), 5)
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--no-reference", action="store_true", help="skip the eager-ATen context run")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    from torcheval_amd.metrics import MulticlassAccuracy
    from torcheval_amd.metrics.toolkit import sync_and_compute
    from torcheval_amd.parallel import init_from_env

    # BENCH_BACKEND=gloo lets the multi-rank path be rehearsed with several ranks per GPU
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    on_cpu = os.environ.get("BENCH_DEVICE", "cuda") == "cpu"
    if on_cpu:
        backend = "gloo"
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", local_rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
    if world > 1:
        init_from_env(device_type="cuda" if backend == "nccl" else "cpu", pg_backend=backend)

    def device_sync():
        if not on_cpu:
            torch.cuda.synchronize()

    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    x_pool = [torch.randn(BATCH, NUM_CLASSES, device=dev, generator=g) for _ in range(POOL)]
    y_pool = [torch.randint(0, NUM_CLASSES, (BATCH,), device=dev, generator=g) for _ in range(POOL)]

    metric = MulticlassAccuracy(device=dev)

    def run(n_steps: int) -> torch.Tensor:
        """The timed sequence: n_steps updates, then the (synced) compute."""
        for i in range(n_steps):
            metric.update(x_pool[i % POOL], y_pool[i % POOL])
        return sync_and_compute(metric) if world > 1 else metric.compute()

    def barrier():
        if world > 1:
            if backend == "nccl":
                dist.barrier(device_ids=[dev.index])
            else:
                dist.barrier()

    # Context measurement first (untimed for the headline): the reference's eager op chain on
    # this GPU.  Running it before the warmup also brings the GPU out of its idle clock state,
    # so the K timed steps see the same clocks as a long run does.
    ref_rate = None
    if not args.no_reference and not on_cpu:
        rate = _reference_eager_rate(x_pool, y_pool, 2000)
        ref_rate = rate if rank == 0 else None

    # No automatic Python garbage-collection pass inside the warmup + ~140 us region (as timeit
    # does), and no explicit collect either: any idle gap between the warmup and t0 lets the GPU
    # drop its clocks (a collect right before the region made it 190-270 us instead of 139-143,
    # profiles/bench_region_gc_placement_r4.json).
    gc.disable()

    # Warmup runs the exact timed sequence (updates + compute / sync_and_compute), twice, so
    # every one-time cost - lazy load of a kernel's code object, allocator growth, RCCL
    # communicator setup - is paid here and not inside the timed region.
    for _ in range(2):
        run(max(args.warmup, 1))
        device_sync()
        metric.reset()

    barrier()
    device_sync()
    t0 = time.perf_counter()
    acc = run(args.steps)  # ends in sync_and_compute at N > 1: the closing rendezvous
    device_sync()
    elapsed = time.perf_counter() - t0
    gc.enable()

    # correctness guard: the synced count must equal world * steps * batch
    total = float(metric.num_total) if world == 1 else None
    if world > 1:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    else:
        assert total == args.steps * BATCH, (total, args.steps * BATCH)
    acc_v = float(acc)
    assert 0.0 <= acc_v <= 0.01, acc_v  # random logits: ~1/1000

    if rank == 0:
        updates_per_s = world * args.steps / elapsed
        out = {
            "metric": "metric-updates/sec (whole node) MulticlassAccuracy bs=8192 at 1/2/4/8 MI355X",
            "value": round(updates_per_s, 2),
            "unit": "updates/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 6),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(updates_per_s / BASELINE_UPDATES_PER_S, 2),
            "dtype": "fp32",
            "data": "synthetic (8-batch pool of randn logits / randint targets per GPU)"
            + (" [CPU rehearsal: not a GPU measurement]" if on_cpu else ""),
            "config": {
                "model": "MulticlassAccuracy",
                "global_batch": BATCH * world,
                "seq_len": None,
                "num_classes": NUM_CLASSES,
                "batch_per_gpu": BATCH,
                "average": "micro",
                "parallelism": f"dp{world}",
            },
            "samples_per_s": round(updates_per_s * BATCH, 1),
            "hbm_GBps_per_gpu": round(updates_per_s / world * BATCH * NUM_CLASSES * 4 / 1e9, 1),
            "reference_eager_same_gpu_updates_per_s": None if ref_rate is None else round(ref_rate, 1),
            "sync_ms": None,
        }

    # Secondary sync timings (N > 1) run AFTER the headline is final.  A collective that one
    # rank abandons (an exception inside an extra) would leave the others blocked forever, so a
    # watchdog bounds the whole section: on expiry rank 0 prints the headline line without the
    # extras and every rank exits 0 - the driver always gets its one JSON line.
    if world > 1 and os.environ.get("BENCH_EXTRAS", "1") != "0":
        import threading

        def _bail():
            if rank == 0:
                out["sync_ms"] = "skipped: secondary sync timings exceeded their time budget"
                print(json.dumps(out), flush=True)
            os._exit(0)

        watchdog = threading.Timer(float(os.environ.get("BENCH_EXTRAS_BUDGET_S", "180")), _bail)
        watchdog.daemon = True
        watchdog.start()
        extras = _sync_extras(dev, world, barrier, metric)
        watchdog.cancel()
        if rank == 0:
            out["sync_ms"] = extras
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        # the sync engine's own RCCL communicators go first, while every peer is still alive
        from torcheval_amd.parallel import rccl_direct

        if not on_cpu:
            torch.cuda.synchronize()
        rccl_direct.destroy_all()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
