"""Multi-rank RCCL on ONE GPU: can two processes share cuda:0 in one RCCL communicator?

Launched as ``torchrun --nproc-per-node 2 --master-addr 127.0.0.1 benchmarks/rccl_two_rank_probe.py``
on the 1-GPU box.  Each rank runs on cuda:0 with the ``nccl`` (RCCL) backend and checks, against
values it can compute locally:
  1. a torch.distributed all_reduce;
  2. the sync engine's direct RCCL communicator (``parallel/rccl_direct.py``): all_gather and
     all_reduce of small tensors;
  3. ``sync_and_compute`` of MulticlassAccuracy, MulticlassConfusionMatrix(1000) and
     BinaryAUROC through the state-buffer engine, against the concatenated-data compute.
Rank 0 prints one JSON line with each step's outcome (RCCL may refuse two ranks on one device;
then step 1 reports the error and nothing else runs)."""
import json
import os
import sys
import time
import traceback

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank = int(os.environ["RANK"])
    ws = int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {"world_size": ws}

    def step(name, fn):
        t0 = time.perf_counter()
        try:
            res = fn()
            out[name] = {"ok": True, "s": round(time.perf_counter() - t0, 3), **(res or {})}
            return True
        except Exception as e:  # noqa: BLE001 - the probe records every failure
            out[name] = {"ok": False, "error": f"{type(e).__name__}: {e}"[:300],
                         "tb": traceback.format_exc()[-600:]}
            return False

    dist.init_process_group("nccl", device_id=dev)

    def torch_all_reduce():
        t = torch.full((4,), float(rank + 1), device=dev)
        dist.all_reduce(t)
        torch.cuda.synchronize()
        want = float(sum(range(1, ws + 1)))
        assert torch.all(t == want).item(), t
        return {"value": float(t[0])}

    if not step("torch_all_reduce", torch_all_reduce):
        finish(rank, out)
        return

    from torcheval_amd.parallel import rccl_direct

    def direct():
        h = rccl_direct.comm_for(dist.group.WORLD, ws, dev)
        assert h is not None, "direct communicator not created"
        src = torch.arange(3, device=dev, dtype=torch.float32) + 10 * rank
        g = torch.empty(3 * ws, device=dev)
        rccl_direct.all_gather(h, src, g)
        r = torch.full((5,), float(rank + 1), device=dev, dtype=torch.float64)
        rccl_direct.all_reduce(h, r, "max")
        torch.cuda.synchronize()
        want = torch.cat([torch.arange(3, dtype=torch.float32) + 10 * q for q in range(ws)])
        assert torch.equal(g.cpu(), want), g
        assert torch.all(r == float(ws)).item(), r
        return {}

    step("direct_rccl", direct)

    from torcheval_amd.metrics import BinaryAUROC, MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.functional import binary_auroc
    from torcheval_amd.metrics.toolkit import sync_and_compute

    def metrics():
        gen = torch.Generator().manual_seed(99)
        xs = [torch.randn(4096, 1000, generator=gen) for _ in range(ws)]
        ys = [torch.randint(0, 1000, (4096,), generator=gen) for _ in range(ws)]
        ss = [torch.rand(200_000, generator=gen) for _ in range(ws)]
        ts = [torch.randint(0, 2, (200_000,), generator=gen) for _ in range(ws)]
        acc = MulticlassAccuracy(device=dev)
        acc.update(xs[rank].to(dev), ys[rank].to(dev))
        cm = MulticlassConfusionMatrix(1000, device=dev)
        cm.update(xs[rank].to(dev), ys[rank].to(dev))
        au = BinaryAUROC(device=dev)
        au.update(ss[rank].to(dev), ts[rank].to(dev))
        a = sync_and_compute(acc).cpu()
        c = sync_and_compute(cm).cpu()
        u = sync_and_compute(au).cpu()
        x, y = torch.cat(xs), torch.cat(ys)
        want_a = (x.argmax(1) == y).float().mean()
        want_c = torch.zeros(1000, 1000)
        want_c.index_put_((y, x.argmax(1)), torch.ones(len(y)), accumulate=True)
        want_u = binary_auroc(torch.cat(ss), torch.cat(ts))
        torch.testing.assert_close(a, want_a)
        assert torch.equal(c.float(), want_c), "confusion matrix mismatch"
        torch.testing.assert_close(u.double(), want_u.double(), rtol=1e-6, atol=1e-6)
        # the timed sequence of bench.py, a few times
        t = []
        for _ in range(20):
            torch.cuda.synchronize()
            dist.barrier(device_ids=[0])
            t0 = time.perf_counter()
            sync_and_compute(acc)
            torch.cuda.synchronize()
            t.append((time.perf_counter() - t0) * 1e6)
        return {"accuracy": float(a), "auroc": float(u), "acc_sync_and_compute_us_median": sorted(t)[len(t) // 2]}

    step("metric_sync", metrics)
    finish(rank, out)


def finish(rank, out):
    if rank == 0:
        print(json.dumps(out), flush=True)
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


if __name__ == "__main__":
    main()
