"""Where the host time of one sync goes (1-rank RCCL group, collectives forced): each phase of
the state-buffer sync of MulticlassAccuracy and MulticlassConfusionMatrix(1000) timed alone,
back to back, plus the end-to-end calls.  Prints one JSON object (us per call)."""

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


def _t(fn, n=300) -> float:
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


def main() -> None:
    from torcheval_amd.metrics import MulticlassAccuracy, MulticlassConfusionMatrix
    from torcheval_amd.metrics.image.fid import FrechetInceptionDistance
    from torcheval_amd.parallel import rccl_direct
    from torcheval_amd.metrics.toolkit import get_synced_metric, sync_and_compute
    from torcheval_amd.parallel import state_buffer as sbm
    from torcheval_amd.parallel.collectives import collectives_at_world_size_1

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
    x = torch.randn(8192, 1000, device=dev)
    y = torch.randint(0, 1000, (8192,), device=dev)
    out = {}
    with collectives_at_world_size_1():
        fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=dev)
        fid.update_activations(torch.randn(1000, 2048, device=dev), True)
        fid.update_activations(torch.randn(1000, 2048, device=dev), False)
        for name, m in (("acc", MulticlassAccuracy(device=dev)), ("cm", MulticlassConfusionMatrix(1000, device=dev)),
                        ("fid", fid)):
            if name != "fid":
                m.update(x, y)
            sync_and_compute(m)
            sb = sbm.buffer_of(m)
            plan = sbm._plan_for(sb, dist.group.WORLD, 1, m)
            res = {
                "get_synced_metric": _t(lambda: get_synced_metric(m)),
                "buffer_valid": _t(lambda: sb.valid(m)),
                "sync_one": _t(lambda: sbm._sync_one(m, sb, plan)),
            }
            if name != "fid":  # FID's compute is the D=2048 eigen-solve (profiled separately)
                res["sync_and_compute"] = _t(lambda: sync_and_compute(m))
                res["local_compute"] = _t(lambda: m.compute())
            if plan.rplan is not None:  # the direct plan's phases
                dst = torch.empty(sb.buf.numel(), dtype=torch.uint8, device=dev)
                res["result_alloc"] = _t(lambda: torch.empty(sb.buf.numel(), dtype=torch.uint8, device=dev))
                res["plan_run"] = _t(lambda: rccl_direct.plan_run(plan.comm, plan.rplan, sb.buf, dst, 1))
                res["merged_copy"] = _t(lambda: sbm._merged_copy(m, dst, plan.dassign))
                res["device_copy_same_bytes"] = _t(lambda: dst.copy_(sb.buf))
                os.environ["TORCHEVAL_AMD_RCCL_WATCHDOG"] = "0"  # A/B: no completion event
                res["plan_run_no_watchdog"] = _t(lambda: rccl_direct.plan_run(plan.comm, plan.rplan, sb.buf, dst, 1))
                res["get_synced_metric_no_watchdog"] = _t(lambda: get_synced_metric(m))
                del os.environ["TORCHEVAL_AMD_RCCL_WATCHDOG"]
                t8 = torch.zeros(2, device=dev)
                res["raw_all_reduce_8B"] = _t(lambda: rccl_direct.all_reduce(plan.comm, t8, "sum"))
                ev = torch.cuda.Event()
                res["torch_event_record"] = _t(lambda: ev.record())
            if plan.src is not None and plan.rplan is None:
                res["gather_only"] = _t(lambda: sbm._gather(plan, plan.src))
            if plan.large and plan.rplan is None:
                res["snapshot_clone"] = _t(lambda: sb.buf[: sb.reduce_end].clone())
                snap = sb.buf[: sb.reduce_end].clone()
                off, nb, dtype, op = plan.large[0]
                res["all_reduce_only"] = _t(lambda: sbm._all_reduce_group(snap[off : off + nb].view(dtype), op, plan.group))
            out[name] = res
    dist.destroy_process_group()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
