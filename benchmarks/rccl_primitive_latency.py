"""Host-observed latency of bare RCCL primitives on a 1-rank group (the floor under the
metric sync engine): all_reduce / all_gather_into_tensor of a few bytes, plus a cat + view."""
import json
import socket
import time

import torch
import torch.distributed as dist


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def t(fn, n=200):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / n * 1e6, 2)


dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, device_id=dev)
a = torch.zeros(2, device=dev)
b = torch.zeros(64, dtype=torch.uint8, device=dev)
o = torch.empty(64, dtype=torch.uint8, device=dev)
x = [torch.zeros(1, device=dev), torch.zeros(1, device=dev)]
res = {
    "all_reduce_8B_us": t(lambda: dist.all_reduce(a)),
    "all_reduce_8B_async_wait_us": t(lambda: dist.all_reduce(a, async_op=True).wait()),
    "all_gather_into_tensor_64B_us": t(lambda: dist.all_gather_into_tensor(o, b)),
    "cat_2_us": t(lambda: torch.cat(x)),
    "sum0_us": t(lambda: o.view(1, 64).sum(0)),
    "empty_kernel_add_us": t(lambda: a.add_(1)),
    "item_sync_us": t(lambda: a.sum().item()),
}
# lower-overhead entry points into the same RCCL calls (the sync engine's choice)
from torch.distributed.distributed_c10d import _get_default_group

pg = _get_default_group()
res["pg_allgather_base_64B_us"] = t(lambda: pg._allgather_base(o, b).wait())
res["empty_plus_all_gather_64B_us"] = t(lambda: dist.all_gather_into_tensor(torch.empty(64, dtype=torch.uint8, device=dev), b))
res["pg_allreduce_8B_us"] = t(lambda: pg.allreduce([a]).wait())
res["host_only_all_gather_64B_us"] = None
t0 = time.perf_counter()
for _ in range(200):
    dist.all_gather_into_tensor(o, b)
res["host_only_all_gather_64B_us"] = round((time.perf_counter() - t0) / 200 * 1e6, 2)
torch.cuda.synchronize()
print(json.dumps(res))
dist.destroy_process_group()
