"""Host profile (cProfile) of sync_and_compute(MulticlassAccuracy) on a 1-rank RCCL group with
the multi-rank engine forced; prints the top functions by total time."""
import cProfile
import os
import pstats
import socket
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402
from torcheval_amd.metrics.toolkit import sync_and_compute  # noqa: E402
from torcheval_amd.parallel.collectives import collectives_at_world_size_1  # noqa: E402

s = socket.socket()
s.bind(("127.0.0.1", 0))
port = s.getsockname()[1]
s.close()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
m = MulticlassAccuracy(device=dev)
m.update(torch.randn(8192, 1000, device=dev), torch.randint(0, 1000, (8192,), device=dev))
with collectives_at_world_size_1():
    for _ in range(100):
        sync_and_compute(m)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(1000):
        sync_and_compute(m)
    host = (time.perf_counter() - t0) / 1000 * 1e6
    torch.cuda.synchronize()
    print("us per sync_and_compute (host, then wall)", round(host, 1), round((time.perf_counter() - t0) / 1000 * 1e6, 1))
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(1000):
        sync_and_compute(m)
    pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
dist.destroy_process_group()
