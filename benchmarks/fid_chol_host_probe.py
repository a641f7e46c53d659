"""Host vs device time of FID compute's blocked Cholesky (K9c + GEMMs) at D = 2048: is the
Python loop the limit?  torch.profiler totals over 10 calls; prints one JSON line."""
import json
import os
import sys
import time

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.image.fid import cholesky_ex  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
a = torch.randn(4000, 2048, device=dev, generator=g)
s1 = torch.cov(a.T.double())
for _ in range(3):
    cholesky_ex(s1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    cholesky_ex(s1)
host_enqueue = (time.perf_counter() - t0) / 10 * 1e3
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 10 * 1e3
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    for _ in range(10):
        cholesky_ex(s1)
    torch.cuda.synchronize()
ev = prof.key_averages()
dev_us = sum(e.self_device_time_total for e in ev) / 10
top = sorted(ev, key=lambda e: -e.self_device_time_total)[:8]
print(json.dumps({"wall_ms": round(wall, 3), "host_enqueue_ms": round(host_enqueue, 3),
                  "device_busy_ms": round(dev_us / 1e3, 3),
                  "top_device_us_per_call": {e.key[:70]: round(e.self_device_time_total / 10, 1) for e in top},
                  "calls_per_call": {e.key[:70]: e.count // 10 for e in top}}))
