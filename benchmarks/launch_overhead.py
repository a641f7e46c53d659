"""Host cost per launch on this box: the K1 micro-accuracy entry point on a tiny batch (GPU
work ~nothing, so the loop is host-bound) vs ATen's own tiny-kernel launch, vs the real
8192 x 1000 update (device-bound when host < device)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torcheval_amd.ops as ops  # noqa: E402
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402

dev = torch.device("cuda", 0)
f = ops._C.micro_accuracy_update
xs, ys = torch.randn(64, 10, device=dev), torch.randint(0, 10, (64,), device=dev)
xb, yb = torch.randn(8192, 1000, device=dev), torch.randint(0, 1000, (8192,), device=dev)
c, t = torch.zeros((), device=dev), torch.zeros((), device=dev)
z = torch.zeros(16, device=dev)
m = MulticlassAccuracy(device=dev)


def rate(fn, n=20000):
    for _ in range(500):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    host = (time.perf_counter() - t0) / n * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / n * 1e6
    return round(host, 2), round(wall, 2)


out = {
    "k1_entry_tiny (host_us, wall_us)": rate(lambda: f(xs, ys, c, t)),
    "aten_add_tiny": rate(lambda: z.add_(1.0)),
    "k1_entry_8192x1000": rate(lambda: f(xb, yb, c, t), 5000),
    "metric_update_8192x1000": rate(lambda: m.update(xb, yb), 5000),
}
print(json.dumps(out))
