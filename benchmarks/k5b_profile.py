"""K5b at 8192x1000 (Sum / PSNR / 64-task CTR updates): host-side cost per call vs device time.
Host cost = wall time of N back-to-back calls without a sync in between / N (launch-bound when
it exceeds the kernel time); run under rocprofv3 --kernel-trace --stats for the device side."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd import metrics as M  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
pool = [torch.rand(8192, 1000, device=dev, generator=g) for _ in range(8)]  # 262 MB: HBM-resident
t = torch.rand(8192, 1000, device=dev, generator=g)
clicks = [(torch.rand(64, 128000, device=dev, generator=g) < 0.3).float() for _ in range(4)]
w = torch.rand(64, 128000, device=dev, generator=g)
s, p, c = M.Sum(device=dev), M.PeakSignalNoiseRatio(device=dev), M.ClickThroughRate(num_tasks=64, device=dev)
for name, fn in (("Sum", lambda i: s.update(pool[i % 8])), ("PSNR", lambda i: p.update(pool[i % 8], t)),
                 ("CTR64", lambda i: c.update(clicks[i % 4], w))):
    for i in range(50):
        fn(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(2000):
        fn(i)
    host = (time.perf_counter() - t0) / 2000 * 1e6
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / 2000 * 1e6
    print(f"{name}: host {host:.2f} us/call, wall {wall:.2f} us/call", flush=True)
