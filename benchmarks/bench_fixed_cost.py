"""Fixed vs per-step cost of bench.py's timed region on one GPU: T(n) for n updates + compute,
bracketed exactly like bench.py (synchronize, t0, run, synchronize), median of 15 repeats per n;
a least-squares fit T = a + b n.  Prints one JSON line."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = 8
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(pool)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(pool)]
    m = MulticlassAccuracy(device=dev)

    def run(n):
        for i in range(n):
            m.update(xs[i % pool], ys[i % pool])
        return m.compute()

    for _ in range(3):
        run(50)
        torch.cuda.synchronize()
        m.reset()
    ns = [1, 2, 5, 10, 20, 40, 100]
    med = {}
    for n in ns:
        ts = []
        for _ in range(15):
            m.reset()
            run(5)  # bench.py runs its warmup right before the timed region
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(n)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e6)
        med[n] = statistics.median(ts)
    xbar = sum(ns) / len(ns)
    ybar = sum(med[n] for n in ns) / len(ns)
    b = sum((n - xbar) * (med[n] - ybar) for n in ns) / sum((n - xbar) ** 2 for n in ns)
    a = ybar - b * xbar
    # host cost of one update (no GPU wait): the time to enqueue 20 updates
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(20):
        m.update(xs[i % pool], ys[i % pool])
    host = (time.perf_counter() - t0) * 1e6 / 20
    torch.cuda.synchronize()
    print(json.dumps({"median_us_by_steps": {str(k): round(v, 2) for k, v in med.items()},
                      "fit_fixed_us": round(a, 2), "fit_per_step_us": round(b, 3),
                      "host_us_per_update": round(host, 2),
                      "rate_at_20_steps": round(20 / med[20] * 1e6, 1)}))


if __name__ == "__main__":
    main()
