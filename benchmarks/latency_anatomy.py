"""Where bench.py's fixed cost goes: host-clock latency of tiny
sequences bracketed exactly like the timed region (synchronize, t0, work, synchronize, t1),
median of 200 repeats each, on one MI355X.  Prints one JSON object (us).

  sync_only            torch.cuda.synchronize() on an idle device
  empty_kernel         one ATen fill of a 1-element tensor (smallest launch) + synchronize
  update_1             one MulticlassAccuracy.update (K1) + synchronize
  update_1_compute     update + compute (the micro_finish fold) + synchronize   == bench T(1)
  update_20_compute    bench.py's timed region at 20 steps
  k1_gpu_20            the same 20 updates timed by events on the GPU (no host wake-up)
  event_sync_1         update + compute, waited through an event instead of the device
"""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = 8
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(pool)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(pool)]
    m = MulticlassAccuracy(device=dev)
    tiny = torch.zeros(1, device=dev)

    def med(fn, reps=200):
        ts = []
        for _ in range(reps):
            m.reset()
            for i in range(5):  # bench.py's warmup right before the region
                m.update(xs[i % pool], ys[i % pool])
            m.compute()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            t1 = time.perf_counter()
            ts.append((t1 - t0) * 1e6)
        return round(statistics.median(ts), 2)

    def upd(n):
        for i in range(n):
            m.update(xs[i % pool], ys[i % pool])

    out = {
        "sync_only": med(lambda: torch.cuda.synchronize()),
        "empty_kernel": med(lambda: (tiny.fill_(1.0), torch.cuda.synchronize())),
        "update_1": med(lambda: (upd(1), torch.cuda.synchronize())),
        "update_1_compute": med(lambda: (upd(1), m.compute(), torch.cuda.synchronize())),
        "update_20_compute": med(lambda: (upd(20), m.compute(), torch.cuda.synchronize())),
    }

    def ev_sync():
        upd(1)
        m.compute()
        e = torch.cuda.Event()
        e.record()
        e.synchronize()

    out["event_sync_1"] = med(ev_sync)
    # GPU-side duration of the 20 updates + fold (events), for the host-vs-device split
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(50):
        torch.cuda.synchronize()
        e0.record()
        upd(20)
        m.compute()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    out["k1_gpu_20"] = round(statistics.median(ts), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
