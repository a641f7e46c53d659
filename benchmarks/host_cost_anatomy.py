"""Host cost of one north-star update, by layer: median over 200 reps of
the host time to enqueue 20 calls (device synchronized before each rep), in us per call.

  update            MulticlassAccuracy.update (bench.py's call)
  native_direct     the extension's micro_accuracy_update called straight (no Metric method)
  native_reject     the same entry given a CPU tensor: returns at its first test (pybind +
                    argument conversion only)
  py_method_noop    a Python method call that does nothing
  aten_add_         ``tiny.add_(1)`` on a 1-element CUDA tensor (one ATen launch)
Prints one JSON object."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402
from torcheval_amd.ops import native  # noqa: E402


class _Noop:
    def update(self, a, b):
        return self


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    pool = 8
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(pool)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(pool)]
    m = MulticlassAccuracy(device=dev)
    m.update(xs[0], ys[0])
    d = m.__dict__
    pend = d["_pend"]
    fast = native().micro_accuracy_update
    cpu_x = torch.zeros(4, 4)
    tiny = torch.zeros(1, device=dev)
    noop = _Noop()

    def per_call(fn, reps=200):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(20):
                fn(i)
            ts.append((time.perf_counter() - t0) * 1e6 / 20)
        torch.cuda.synchronize()
        return round(statistics.median(ts), 3)

    out = {
        "update": per_call(lambda i: m.update(xs[i % pool], ys[i % pool])),
        "native_direct": per_call(lambda i: fast(xs[i % pool], ys[i % pool], d["_nc"], d["num_total"], 0, pend)),
        "native_reject": per_call(lambda i: fast(cpu_x, ys[i % pool], d["_nc"], d["num_total"], 0, pend)),
        "py_method_noop": per_call(lambda i: noop.update(xs[i % pool], ys[i % pool])),
        "aten_add_": per_call(lambda i: tiny.add_(1)),
    }
    # bench.py's timed region (20 updates + compute, synchronize on both sides) in variants, to
    # locate the gap to the same region driven from C++ (csrc/bench/k1_floor.hip)
    fin = native().micro_accuracy_finish
    res = torch.empty((), dtype=torch.float32, device=dev)

    def region(body, sync=torch.cuda.synchronize, reps=100):
        ts = []
        for _ in range(reps):
            m.reset()
            for i in range(5):
                m.update(xs[i % pool], ys[i % pool])
            m.compute()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            body()
            sync()
            ts.append((time.perf_counter() - t0) * 1e6)
        return round(statistics.median(ts), 2)

    def metric_body():
        for i in range(20):
            m.update(xs[i % pool], ys[i % pool])
        m.compute()

    def native_body():
        nc, nt = d["_nc"], d["num_total"]
        for i in range(20):
            fast(xs[i % pool], ys[i % pool], nc, nt, 0, pend)
        fin(pend, nc, nt, res)

    def updates_only():
        for i in range(20):
            m.update(xs[i % pool], ys[i % pool])

    stream = torch.cuda.current_stream()
    out["region_metric"] = region(metric_body)
    out["region_native"] = region(native_body)
    out["region_updates_only"] = region(updates_only)
    out["region_metric_stream_sync"] = region(metric_body, sync=stream.synchronize)

    def ev_sync():
        e = torch.cuda.Event()
        e.record()
        e.synchronize()

    out["region_metric_event_sync"] = region(metric_body, sync=ev_sync)
    # host time of compute() alone while the GPU is still busy with the 20 updates
    ts = []
    for _ in range(100):
        torch.cuda.synchronize()
        updates_only()
        t0 = time.perf_counter()
        m.compute()
        ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    out["compute_host_us"] = round(statistics.median(ts), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
