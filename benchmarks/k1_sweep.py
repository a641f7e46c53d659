"""MulticlassAccuracy.update (K1) across batch sizes and class counts on one MI355X: GPU time per
update from events over 200 back-to-back updates (a pool of 4 batches), logits bandwidth, and
the eager ATen chain (argmax / eq / sum / add) on the same data for context.  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402


def _per_update_us(fn, n=200):
    for _ in range(10):
        fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []
    for c in (10, 100, 1000, 32000):
        for bs in (256, 1024, 4096, 8192, 16384, 65536):
            if bs * c * 4 * 4 > 8 << 30:
                continue
            xs = [torch.randn(bs, c, device=dev, generator=g) for _ in range(4)]
            ys = [torch.randint(0, c, (bs,), device=dev, generator=g) for _ in range(4)]
            m = MulticlassAccuracy(device=dev)
            us = _per_update_us(lambda i: m.update(xs[i % 4], ys[i % 4]))
            nc = torch.zeros((), device=dev)
            nt = torch.zeros((), device=dev)

            def eager(i):
                nc.add_((xs[i % 4].argmax(1) == ys[i % 4]).sum())
                nt.add_(bs)

            us_e = _per_update_us(eager, 50)
            rows.append({"bs": bs, "C": c, "us_per_update": round(us, 2), "TBps": round(bs * c * 4 / us / 1e6, 2),
                         "eager_aten_us": round(us_e, 2), "speedup": round(us_e / us, 2)})
            del xs, ys
    print(json.dumps({"what": __doc__.split(".")[0], "rows": rows}))


if __name__ == "__main__":
    main()
