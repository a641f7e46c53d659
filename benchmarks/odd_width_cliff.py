"""Odd-width cost of the 16-B load paths: per-update GPU time (events over 200 updates, a pool of
4 batches) of MulticlassAccuracy (K1), MeanSquaredError (K5 row sums) and Sum / PSNR-style
reductions at widths that are and are not multiples of 4 (1000 vs 1001 columns, 8192 rows).
Rows of an odd width take the scalar path in these kernels; K7 got a head/body/tail split for
this (profiles/k7_grid_cap_ab_r4.json).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MeanSquaredError, MulticlassAccuracy, Sum  # noqa: E402


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
    out = {}
    for c in (1000, 1001, 4096, 4097):
        xs = [torch.randn(8192, c, device=dev, generator=g) for _ in range(4)]
        ts = [torch.randn(8192, c, device=dev, generator=g) for _ in range(4)]
        ys = [torch.randint(0, c, (8192,), device=dev, generator=g) for _ in range(4)]
        acc, mse, sm = MulticlassAccuracy(device=dev), MeanSquaredError(device=dev), Sum(device=dev)
        gb = 8192 * c * 4 / 1e3
        row = {}
        for name, fn, nbytes in (("accuracy", lambda i: acc.update(xs[i % 4], ys[i % 4]), gb),
                                 ("mse", lambda i: mse.update(xs[i % 4], ts[i % 4]), 2 * gb),
                                 ("sum", lambda i: sm.update(xs[i % 4]), gb)):
            us = _per_update_us(fn)
            row[name] = {"us": round(us, 2), "TBps": round(nbytes / us / 1e3, 2)}
        out[f"8192x{c}"] = row
        del xs, ts, ys
    print(json.dumps({"what": __doc__.split(".")[0], "rows": out}))


if __name__ == "__main__":
    main()
