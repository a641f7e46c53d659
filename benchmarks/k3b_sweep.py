"""K3b (bucketed, no global sort) vs K3a sort + K3 scan: binary_auroc / binary_auprc latency per
call over n, uniform and normal scores.  Prints one JSON object (us per call, device-synced
loop of back-to-back calls, so it includes the host launch cost)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.functional import binary_auprc, binary_auroc  # noqa: E402


def _t(fn, iters=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - t0) / iters * 1e6, 2)


def main():
    dev = torch.device("cuda", 0)
    out = {}
    for n in [1 << 15, 1 << 16, 1 << 17, 1 << 18, 1 << 19, 1_000_000, 1 << 21, 1 << 22]:
        g = torch.Generator(device=dev).manual_seed(n)
        t = torch.randint(0, 2, (n,), device=dev, generator=g)
        for dist in ("uniform", "normal"):
            x = torch.rand(n, device=dev, generator=g) if dist == "uniform" else torch.randn(n, device=dev, generator=g)
            row = {}
            for path in ("1", "0"):
                os.environ["TORCHEVAL_AMD_K3B"] = path
                key = "k3b" if path == "1" else "k3a_k3"
                row[key + "_auroc_us"] = _t(lambda: binary_auroc(x, t))
                row[key + "_auprc_us"] = _t(lambda: binary_auprc(x, t))
            out[f"{dist}_{n}"] = row
            print(f"{dist} {n} {row}", flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
