"""Host-side cost per call of the north-star update path (the GPU work is made trivial).

With bs=64 rows the K1 kernel takes ~2 us, so back-to-back calls measure how fast the host
can enqueue them: the per-update Python + binding + launch cost that bench.py's step time
hides only while the kernel itself is longer.  Prints one JSON object (us per call).
"""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rate(fn, iters: int = 20000) -> float:
    for _ in range(200):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / iters * 1e6


def main() -> None:
    from torcheval_amd import _C
    from torcheval_amd.metrics import MulticlassAccuracy

    dev = torch.device("cuda", 0)
    x = torch.randn(64, 1000, device=dev)
    y = torch.randint(0, 1000, (64,), device=dev)
    m = MulticlassAccuracy(device=dev)
    a, b = m.num_correct, m.num_total
    out = {
        "metric.update (bs64, C1000)": _rate(lambda: m.update(x, y)),
        "_C.micro_accuracy_update direct": _rate(lambda: _C.micro_accuracy_update(x, y, a, b)),
        "torch add_ (1 ATen launch)": _rate(lambda: a.add_(1.0)),
    }
    if hasattr(torch.ops.torcheval_amd, "micro_accuracy_update"):
        op = torch.ops.torcheval_amd.micro_accuracy_update.default
        out["torch.ops micro_accuracy_update"] = _rate(lambda: op(x, y, a, b))
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))


if __name__ == "__main__":
    main()
