"""bench.py's timed region, one per fresh metric, in one process: (a) bench.py's order
(warm-up sequences, then gc.collect() right before the region) against (b) gc.collect() before
the warm-up, so the GPU is busy until the region starts.  Region times in us, in order."""
import gc
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from torcheval_amd.metrics import MulticlassAccuracy  # noqa: E402


def main(n: int = 6):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1234)
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(8)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(8)]
    bench._reference_eager_rate(xs, ys, 2000)
    res = {"gc_before_region": [], "gc_before_warmup": [], "no_gc_call": []}
    for _ in range(n):
        for arm in res:
            m = MulticlassAccuracy(device=dev)

            def run(k):
                for i in range(k):
                    m.update(xs[i % 8], ys[i % 8])
                return m.compute()

            if arm == "gc_before_warmup":
                gc.collect()
                gc.disable()
            for _ in range(2):
                run(5)
                torch.cuda.synchronize()
                m.reset()
            if arm == "gc_before_region":
                gc.collect()
                gc.disable()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(20)
            torch.cuda.synchronize()
            res[arm].append(round((time.perf_counter() - t0) * 1e6, 1))
            gc.enable()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
