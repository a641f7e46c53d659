"""K5b deferred-mode A/B: Sum / Mean .update per-update device time (events around 200 updates
over a 4-batch pool) at 8192 x 1000 / 1001 / 4096 fp32 under the grid-size cap
(TORCHEVAL_AMD_K5B_GRID) and loads per thread (TORCHEVAL_AMD_K5B_PEND_VPT, read once per
process: run one process per value).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import Mean, Sum  # noqa: E402


def _per_call_us(fn, n=200):
    for i in range(10):
        fn(i)
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
    out = {"vpt": os.environ.get("TORCHEVAL_AMD_K5B_PEND_VPT", "8")}
    for cap in (256, 512, 1024, 2048):
        os.environ["TORCHEVAL_AMD_K5B_GRID"] = str(cap)
        for c in (1000, 1001, 4096):
            xs = [torch.randn(8192, c, device=dev, generator=g) for _ in range(4)]
            s, m = Sum(device=dev), Mean(device=dev)
            mb = 8192 * c * 4 / 1e6
            for name, fn in (("sum", lambda i: s.update(xs[i % 4])), ("mean", lambda i: m.update(xs[i % 4]))):
                us = _per_call_us(fn)
                out[f"cap{cap}_{name}_8192x{c}"] = {"us": round(us, 2), "TBps": round(mb / us, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
