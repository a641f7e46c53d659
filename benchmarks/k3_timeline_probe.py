"""binary_auroc at 1M, 60 back-to-back calls: under rocprofv3 --kernel-trace the timeline shows
whether a call is GPU-bound (kernels back to back) or host-bound (gaps between them)."""
import sys
import time

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.metrics.functional import binary_auroc  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
x = torch.rand(1_000_000, device="cuda", generator=g)
t = torch.randint(0, 2, (1_000_000,), device="cuda", generator=g)
for _ in range(10):
    binary_auroc(x, t)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(60):
    v = binary_auroc(x, t)
torch.cuda.synchronize()
print("us per call", (time.perf_counter() - t0) / 60 * 1e6, float(v))
