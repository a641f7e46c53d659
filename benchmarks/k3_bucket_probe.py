"""binary_auroc N=1M in splitter-bucket mode, a few calls (for rocprofv3 --kernel-trace --stats)."""
import sys

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.metrics.functional import binary_auroc  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.rand(1_000_000, device=dev, generator=g)
t = torch.randint(0, 2, (1_000_000,), device=dev, generator=g)
for _ in range(30):
    binary_auroc(x, t)
torch.cuda.synchronize()
print(float(binary_auroc(x, t)))
