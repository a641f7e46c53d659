"""binary_auroc N=1M kernel breakdown: run under rocprofv3 --kernel-trace --stats."""
import os
import sys

os.environ.setdefault("TORCHEVAL_AMD_K3S", "1")

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.functional import binary_auroc  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.rand(1_000_000, device=dev, generator=g)
t = torch.randint(0, 2, (1_000_000,), device=dev, generator=g)
for _ in range(20):
    binary_auroc(x, t)
torch.cuda.synchronize()
print("done")
