"""binary_auroc + binary_auprc kernel breakdown (N=1M, or AUROC_N): run under
rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.functional import binary_auprc, binary_auroc  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
n = int(os.environ.get("AUROC_N", "1000000"))
x = torch.rand(n, device=dev, generator=g)
t = torch.randint(0, 2, (n,), device=dev, generator=g)
for _ in range(20):
    binary_auroc(x, t)
    binary_auprc(x, t)
torch.cuda.synchronize()
print("done")
