"""multiclass_auroc kernel breakdown (N=100k, C=100: 100 one-vs-rest rows of 100k samples):
run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.functional import multiclass_auroc  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.rand(100_000, 100, device=dev, generator=g)
t = torch.randint(0, 100, (100_000,), device=dev, generator=g)
for _ in range(20):
    multiclass_auroc(x, t, num_classes=100)
torch.cuda.synchronize()
print("done")
