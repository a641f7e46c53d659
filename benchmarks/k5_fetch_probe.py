"""FETCH_SIZE probe of the K5 / K5b / K1 update kernels (run under rocprofv3 --pmc FETCH_SIZE):
4 updates per case, cases in a fixed order, so each kernel's dispatches map to the cases in
order.  Cases: MeanSquaredError 8192x1000 and 8192x1001 (x and t: 2 x 4 B / element),
R2Score 8192x1000, Sum 8192x1000 (4 B / element), MulticlassAccuracy 8192x1000 (scores 4 B /
element + int64 targets)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MeanSquaredError, MulticlassAccuracy, R2Score, Sum  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
CASES = [("mse_8192x1000", MeanSquaredError, 1000, 2), ("mse_8192x1001", MeanSquaredError, 1001, 2),
         ("r2_8192x1000", R2Score, 1000, 2), ("sum_8192x1000", Sum, 1000, 1), ("acc_8192x1000", MulticlassAccuracy, 1000, 0)]
for name, cls, c, ops in CASES:
    x = torch.randn(8192, c, device=dev, generator=g)
    t = torch.randn(8192, c, device=dev, generator=g) if ops == 2 else torch.randint(0, c, (8192,), device=dev, generator=g)
    m = cls(device=dev)
    for _ in range(4):
        if ops == 1:
            m.update(x)
        else:
            m.update(x, t)
    torch.cuda.synchronize()
    m.compute()
    torch.cuda.synchronize()
print("done")
