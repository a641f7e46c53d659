"""RetrievalPrecision(k=10, 1000 queries) update on 1M samples: run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import RetrievalPrecision  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.rand(1_000_000, device=dev, generator=g)
t = torch.randint(0, 2, (1_000_000,), device=dev, generator=g)
i = torch.randint(0, 1000, (1_000_000,), device=dev, generator=g)
m = RetrievalPrecision(k=10, num_queries=1000, device=dev)
for _ in range(20):
    m.update(x, t, indexes=i)
m.compute()
torch.cuda.synchronize()
print("done")
