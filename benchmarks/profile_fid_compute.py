"""frechet_distance at D = 2048 (K9c blocked Cholesky, L^T S2 L, K9b eigenvalues), 5 calls:
run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.image.fid import frechet_distance  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(1)
a1 = torch.randn(4000, 2048, device=dev, generator=g)
a2 = torch.randn(4000, 2048, device=dev, generator=g) * 1.1
s1, s2 = torch.cov(a1.T.double()), torch.cov(a2.T.double())
mu1, mu2 = a1.double().mean(0), a2.double().mean(0)
for _ in range(5):
    frechet_distance(mu1, s1, mu2, s2).item()
torch.cuda.synchronize()
print("done", flush=True)
