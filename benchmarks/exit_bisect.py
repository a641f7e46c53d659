"""Exit-time crash bisection under rocprofv3: one workload stage per run,
selected by argv[1]; prints "done" and exits normally.  Stages:
  import      import torcheval_amd and load _C.so, touch the GPU
  k1          one MulticlassAccuracy update + compute
  chol        cholesky_ex (K9c potrf blocks + GEMMs) at D=512
  eig         sym_eigvalsh (K9b cooperative tridiagonalisation + multisection) at D=512
  fid         frechet_distance at D=512 (all of the above)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

stage = sys.argv[1]
dev = torch.device("cuda", 0)
import torcheval_amd  # noqa: E402,F401
from torcheval_amd.ops import native  # noqa: E402

native()
torch.zeros(1, device=dev).sum().item()
if stage == "k1":
    from torcheval_amd.metrics import MulticlassAccuracy

    m = MulticlassAccuracy(device=dev)
    m.update(torch.randn(64, 100, device=dev), torch.randint(0, 100, (64,), device=dev))
    m.compute().item()
elif stage in ("chol", "eig", "fid"):
    from torcheval_amd.metrics.image.fid import cholesky_ex, frechet_distance, sym_eigvalsh

    a = torch.randn(1000, 512, device=dev, dtype=torch.float64)
    s = torch.cov(a.T)
    if stage == "chol":
        cholesky_ex(s)[0].sum().item()
    elif stage == "eig":
        sym_eigvalsh(s).sum().item()
    else:
        mu = a.mean(0)
        frechet_distance(mu, s, mu * 1.1, s * 1.2).item()
torch.cuda.synchronize()
print("done", flush=True)
