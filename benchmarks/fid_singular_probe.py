"""FID compute with rank-deficient covariances (1000 samples, D = 2048): the eigh + rank-r path."""
import sys
sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import time, torch
from torcheval_amd.metrics.image.fid import _tr_sqrt_product
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(1000, 2048, device=dev, generator=g, dtype=torch.float64)
b = torch.randn(1000, 2048, device=dev, generator=g, dtype=torch.float64)
s1, s2 = torch.cov(a.T), torch.cov(b.T)
for _ in range(2): _tr_sqrt_product(s1, s2)
torch.cuda.synchronize(); t = time.perf_counter()
for _ in range(5): v = _tr_sqrt_product(s1, s2)
torch.cuda.synchronize(); print("rank-deficient tr sqrt ms", (time.perf_counter() - t) / 5 * 1e3, float(v))
