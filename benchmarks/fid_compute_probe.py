"""FID compute at D = 2048 from full-rank states (the suite's row): a few calls for a kernel
timeline (rocprofv3 --kernel-trace) - where the ~10.6 ms go, gaps included."""
import sys

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.metrics.image.fid import FrechetInceptionDistance  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
D = 2048
m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D, device=dev)
for real in (True, False):
    m.update_activations(torch.randn(4 * D, D, device=dev, generator=g) * (1.0 if real else 1.1), real)
for _ in range(4):
    v = m.compute()
torch.cuda.synchronize()
print(float(v))
