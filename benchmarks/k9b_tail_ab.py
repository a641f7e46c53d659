"""K9b tail A/B: FID compute at D = 2048 (full rank) and sym_eigvalsh accuracy against torch's
eigvalsh, one process per arm (TORCHEVAL_AMD_SYMEIG_TAIL is read once per process).
TORCHEVAL_AMD_SYMEIG_TAIL=0 runs the grid-only reduction (profiles/k9b_tail_r6.json)."""
import json
import os
import sys
import time

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.metrics.image.fid import FrechetInceptionDistance, sym_eigvalsh  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
out = {"tail": os.environ.get("TORCHEVAL_AMD_SYMEIG_TAIL", "1")}
for D in (300, 1000, 2048):
    x = torch.randn(D, D, device=dev, generator=g, dtype=torch.float64)
    s = (x + x.T) / 2
    ref = torch.linalg.eigvalsh(s)
    lam = torch.sort(sym_eigvalsh(s)).values
    out[f"eig_maxrel_D{D}"] = float(((lam - ref).abs().max() / ref.abs().max()))
D = 2048
m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D, device=dev)
for real in (True, False):
    m.update_activations(torch.randn(4 * D, D, device=dev, generator=g) * (1.0 if real else 1.1), real)
v = m.compute()
torch.cuda.synchronize()
ts = []
for _ in range(8):
    t = time.perf_counter()
    v = m.compute()
    torch.cuda.synchronize()
    ts.append((time.perf_counter() - t) * 1e3)
out["fid"] = float(v)
out["fid_compute_ms_min"] = min(ts)
out["fid_compute_ms_med"] = sorted(ts)[4]
print(json.dumps(out))
