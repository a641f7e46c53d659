"""K9d on a single 64 x 64 tile (one workgroup: the pair-owner task D_0 = load + factor + inverse
+ publish), repeated - the launch profiled with SQ counters to see where the factorisation's
cycles go."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.ops import native  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(64, 200, device=dev, dtype=torch.float64, generator=g)
s = x @ x.T / 200
L = torch.empty(64, 64, dtype=torch.float64, device=dev)
linv = torch.empty(4096, dtype=torch.float64, device=dev)
ctl = torch.empty(1, dtype=torch.int32, device=dev)
st = torch.empty(2, dtype=torch.int32, device=dev)
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    native().cholesky_factor(s, L, linv, ctl, st)
torch.cuda.synchronize()
print("ok", st.tolist(), float((L @ L.T - s).abs().max()))
