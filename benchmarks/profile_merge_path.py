"""Kernel breakdown of the sorted-run synced AUROC (8 runs x 1M) vs binary_auroc of the union;
run under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics.functional import binary_auroc  # noqa: E402
from torcheval_amd.metrics.functional.classification._curve import merged_areas, sort_run  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
R, per = 8, 1_000_000
runs = [sort_run(torch.rand(per, device=dev, generator=g), torch.randint(0, 2, (per,), device=dev, generator=g), None)
        for _ in range(R)]
xs, ts = [r[0] for r in runs], [r[1] for r in runs]
X, T = torch.cat(xs), torch.cat(ts)
which = sys.argv[1] if len(sys.argv) > 1 else "merge"
for _ in range(3):
    merged_areas(xs, ts, None, roc=True, pr=False) if which == "merge" else binary_auroc(X, T)
torch.cuda.synchronize()
for _ in range(10):
    merged_areas(xs, ts, None, roc=True, pr=False) if which == "merge" else binary_auroc(X, T)
torch.cuda.synchronize()
print("done", which)
