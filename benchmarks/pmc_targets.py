"""Fixed workload for rocprofv3 PMC counter runs: each hot native kernel at its BASELINE shape,
20 dispatches each (after warm-up), so per-kernel counter rows are easy to aggregate.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace --output-format csv -d DIR -- python3 benchmarks/pmc_targets.py

``PMC_ONLY=<substring>`` restricts the run to matching workloads.
"""

import os
import sys

import torch

os.environ.setdefault("TORCHEVAL_AMD_FID_STAGE_ROWS", "0")  # K8 once per FID update (no staging)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd import metrics as M  # noqa: E402
from torcheval_amd.metrics import functional as F  # noqa: E402
from torcheval_amd.metrics.image.fid import FrechetInceptionDistance  # noqa: E402

REPS = 20


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    work = []
    x = torch.randn(8192, 1000, device=dev, generator=g)
    y = torch.randint(0, 1000, (8192,), device=dev, generator=g)
    acc = M.MulticlassAccuracy(device=dev)
    work.append(("K1 accuracy 8192x1000", lambda: acc.update(x, y)))
    conf = M.MulticlassConfusionMatrix(1000, device=dev)
    work.append(("K1 confusion 8192x1000", lambda: conf.update(x, y)))
    t = (torch.rand(8192, 1000, device=dev, generator=g) < 0.5).long()
    ml = M.MultilabelAccuracy(criteria="hamming", device=dev)
    work.append(("K2 multilabel hamming", lambda: ml.update(x, t)))
    s = torch.rand(1_000_000, device=dev, generator=g)
    lab = torch.randint(0, 2, (1_000_000,), device=dev, generator=g)
    work.append(("K3a+K3 binary_auroc 1M", lambda: F.binary_auroc(s, lab)))
    bin_m = M.BinaryBinnedAUPRC(threshold=200, device=dev)
    work.append(("K4 binned 1M T=200", lambda: bin_m.update(s, lab)))
    xr, yr = torch.rand(8192, 1000, device=dev, generator=g), torch.rand(8192, 1000, device=dev, generator=g)
    work.append(("K5 mse 8192x1000", lambda: F.mean_squared_error(xr, yr)))
    logits = torch.randn(4, 1024, 32000, device=dev, generator=g)
    tok = torch.randint(0, 32000, (4, 1024), device=dev, generator=g)
    ppl = M.Perplexity(device=dev)
    work.append(("K7 perplexity 4x1024x32000", lambda: ppl.update(logits, tok)))
    act = torch.randn(1000, 2048, device=dev, generator=g)
    fid = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=dev)
    work.append(("K8 fid cov 1000x2048", lambda: fid.update_activations(act, True)))
    act50k = torch.randn(50_000, 2048, device=dev, generator=g)
    work.append(("K8 fid cov 50000x2048", lambda: fid.update_activations(act50k, False)))
    xm = torch.rand(100_000, 100, device=dev, generator=g)
    ym = torch.randint(0, 100, (100_000,), device=dev, generator=g)
    mb = M.MulticlassBinnedAUPRC(num_classes=100, threshold=100, device=dev)
    work.append(("K4 dense multiclass 100k x 100 T=100", lambda: mb.update(xm, ym)))
    xs = torch.rand(8192, 1000, device=dev, generator=g)
    ts = torch.rand(8192, 1000, device=dev, generator=g)
    msum = M.Sum(device=dev)
    work.append(("K5b sum 8192x1000", lambda: msum.update(xs)))
    mpsnr = M.PeakSignalNoiseRatio(device=dev)
    work.append(("K5b psnr 8192x1000", lambda: mpsnr.update(xs, ts)))
    clicks = (torch.rand(64, 128000, device=dev, generator=g) < 0.3).float()
    wts = torch.rand(64, 128000, device=dev, generator=g)
    mctr = M.ClickThroughRate(num_tasks=64, device=dev)
    work.append(("K5b ctr 64x128000", lambda: mctr.update(clicks, wts)))
    work.append(("K4b multiclass binned auroc 100k x 100 T=200",
                 lambda: F.multiclass_binned_auroc(xm, ym, num_classes=100, threshold=200)))
    xo = torch.rand(8192, 1001, device=dev, generator=g)
    yo = torch.rand(8192, 1001, device=dev, generator=g)
    work.append(("K5 mse 8192x1001", lambda: F.mean_squared_error(xo, yo)))
    only = os.environ.get("PMC_ONLY")
    if only:
        work = [w for w in work if only in w[0]]
    for name, fn in work:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        for _ in range(REPS):
            fn()
        torch.cuda.synchronize()
        print("done", name, flush=True)


if __name__ == "__main__":
    main()
