"""The reference itself (Connor-Guo/torcheval, pure Python over ATen) on the same MI355X, same
tensors, same timing loop as torcheval_amd - the baseline BASELINE.md §2 asks for ("re-run
with device='cuda' ... that is the number the new framework must beat").

The reference source is not part of this repository.  For a GPU run it is staged read-only
into the git-ignored ``.ref_snapshot/`` (``cp -r /root/reference/torcheval .ref_snapshot/``)
and loaded through the import shims of ``tests/parity/_refload.py``.

    python benchmarks/reference_on_gpu.py [--out profiles/reference_on_mi355x.json]
"""

import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "parity"))
os.environ.setdefault("TORCHEVAL_REFERENCE", os.path.join(REPO, ".ref_snapshot"))

import _refload  # noqa: E402

from torcheval_amd import metrics as M  # noqa: E402
from torcheval_amd.metrics import functional as F  # noqa: E402


def rate(fn, iters, warm=5):
    """ms per call: warm-up, then ``iters`` calls bracketed by device syncs."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


class _Feats(torch.nn.Module):
    """FID feature model stand-in: returns fixed activations (the covariance update is timed,
    not Inception-v3, whose weights cannot be fetched here)."""

    def __init__(self, act):
        super().__init__()
        self.act = act

    def forward(self, x):
        return self.act


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    RM, RF = _refload.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    rows = []

    def case(name, ours, ref, iters):
        o = rate(ours, iters)
        r = rate(ref, max(3, iters // 10))
        rows.append({"case": name, "torcheval_amd_ms": round(o, 4), "reference_same_gpu_ms": round(r, 4),
                     "speedup": round(r / o, 2)})
        print(json.dumps(rows[-1]), flush=True)

    # north star: MulticlassAccuracy bs=8192, C=1000, 8-batch pool (262 MB > the 256 MiB MALL)
    xs = [torch.randn(8192, 1000, device=dev, generator=g) for _ in range(8)]
    ys = [torch.randint(0, 1000, (8192,), device=dev, generator=g) for _ in range(8)]
    for avg in ("micro", "macro"):
        kw = {"average": avg, "num_classes": 1000}
        mo, mr = M.MulticlassAccuracy(device=dev, **kw), RM.MulticlassAccuracy(device=dev, **kw)
        it = {"i": 0}

        def step(m):
            i = it["i"] = (it["i"] + 1) % 8
            m.update(xs[i], ys[i])

        case(f"MulticlassAccuracy.update {avg} bs8192 C1000", lambda: step(mo), lambda: step(mr), 2000)
    co, cr = M.MulticlassConfusionMatrix(1000, device=dev), RM.MulticlassConfusionMatrix(1000, device=dev)
    case("MulticlassConfusionMatrix(1000).update bs8192", lambda: co.update(xs[0], ys[0]),
         lambda: cr.update(xs[0], ys[0]), 500)

    s = torch.rand(1_000_000, device=dev, generator=g)
    t = torch.randint(0, 2, (1_000_000,), device=dev, generator=g)
    case("binary_auroc N=1M", lambda: F.binary_auroc(s, t), lambda: RF.binary_auroc(s, t), 100)

    def auroc_class(mod):
        m = mod.BinaryAUROC(device=dev)
        m.update(s, t)
        return m.compute()

    case("BinaryAUROC.update+compute N=1M", lambda: auroc_class(M), lambda: auroc_class(RM), 100)
    case("binary_binned_auroc N=1M T=200", lambda: F.binary_binned_auroc(s, t, threshold=200),
         lambda: RF.binary_binned_auroc(s, t, threshold=200), 100)
    bo, br = M.BinaryBinnedAUPRC(threshold=200, device=dev), RM.BinaryBinnedAUPRC(threshold=200, device=dev)
    case("BinaryBinnedAUPRC(200).update N=1M", lambda: bo.update(s, t), lambda: br.update(s, t), 200)

    # K3c: PR curves / recall at fixed precision (the reference loops labels in Python)
    case("binary_precision_recall_curve N=1M", lambda: F.binary_precision_recall_curve(s, t),
         lambda: RF.binary_precision_recall_curve(s, t), 50)
    case("binary_recall_at_fixed_precision N=1M p=0.5",
         lambda: F.binary_recall_at_fixed_precision(s, t, min_precision=0.5),
         lambda: RF.binary_recall_at_fixed_precision(s, t, min_precision=0.5), 50)
    xl = torch.rand(100_000, 100, device=dev, generator=g)
    tl = torch.randint(0, 2, (100_000, 100), device=dev, generator=g)
    case("multilabel_precision_recall_curve 100k x 100", lambda: F.multilabel_precision_recall_curve(xl, tl, num_labels=100),
         lambda: RF.multilabel_precision_recall_curve(xl, tl, num_labels=100), 10)
    case("multilabel_recall_at_fixed_precision 100k x 100 p=0.5",
         lambda: F.multilabel_recall_at_fixed_precision(xl, tl, num_labels=100, min_precision=0.5),
         lambda: RF.multilabel_recall_at_fixed_precision(xl, tl, num_labels=100, min_precision=0.5), 10)
    del xl, tl

    qidx = torch.randint(0, 1000, (1_000_000,), device=dev, generator=g)

    def rp_run(mod):
        # the reference creates its list states on the CPU whatever `device` says (.to() moves
        # them), and its compute() fails on a GPU (it cats CPU NaN placeholders with device
        # results), so the comparison times update() only
        m = mod.RetrievalPrecision(k=10, num_queries=1000, device=dev).to(dev)
        m.update(s, t, indexes=qidx)
        return m

    case("RetrievalPrecision(k=10, 1000 queries).update N=1M", lambda: rp_run(M), lambda: rp_run(RM), 20)

    xm = torch.rand(100_000, 100, device=dev, generator=g)
    ym = torch.randint(0, 100, (100_000,), device=dev, generator=g)
    case("multiclass_auroc N=100k C=100", lambda: F.multiclass_auroc(xm, ym, num_classes=100),
         lambda: RF.multiclass_auroc(xm, ym, num_classes=100), 20)
    case("multiclass_precision_recall_curve N=100k C=100",
         lambda: F.multiclass_precision_recall_curve(xm, ym, num_classes=100),
         lambda: RF.multiclass_precision_recall_curve(xm, ym, num_classes=100), 10)
    mbo = M.MulticlassBinnedAUPRC(num_classes=100, threshold=100, device=dev)
    mbr = RM.MulticlassBinnedAUPRC(num_classes=100, threshold=100, device=dev)
    case("MulticlassBinnedAUPRC(C=100,T=100).update N=100k", lambda: mbo.update(xm, ym),
         lambda: mbr.update(xm, ym), 100)

    ml = (torch.rand(8192, 1000, device=dev, generator=g) < 0.5).long()
    mlo, mlr = M.MultilabelAccuracy(criteria="hamming", device=dev), RM.MultilabelAccuracy(criteria="hamming", device=dev)
    case("MultilabelAccuracy(hamming).update 8192x1000", lambda: mlo.update(xs[1], ml), lambda: mlr.update(xs[1], ml), 200)
    case("topk_multilabel_accuracy 8192x1000 k=2", lambda: F.topk_multilabel_accuracy(xs[1], ml, k=2),
         lambda: RF.topk_multilabel_accuracy(xs[1], ml, k=2), 200)

    logits = torch.randn(4, 1024, 32000, device=dev, generator=g)
    tok = torch.randint(0, 32000, (4, 1024), device=dev, generator=g)
    case("perplexity (4,1024,32000)", lambda: F.perplexity(logits, tok), lambda: RF.perplexity(logits, tok), 50)
    del logits
    xr, yr = torch.rand(8192, 1000, device=dev, generator=g), torch.rand(8192, 1000, device=dev, generator=g)
    case("mean_squared_error 8192x1000", lambda: F.mean_squared_error(xr, yr), lambda: RF.mean_squared_error(xr, yr), 200)
    case("r2_score 8192x1000", lambda: F.r2_score(xr, yr), lambda: RF.r2_score(xr, yr), 200)

    act = torch.randn(1000, 2048, device=dev, generator=g)
    imgs = torch.zeros(1000, 3, 1, 1, device=dev)
    fo = M.FrechetInceptionDistance(model=_Feats(act), feature_dim=2048, device=dev)
    fr = RM.FrechetInceptionDistance(model=_Feats(act), feature_dim=2048, device=dev)
    case("FrechetInceptionDistance.update 1000x2048 activations", lambda: fo.update(imgs, True),
         lambda: fr.update(imgs, True), 100)
    fo.update(imgs, False)
    fr.update(imgs, False)
    case("FrechetInceptionDistance.compute D=2048", lambda: fo.compute(), lambda: fr.compute(), 5)

    out = {"device": torch.cuda.get_device_name(0), "torch": torch.__version__, "rows": rows}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
