"""Small-batch CPU updates (bs = 8): torcheval_amd (host twins) vs the reference itself, same
process, same tensors.  The reference is loaded read-only from /root/reference through the
parity import shims; rows print as JSON.

    python benchmarks/cpu_small_batch.py [--out profiles/cpu_small_batch.json]
"""

import argparse
import logging
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "parity"))

import _refload  # noqa: E402

from torcheval_amd import metrics as M  # noqa: E402
from torcheval_amd.metrics import functional as F_ours  # noqa: E402


def per_call_us(fn, iters=20000):
    import warnings

    warnings.simplefilter("ignore")
    for _ in range(500):
        fn()
    best = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    torch.set_num_threads(1)
    RM, RF = _refload.load()
    logging.disable(logging.WARNING)  # both libraries warn on absent classes; keep logging out of the timings
    g = torch.Generator().manual_seed(0)
    x, t = torch.rand(8, generator=g), torch.rand(8, generator=g)
    w = torch.rand(8, generator=g)
    x2, t2 = torch.rand(8, 4, generator=g), torch.rand(8, 4, generator=g)
    clicks = (torch.rand(8, generator=g) < 0.3).float()
    img_x, img_t = torch.rand(2, 3, 2, 2, generator=g), torch.rand(2, 3, 2, 2, generator=g)
    cases = [
        ("Mean.update bs=8", lambda m: m.update(x), "Mean", {}),
        ("Mean.update weighted bs=8", lambda m: m.update(x, weight=w), "Mean", {}),
        ("Sum.update bs=8", lambda m: m.update(x), "Sum", {}),
        ("ClickThroughRate.update bs=8", lambda m: m.update(clicks, w), "ClickThroughRate", {}),
        ("WeightedCalibration.update bs=8", lambda m: m.update(x, t), "WeightedCalibration", {}),
        ("PeakSignalNoiseRatio.update 2x3x2x2", lambda m: m.update(img_x, img_t), "PeakSignalNoiseRatio", {}),
        ("WindowedClickThroughRate.update bs=8", lambda m: m.update(clicks, w), "WindowedClickThroughRate", {}),
        ("WindowedWeightedCalibration.update bs=8", lambda m: m.update(x, t), "WindowedWeightedCalibration", {}),
        ("MeanSquaredError.update bs=8x4", lambda m: m.update(x2, t2), "MeanSquaredError", {}),
        ("R2Score.update bs=8x4", lambda m: m.update(x2, t2), "R2Score", {}),
    ]
    # classification (BASELINE.json config 1 is the first row's shape)
    xc, yc = torch.randn(8, 6, generator=g), torch.randint(0, 6, (8,), generator=g)
    xb, yb = torch.rand(8, generator=g), torch.randint(0, 2, (8,), generator=g)
    cases += [
        ("MulticlassAccuracy.update bs=8 C=6", lambda m: m.update(xc, yc), "MulticlassAccuracy", {}),
        ("MulticlassF1Score(macro).update bs=8 C=6", lambda m: m.update(xc, yc), "MulticlassF1Score",
         {"num_classes": 6, "average": "macro"}),
        ("MulticlassConfusionMatrix(6).update bs=8", lambda m: m.update(xc, yc), "MulticlassConfusionMatrix",
         {"num_classes": 6}),
        ("BinaryAccuracy.update bs=8", lambda m: m.update(xb, yb), "BinaryAccuracy", {}),
        ("BinaryPrecision.update bs=8", lambda m: m.update(xb, yb), "BinaryPrecision", {}),
        ("BinaryRecall.update bs=8", lambda m: m.update(xb, yb), "BinaryRecall", {}),
        ("BinaryF1Score.update bs=8", lambda m: m.update(xb, yb), "BinaryF1Score", {}),
        ("BinaryAUROC.update bs=8", lambda m: m.update(xb, yb), "BinaryAUROC", {}),
        ("BinaryAUPRC.update bs=8", lambda m: m.update(xb, yb), "BinaryAUPRC", {}),
    ]
    fcases = [
        ("multiclass_accuracy bs=8 C=6", lambda F: F.multiclass_accuracy(xc, yc)),
        ("multiclass_accuracy macro bs=8 C=6", lambda F: F.multiclass_accuracy(xc, yc, average="macro", num_classes=6)),
        ("multiclass_f1_score macro bs=8 C=6", lambda F: F.multiclass_f1_score(xc, yc, num_classes=6, average="macro")),
        ("multiclass_confusion_matrix bs=8 C=6", lambda F: F.multiclass_confusion_matrix(xc, yc, num_classes=6)),
        ("binary_accuracy bs=8", lambda F: F.binary_accuracy(xb, yb)),
        ("binary_f1_score bs=8", lambda F: F.binary_f1_score(xb, yb)),
        ("binary_precision bs=8", lambda F: F.binary_precision(xb, yb)),
        ("binary_recall bs=8", lambda F: F.binary_recall(xb, yb)),
        ("binary_confusion_matrix bs=8", lambda F: F.binary_confusion_matrix(xb, yb)),
        ("binary_auroc bs=8", lambda F: F.binary_auroc(xb, yb)),
        ("binary_auprc bs=8", lambda F: F.binary_auprc(xb, yb)),
        ("mean_squared_error bs=8", lambda F: F.mean_squared_error(xb, xb * 0.5)),
        ("r2_score bs=8", lambda F: F.r2_score(xb, xb * 0.5)),
    ]
    computes = [
        ("BinaryAUROC.compute bs=8", "BinaryAUROC", {}, (xb, yb)),
        ("BinaryAUPRC.compute bs=8", "BinaryAUPRC", {}, (xb, yb)),
        ("MulticlassF1Score(macro).compute", "MulticlassF1Score", {"num_classes": 6, "average": "macro"}, (xc, yc)),
        ("MulticlassConfusionMatrix(6).compute", "MulticlassConfusionMatrix", {"num_classes": 6}, (xc, yc)),
    ]
    rows = []
    for name, fn in fcases:
        o = per_call_us(lambda: fn(F_ours), 5000)
        r = per_call_us(lambda: fn(RF), 5000)
        rows.append({"case": name, "torcheval_amd_us": round(o, 2), "reference_us": round(r, 2), "speedup": round(r / o, 2)})
        print(json.dumps(rows[-1]), flush=True)
    for name, cls, kw, args_ in computes:
        ours = getattr(M, cls)(**kw)
        ref = getattr(RM, cls)(**kw)
        ours.update(*args_)
        ref.update(*args_)
        o = per_call_us(lambda: ours.compute(), 3000)
        r = per_call_us(lambda: ref.compute(), 3000)
        rows.append({"case": name, "torcheval_amd_us": round(o, 2), "reference_us": round(r, 2), "speedup": round(r / o, 2)})
        print(json.dumps(rows[-1]), flush=True)
    for name, step, cls, kw in cases:
        ours = getattr(M, cls)(**kw)
        ref = getattr(RM, cls)(**kw)
        o = per_call_us(lambda: step(ours))
        r = per_call_us(lambda: step(ref))
        rows.append({"case": name, "torcheval_amd_us": round(o, 2), "reference_us": round(r, 2), "speedup": round(r / o, 2)})
        print(json.dumps(rows[-1]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"threads": 1, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
