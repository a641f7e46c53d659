"""Small-batch CPU updates (bs = 8): torcheval_amd (host twins) vs the reference itself, same
process, same tensors.  The reference is loaded read-only from /root/reference through the
parity import shims; rows print as JSON.

    python benchmarks/cpu_small_batch.py [--out profiles/cpu_small_batch.json]
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

import _refload  # noqa: E402

from torcheval_amd import metrics as M  # noqa: E402


def per_call_us(fn, iters=20000):
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
    RM, _ = _refload.load()
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
    rows = []
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
