"""Per-config benchmark suite for the BASELINE.md table on ONE MI355X.

Every row runs twice on the same GPU and the same tensors:
  * ``native``  - the framework's HIP/CDNA4 kernels (the default path);
  * ``aten``    - the same metric with ``TORCHEVAL_AMD_DISABLE_HIP`` semantics, i.e. the eager
                  ATen op chains (the reference's execution model) on the GPU.
The CPU numbers of the reference itself are in BASELINE.md and are quoted per row.

Usage: python benchmarks/bench_suite.py [--only NAME] [--out profiles/bench_suite.json]
       python benchmarks/bench_suite.py --smoke      (tiny shapes on CPU: plumbing check)
"""

import argparse
import re
import json
import os
import sys
import time
from typing import Callable, Dict, List, Optional

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torcheval_amd.ops as ops  # noqa: E402
from torcheval_amd import metrics as M  # noqa: E402
from torcheval_amd.metrics import functional as F  # noqa: E402

# BASELINE.md "measured here" reference numbers (8-core CPU), ms per call
REF_CPU_MS = {
    "multiclass_accuracy functional bs=8 C=6": 1000 / 42013,
    "MulticlassAccuracy.update bs=8 C=6": None,
    "MulticlassAccuracy.update micro bs8192 C1000": 1000 / 351,
    "MulticlassAccuracy.update macro bs8192 C1000": 1000 / 423,
    "MulticlassConfusionMatrix(1000).update bs8192": 1000 / 224,
    "binary_auroc N=1M": 124.0,
    "BinaryAUROC.update+compute N=1M": 132.0,
    "binary_binned_auroc N=1M T=200": 730.0,
    "binary_binned_precision_recall_curve N=1M T=100": 12.4,
    "BinaryBinnedAUPRC(200).update N=1M": 13.5,
    "multiclass_auroc N=100k C=100": 637.0,
    "multiclass_auprc N=100k C=100": 668.0,
    "MulticlassBinnedAUPRC(C=100,T=100).update N=100k": 200.0,
    "MultilabelAccuracy(hamming).update 8192x1000": 29.3,
    "topk_multilabel_accuracy 8192x1000": 12.9,
    "perplexity (4,1024,32000)": 123.0,
    "mean_squared_error 8192x1000": 6.7,
    "r2_score 8192x1000": 15.7,
    "FID update 1000x2048 activations": 1570.0 / 100,
    "FID compute D=2048": 2850.0,
}


def _time(fn: Callable[[], object], dev: torch.device, min_time: float, max_iters: int) -> float:
    fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    # calibrate
    t0 = time.perf_counter()
    fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    one = max(time.perf_counter() - t0, 1e-6)
    iters = int(max(3, min(max_iters, min_time / one)))
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def cases(dev: torch.device, s: float) -> Dict[str, Callable[[], Callable[[], object]]]:
    """name -> factory returning a zero-arg callable; ``s`` scales sizes (1.0 = BASELINE)."""
    g = torch.Generator(device=dev).manual_seed(0)

    def n(x: int) -> int:
        return max(8, int(x * s))

    def rand(*shape):
        return torch.rand(*shape, device=dev, generator=g)

    def randint(hi, *shape):
        return torch.randint(0, hi, shape, device=dev, generator=g)

    B, C = n(8192), 1000 if s >= 1 else 10

    def acc(avg):
        def make():
            x, y = torch.randn(B, C, device=dev, generator=g), randint(C, B)
            m = M.MulticlassAccuracy(average=avg, num_classes=C, device=dev)
            return lambda: m.update(x, y)
        return make

    def confusion():
        x, y = torch.randn(B, C, device=dev, generator=g), randint(C, B)
        m = M.MulticlassConfusionMatrix(C, device=dev)
        return lambda: m.update(x, y)

    N1M = n(1_000_000)

    def bauroc():
        x, y = rand(N1M), randint(2, N1M)
        return lambda: F.binary_auroc(x, y)

    def bauroc_cls():
        x, y = rand(N1M), randint(2, N1M)

        def run():
            m = M.BinaryAUROC(device=dev)
            m.update(x, y)
            return m.compute()
        return run

    def binned_auroc():
        x, y = rand(N1M), randint(2, N1M)
        return lambda: F.binary_binned_auroc(x, y, threshold=200)

    def binned_prc():
        x, y = rand(N1M), randint(2, N1M)
        return lambda: F.binary_binned_precision_recall_curve(x, y, threshold=100)

    def binned_auprc_cls():
        x, y = rand(N1M), randint(2, N1M)
        m = M.BinaryBinnedAUPRC(threshold=200, device=dev)
        return lambda: m.update(x, y)

    def bprc():
        x, y = rand(N1M), randint(2, N1M)
        return lambda: F.binary_precision_recall_curve(x, y)

    def brafp():
        x, y = rand(N1M), randint(2, N1M)
        return lambda: F.binary_recall_at_fixed_precision(x, y, min_precision=0.5)

    N100k, C100 = n(100_000), 100 if s >= 1 else 5

    def mlprc():
        x, y = rand(N100k, C100), randint(2, N100k, C100)
        return lambda: F.multilabel_precision_recall_curve(x, y, num_labels=C100)

    def mlrafp():
        x, y = rand(N100k, C100), randint(2, N100k, C100)
        return lambda: F.multilabel_recall_at_fixed_precision(x, y, num_labels=C100, min_precision=0.5)

    def mcprc():
        x, y = rand(N100k, C100), randint(C100, N100k)
        return lambda: F.multiclass_precision_recall_curve(x, y, num_classes=C100)

    def mc_auroc():
        x, y = rand(N100k, C100), randint(C100, N100k)
        return lambda: F.multiclass_auroc(x, y, num_classes=C100)

    def mc_auprc():
        x, y = rand(N100k, C100), randint(C100, N100k)
        return lambda: F.multiclass_auprc(x, y, num_classes=C100)

    def mc_binned_auroc():
        # the reference-default (per-sample) multiclass binned AUROC: K4b
        x, y = rand(N100k, C100), randint(C100, N100k)
        return lambda: F.multiclass_binned_auroc(x, y, num_classes=C100, threshold=200)

    def mc_binned_auprc_cls():
        x, y = rand(N100k, C100), randint(C100, N100k)
        m = M.MulticlassBinnedAUPRC(num_classes=C100, threshold=100, device=dev)
        return lambda: m.update(x, y)

    def ml_hamming():
        x, y = rand(B, C), randint(2, B, C)
        m = M.MultilabelAccuracy(criteria="hamming", device=dev)
        return lambda: m.update(x, y)

    def topk_ml():
        x, y = rand(B, C), randint(2, B, C)
        return lambda: F.topk_multilabel_accuracy(x, y, k=2)

    def rr():
        x, y = rand(B, C), randint(C, B)
        return lambda: F.reciprocal_rank(x, y, k=10)

    def hr():
        x, y = rand(B, C), randint(C, B)
        m = M.HitRate(k=10, device=dev)

        def step():
            m.update(x, y)
            if len(m.scores) > 256:  # bound the sample list over long timing loops
                m.scores.clear()

        return step

    def ppl():
        V = 32000 if s >= 1 else 50
        x, y = torch.randn(4, n(1024), V, device=dev, generator=g), randint(V, 4, n(1024))
        return lambda: F.perplexity(x, y)

    def mse():
        x, y = rand(B, C), rand(B, C)
        return lambda: F.mean_squared_error(x, y)

    def r2():
        x, y = rand(B, C), rand(B, C)
        return lambda: F.r2_score(x, y)

    D = 2048 if s >= 1 else 64

    def k5b(cls, kind):
        def make():
            x = rand(B, C)
            if kind == "sum":
                m = cls(device=dev)
                return lambda: m.update(x)
            if kind == "psnr":
                t = rand(B, C)
                m = cls(device=dev)
                return lambda: m.update(x, t)
            clicks = (rand(64, B * C // 64) < 0.3).float()
            w = rand(64, B * C // 64)
            m = cls(num_tasks=64, device=dev)
            if kind == "ctr":
                return lambda: m.update(clicks, w)
            return lambda: m.update(w, clicks, w)
        return make

    def rp_queries():
        Q = 1000 if s >= 1 else 10
        x, y, q = rand(N1M), randint(2, N1M), randint(Q, N1M)

        def run():
            m = M.RetrievalPrecision(k=10, num_queries=Q, device=dev)
            m.update(x, y, indexes=q)
            return m.compute()
        return run

    def fid_50k():
        # BASELINE config 5 shape: activations streamed into FID's covariance states in batches
        # of 1000 (50 updates = 50k x 2048), real and fake
        d = 2048 if s >= 1 else 16
        acts = [torch.randn(1000 if s >= 1 else 8, d, device=dev, generator=g) for _ in range(4)]
        m = M.FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=d, device=dev)

        def run():
            for i in range(50):
                m.update_activations(acts[i % 4], i % 2 == 0)
            m.real_cov_sum, m.fake_cov_sum  # reading the states folds the staged rows in (K8)
        return run

    def merge_runs():
        # the receiver side of a sorted-run sync: 8 ranks x 1M samples (K3m merge + K3 scan)
        from torcheval_amd.metrics.functional.classification._curve import merged_areas, sort_run

        R, per = (8, n(1_000_000))
        runs = [sort_run(rand(per), randint(2, per), None) for _ in range(R)]
        return lambda: merged_areas([r[0] for r in runs], [r[1] for r in runs], None, roc=True, pr=False)

    def union_auroc():
        x, y = rand(8 * n(1_000_000)), randint(2, 8 * n(1_000_000))
        return lambda: F.binary_auroc(x, y)

    def fid_update():
        from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

        act = torch.randn(n(1000), D, device=dev, generator=g)
        m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D, device=dev)
        return lambda: m.update_activations(act, True)

    def fid_compute():
        from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

        m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D, device=dev)
        for real in (True, False):
            m.update_activations(torch.randn(4 * D, D, device=dev, generator=g) * (1.0 if real else 1.1), real)
        return m.compute

    def fid_compute_singular():
        # 1000 real + 1000 fake activations at D = 2048: both covariances singular (rank <= 999),
        # so no Cholesky exists - K9p pivoted Cholesky + K9b on the r x r W S2 W^T
        from torcheval_amd.metrics.image.fid import FrechetInceptionDistance

        m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=D, device=dev)
        for real in (True, False):
            m.update_activations(torch.randn(n(1000), D, device=dev, generator=g) * (1.0 if real else 1.1), real)
        return m.compute

    def small_functional():
        x, y = torch.randn(8, 6, device=dev, generator=g), randint(6, 8)
        return lambda: F.multiclass_accuracy(x, y)

    def small_class():
        x, y = torch.randn(8, 6, device=dev, generator=g), randint(6, 8)
        m = M.MulticlassAccuracy(device=dev)
        return lambda: m.update(x, y)

    def small_graphed():
        x, y = torch.randn(8, 6, device=dev, generator=g), randint(6, 8)
        m = M.MulticlassAccuracy(device=dev)
        if dev.type != "cuda":
            return lambda: m.update(x, y)
        from torcheval_amd.utils.graphs import GraphedUpdate

        step = GraphedUpdate(m, x, y)
        return lambda: step(x, y)

    def five(bs, c):
        # a training step's classification metrics, all fed the same batch
        return [
            M.MulticlassAccuracy(num_classes=c, device=dev),
            M.MulticlassPrecision(num_classes=c, device=dev),
            M.MulticlassRecall(num_classes=c, device=dev),
            M.MulticlassF1Score(num_classes=c, device=dev),
            M.MulticlassConfusionMatrix(c, device=dev),
        ]

    def five_direct(bs, c):
        def make():
            x, y = torch.randn(bs, c, device=dev, generator=g), randint(c, bs)
            ms = five(bs, c)

            def step():
                for m in ms:
                    m.update(x, y)

            return step
        return make

    def five_graphed(bs, c):
        def make():
            x, y = torch.randn(bs, c, device=dev, generator=g), randint(c, bs)
            ms = five(bs, c)
            if dev.type != "cuda":
                return lambda: [m.update(x, y) for m in ms]
            from torcheval_amd.utils.graphs import GraphedUpdate

            step = GraphedUpdate(ms, x, y, check_speed=False)
            return lambda: step(x, y)
        return make

    return {
        "5 multiclass metrics (acc/prec/rec/F1/CM) .update bs=8 C=6": five_direct(n(8), 6),
        "5 multiclass metrics .update bs=8 C=6, one HIP graph": five_graphed(n(8), 6),
        "5 multiclass metrics .update bs8192 C1000": five_direct(B, C),
        "5 multiclass metrics .update bs8192 C1000, one HIP graph": five_graphed(B, C),
        "multiclass_accuracy functional bs=8 C=6": small_functional,
        "MulticlassAccuracy.update bs=8 C=6": small_class,
        "MulticlassAccuracy.update bs=8 C=6 HIP-graph replay": small_graphed,
        "MulticlassAccuracy.update micro bs8192 C1000": acc("micro"),
        "MulticlassAccuracy.update macro bs8192 C1000": acc("macro"),
        "MulticlassConfusionMatrix(1000).update bs8192": confusion,
        "binary_auroc N=1M": bauroc,
        "BinaryAUROC.update+compute N=1M": bauroc_cls,
        "binary_binned_auroc N=1M T=200": binned_auroc,
        "binary_binned_precision_recall_curve N=1M T=100": binned_prc,
        "BinaryBinnedAUPRC(200).update N=1M": binned_auprc_cls,
        "binary_precision_recall_curve N=1M": bprc,
        "binary_recall_at_fixed_precision N=1M p=0.5": brafp,
        "multilabel_precision_recall_curve 100k x 100": mlprc,
        "multilabel_recall_at_fixed_precision 100k x 100 p=0.5": mlrafp,
        "multiclass_precision_recall_curve N=100k C=100": mcprc,
        "multiclass_auroc N=100k C=100": mc_auroc,
        "multiclass_auprc N=100k C=100": mc_auprc,
        "MulticlassBinnedAUPRC(C=100,T=100).update N=100k": mc_binned_auprc_cls,
        "multiclass_binned_auroc N=100k C=100 T=200 (K4b)": mc_binned_auroc,
        "MultilabelAccuracy(hamming).update 8192x1000": ml_hamming,
        "topk_multilabel_accuracy 8192x1000": topk_ml,
        "reciprocal_rank 8192x1000 k=10 (K10)": rr,
        "HitRate(k=10).update 8192x1000 (K10)": hr,
        "perplexity (4,1024,32000)": ppl,
        "mean_squared_error 8192x1000": mse,
        "r2_score 8192x1000": r2,
        "Sum.update 8192x1000 (K5b)": k5b(M.Sum, "sum"),
        "Mean.update 8192x1000 (K5b)": k5b(M.Mean, "sum"),
        "PeakSignalNoiseRatio.update 8192x1000 (K5b)": k5b(M.PeakSignalNoiseRatio, "psnr"),
        "ClickThroughRate(64 tasks).update 8192x1000 (K5b)": k5b(M.ClickThroughRate, "ctr"),
        "WeightedCalibration(64 tasks).update 8192x1000 (K5b)": k5b(M.WeightedCalibration, "wc"),
        "WindowedClickThroughRate(64 tasks).update 8192x1000 (K5b)": k5b(M.WindowedClickThroughRate, "ctr"),
        "RetrievalPrecision(k=10, 1000 queries) update+compute N=1M": rp_queries,
        "sorted-run AUROC of 8 x 1M synced samples (K3m merge + K3)": merge_runs,
        "binary_auroc of the 8M union (K3a sort + K3)": union_auroc,
        "FID update 1000x2048 activations": fid_update,
        "FID 50k x 2048 activations (50 updates of 1000)": fid_50k,
        "FID compute D=2048": fid_compute,
        "FID compute D=2048, 1000+1000 activations (rank-deficient, K9p)": fid_compute_singular,
    }


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--smoke", action="store_true")
    ap.add_argument("--min-time", type=float, default=0.5)
    ap.add_argument("--no-aten", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cpu") if args.smoke else torch.device("cuda", 0)
    scale = 0.001 if args.smoke else 1.0
    rows: List[Dict[str, object]] = []
    for name, make in cases(dev, scale).items():
        if args.only and not re.search(args.only, name):
            continue
        row: Dict[str, object] = {"case": name}
        for mode in ("native", "aten"):
            if mode == "aten" and args.no_aten:
                continue
            ops.DISABLE_HIP = mode == "aten"
            try:
                fn = make()
                row[f"{mode}_ms"] = round(_time(fn, dev, args.min_time, 20000), 4)
            except Exception as e:  # report, keep going
                row[f"{mode}_ms"] = None
                row[f"{mode}_error"] = f"{type(e).__name__}: {e}"[:200]
            finally:
                ops.DISABLE_HIP = False
            if dev.type == "cuda":
                torch.cuda.empty_cache()
        ref = REF_CPU_MS.get(name)
        row["reference_cpu_ms"] = None if ref is None else round(ref, 3)
        if row.get("native_ms"):
            if row.get("aten_ms"):
                row["speedup_vs_aten_same_gpu"] = round(row["aten_ms"] / row["native_ms"], 2)
            if ref:
                row["speedup_vs_reference_cpu"] = round(ref / row["native_ms"], 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(0) if dev.type == "cuda" else "cpu", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
