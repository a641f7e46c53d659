"""Classification family (beyond accuracy) on CPU against scikit-learn / brute-force oracles,
plus the full MetricClassTester conformance suite per class
(parity: tests/metrics/classification/test_{precision,recall,f1_score,confusion_matrix,auroc,
auprc,precision_recall_curve,recall_at_fixed_precision,binned_*,normalized_entropy}.py).
The GPU suite (tests/gpu) then checks the HIP kernels against these CPU paths."""

import numpy as np
import pytest
import torch
from sklearn.metrics import (
    average_precision_score,
    confusion_matrix,
    f1_score,
    precision_recall_curve,
    precision_score,
    recall_score,
    roc_auc_score,
)

from torcheval_amd.metrics import (
    BinaryAUPRC,
    BinaryAUROC,
    BinaryBinnedAUPRC,
    BinaryBinnedAUROC,
    BinaryBinnedPrecisionRecallCurve,
    BinaryConfusionMatrix,
    BinaryF1Score,
    BinaryNormalizedEntropy,
    BinaryPrecision,
    BinaryPrecisionRecallCurve,
    BinaryRecall,
    BinaryRecallAtFixedPrecision,
    MulticlassAUPRC,
    MulticlassAUROC,
    MulticlassBinnedAUPRC,
    MulticlassBinnedPrecisionRecallCurve,
    MulticlassConfusionMatrix,
    MulticlassF1Score,
    MulticlassPrecision,
    MulticlassPrecisionRecallCurve,
    MulticlassRecall,
    MultilabelAUPRC,
    MultilabelBinnedAUPRC,
    MultilabelPrecisionRecallCurve,
)
from torcheval_amd.metrics.functional import (
    binary_auroc,
    binary_binned_auroc,
    binary_binned_precision_recall_curve,
    binary_normalized_entropy,
    binary_recall_at_fixed_precision,
    multiclass_auroc,
    multiclass_binned_auroc,
    multilabel_recall_at_fixed_precision,
)
from torcheval_amd.utils.test_utils import MetricClassTester

U, B, C = 8, 32, 4  # updates, batch, classes
F64 = torch.float64


def _mc_data(seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(U, B, C, generator=g)
    y = torch.randint(0, C, (U, B), generator=g)
    y[:, :C] = torch.arange(C)  # every class present in every update
    return x, y


class TestPrecisionRecallF1(MetricClassTester):
    def test_multiclass(self) -> None:
        x, y = _mc_data(1)
        pred, tgt = x.argmax(-1).flatten().numpy(), y.flatten().numpy()
        for avg in ("micro", "macro", "weighted", None):
            kw = dict(labels=list(range(C)), zero_division=0, average=avg)
            for cls, fn in ((MulticlassPrecision, precision_score), (MulticlassRecall, recall_score),
                            (MulticlassF1Score, f1_score)):
                expected = torch.tensor(fn(tgt, pred, **kw), dtype=torch.float32)
                m = cls(average=avg, num_classes=C)
                for i in range(U):
                    m.update(x[i], y[i])
                torch.testing.assert_close(m.compute(), expected, atol=1e-6, rtol=1e-5)

    def test_class_suites(self) -> None:
        x, y = _mc_data(2)
        pred, tgt = x.argmax(-1).flatten().numpy(), y.flatten().numpy()
        self.run_class_implementation_tests(
            metric=MulticlassPrecision(average="macro", num_classes=C),
            state_names={"num_tp", "num_fp", "num_label"},
            update_kwargs={"input": x, "target": y},
            compute_result=torch.tensor(precision_score(tgt, pred, average="macro"), dtype=torch.float32),
            atol=1e-6,
        )
        self.run_class_implementation_tests(
            metric=MulticlassRecall(average="macro", num_classes=C),
            state_names={"num_tp", "num_labels", "num_predictions"},
            update_kwargs={"input": x, "target": y},
            compute_result=torch.tensor(recall_score(tgt, pred, average="macro"), dtype=torch.float32),
            atol=1e-6,
        )
        self.run_class_implementation_tests(
            metric=MulticlassF1Score(average="weighted", num_classes=C),
            state_names={"num_tp", "num_label", "num_prediction"},
            update_kwargs={"input": x, "target": y},
            compute_result=torch.tensor(f1_score(tgt, pred, average="weighted"), dtype=torch.float32),
            atol=1e-6,
        )

    def test_binary(self) -> None:
        g = torch.Generator().manual_seed(3)
        x, t = torch.rand(U, B, generator=g), torch.randint(0, 2, (U, B), generator=g)
        pred, tgt = (x >= 0.4).long().flatten().numpy(), t.flatten().numpy()
        for cls, fn, names in (
            (BinaryPrecision, precision_score, {"num_tp", "num_fp", "num_label"}),
            (BinaryRecall, recall_score, {"num_tp", "num_true_labels"}),
            (BinaryF1Score, f1_score, {"num_tp", "num_label", "num_prediction"}),
        ):
            self.run_class_implementation_tests(
                metric=cls(threshold=0.4),
                state_names=names,
                update_kwargs={"input": x, "target": t},
                compute_result=torch.tensor(fn(tgt, pred), dtype=torch.float32),
                atol=1e-6,
            )


class TestConfusionMatrix(MetricClassTester):
    def test_multiclass(self) -> None:
        x, y = _mc_data(4)
        for normalize in (None, "true", "pred", "all"):
            cm = confusion_matrix(y.flatten().numpy(), x.argmax(-1).flatten().numpy(), labels=list(range(C)),
                                  normalize=normalize)
            self.run_class_implementation_tests(
                metric=MulticlassConfusionMatrix(C, normalize=normalize),
                state_names={"confusion_matrix"},
                update_kwargs={"input": x, "target": y},
                compute_result=torch.tensor(cm, dtype=torch.float32),
                atol=1e-6,
            )

    def test_binary(self) -> None:
        g = torch.Generator().manual_seed(5)
        x, t = torch.rand(U, B, generator=g), torch.randint(0, 2, (U, B), generator=g)
        cm = confusion_matrix(t.flatten().numpy(), (x >= 0.5).long().flatten().numpy(), labels=[0, 1])
        self.run_class_implementation_tests(
            metric=BinaryConfusionMatrix(),
            state_names={"confusion_matrix"},
            update_kwargs={"input": x, "target": t},
            compute_result=torch.tensor(cm, dtype=torch.float32),
        )


class TestAUROCAUPRC(MetricClassTester):
    def test_binary_auroc_ties_and_weights(self) -> None:
        g = torch.Generator().manual_seed(6)
        x = torch.randint(0, 20, (U, B), generator=g).float() / 20  # many ties
        t = torch.randint(0, 2, (U, B), generator=g)
        w = torch.rand(U, B, generator=g)
        ref = roc_auc_score(t.flatten().numpy(), x.flatten().numpy(), sample_weight=w.flatten().numpy())
        torch.testing.assert_close(binary_auroc(x.flatten(), t.flatten(), weight=w.flatten()), torch.tensor(ref, dtype=F64))
        self.run_class_implementation_tests(
            metric=BinaryAUROC(),
            state_names={"inputs", "targets", "weights"},
            update_kwargs={"input": x, "target": t},
            compute_result=torch.tensor(roc_auc_score(t.flatten().numpy(), x.flatten().numpy()), dtype=F64),
        )

    def test_multiclass_auroc(self) -> None:
        x, y = _mc_data(7)
        X, Y = x.reshape(-1, C), y.flatten()
        per = [roc_auc_score((Y == c).numpy(), X[:, c].numpy()) for c in range(C)]
        torch.testing.assert_close(multiclass_auroc(X, Y, num_classes=C, average=None), torch.tensor(per, dtype=F64).float(), atol=1e-6, rtol=1e-5)
        self.run_class_implementation_tests(
            metric=MulticlassAUROC(num_classes=C),
            state_names={"inputs", "targets"},
            update_kwargs={"input": x, "target": y},
            compute_result=torch.tensor(np.mean(per), dtype=torch.float32),
            atol=1e-6,
        )

    def test_auprc_binary_multiclass_multilabel(self) -> None:
        g = torch.Generator().manual_seed(8)
        x, t = torch.rand(U, B, generator=g), torch.randint(0, 2, (U, B), generator=g)
        self.run_class_implementation_tests(
            metric=BinaryAUPRC(),
            state_names={"inputs", "targets"},
            update_kwargs={"input": x, "target": t},
            compute_result=torch.tensor(average_precision_score(t.flatten().numpy(), x.flatten().numpy()), dtype=torch.float32),
            atol=1e-6,
        )
        xm, ym = _mc_data(9)
        X, Y = xm.reshape(-1, C), ym.flatten()
        ap = [average_precision_score((Y == c).numpy(), X[:, c].numpy()) for c in range(C)]
        self.run_class_implementation_tests(
            metric=MulticlassAUPRC(num_classes=C),
            state_names={"inputs", "targets"},
            update_kwargs={"input": xm, "target": ym},
            compute_result=torch.tensor(np.mean(ap), dtype=torch.float32),
            atol=1e-6,
        )
        tl = torch.randint(0, 2, (U, B, C), generator=g)
        T = tl.reshape(-1, C)
        apl = [average_precision_score(T[:, c].numpy(), X[:, c].numpy()) for c in range(C)]
        self.run_class_implementation_tests(
            metric=MultilabelAUPRC(num_labels=C, average=None),
            state_names={"inputs", "targets"},
            update_kwargs={"input": xm, "target": tl},
            compute_result=torch.tensor(apl, dtype=torch.float32),
            atol=1e-6,
        )


class TestPRCurves(MetricClassTester):
    def test_binary_curve_matches_sklearn(self) -> None:
        g = torch.Generator().manual_seed(10)
        x, t = torch.rand(U, B, generator=g), torch.randint(0, 2, (U, B), generator=g)
        sp, sr, sth = precision_recall_curve(t.flatten().numpy(), x.flatten().numpy())
        expected = (torch.tensor(sp.copy(), dtype=torch.float32), torch.tensor(sr.copy(), dtype=torch.float32), torch.tensor(sth.copy()))
        self.run_class_implementation_tests(
            metric=BinaryPrecisionRecallCurve(),
            state_names={"inputs", "targets"},
            update_kwargs={"input": x, "target": t},
            compute_result=expected,
            atol=1e-6,
        )

    def test_multiclass_and_multilabel_curves(self) -> None:
        x, y = _mc_data(11)
        X, Y = x.reshape(-1, C), y.flatten()
        m = MulticlassPrecisionRecallCurve(num_classes=C)
        ml = MultilabelPrecisionRecallCurve(num_labels=C)
        tl = (torch.rand(U, B, C) < 0.5).long()
        for i in range(U):
            m.update(x[i], y[i])
            ml.update(x[i], tl[i])
        p, r, th = m.compute()
        pl, rl, thl = ml.compute()
        T = tl.reshape(-1, C)
        for c in range(C):
            sp, sr, sth = precision_recall_curve((Y == c).numpy(), X[:, c].numpy())
            torch.testing.assert_close(p[c], torch.tensor(sp.copy(), dtype=torch.float32), atol=1e-6, rtol=1e-5)
            torch.testing.assert_close(r[c], torch.tensor(sr.copy(), dtype=torch.float32), atol=1e-6, rtol=1e-5)
            torch.testing.assert_close(th[c], torch.tensor(sth.copy()), atol=0, rtol=0)
            sp, sr, sth = precision_recall_curve(T[:, c].numpy(), X[:, c].numpy())
            torch.testing.assert_close(pl[c], torch.tensor(sp.copy(), dtype=torch.float32), atol=1e-6, rtol=1e-5)
            torch.testing.assert_close(rl[c], torch.tensor(sr.copy(), dtype=torch.float32), atol=1e-6, rtol=1e-5)

    def test_recall_at_fixed_precision_bruteforce(self) -> None:
        g = torch.Generator().manual_seed(12)
        x, t = torch.rand(200, generator=g), torch.randint(0, 2, (200,), generator=g)
        for p_min in (0.0, 0.3, 0.5, 0.7, 0.9):
            sp, sr, sth = precision_recall_curve(t.numpy(), x.numpy())
            ok = sp[:-1] >= p_min
            best = sr[:-1][ok].max() if ok.any() else 0.0
            thr = sth[(sr[:-1] == best) & ok].max() if ok.any() else 1e6
            rec, th = binary_recall_at_fixed_precision(x, t, min_precision=p_min)
            assert float(rec) == pytest.approx(best, abs=1e-6)
            if ok.any():
                assert float(th) == pytest.approx(thr, abs=1e-7)
        xl, tl = torch.rand(100, 3, generator=g), torch.randint(0, 2, (100, 3), generator=g)
        recs, ths = multilabel_recall_at_fixed_precision(xl, tl, num_labels=3, min_precision=0.5)
        for c in range(3):
            r_c, t_c = binary_recall_at_fixed_precision(xl[:, c], tl[:, c], min_precision=0.5)
            torch.testing.assert_close(recs[c], r_c)
            torch.testing.assert_close(ths[c], t_c)
        self.run_class_implementation_tests(
            metric=BinaryRecallAtFixedPrecision(min_precision=0.5),
            state_names={"inputs", "targets"},
            update_kwargs={"input": x.reshape(8, 25), "target": t.reshape(8, 25)},
            compute_result=binary_recall_at_fixed_precision(x, t, min_precision=0.5),
        )


def _binned_counts(x, t, thr):
    tp = torch.stack([((x >= th) & (t == 1)).sum() for th in thr]).double()
    fp = torch.stack([((x >= th) & (t == 0)).sum() for th in thr]).double()
    return tp, fp, t.sum().double() - tp


class TestBinned(MetricClassTester):
    def test_binary_binned_curve_bruteforce(self) -> None:
        g = torch.Generator().manual_seed(13)
        x, t = torch.rand(U, B, generator=g), torch.randint(0, 2, (U, B), generator=g)
        thr = torch.tensor([0.0, 0.1, 0.33, 0.5, 0.8, 1.0])
        tp, fp, fn = _binned_counts(x.flatten(), t.flatten(), thr)
        prec = torch.where(tp + fp == 0, torch.ones_like(tp), tp / (tp + fp))
        rec = torch.where(tp + fn == 0, torch.zeros_like(tp), tp / (tp + fn))
        expected = (torch.cat([prec.float(), torch.ones(1)]), torch.cat([rec.float(), torch.zeros(1)]), thr)
        got = binary_binned_precision_recall_curve(x.flatten(), t.flatten(), threshold=thr)
        for a, b in zip(got, expected):
            torch.testing.assert_close(a, b, atol=1e-6, rtol=1e-5)
        self.run_class_implementation_tests(
            metric=BinaryBinnedPrecisionRecallCurve(threshold=thr),
            state_names={"num_tp", "num_fp", "num_fn"},
            update_kwargs={"input": x, "target": t},
            compute_result=expected,
            atol=1e-6,
        )
        auprc = -torch.sum((expected[1][1:] - expected[1][:-1]) * expected[0][:-1])
        self.run_class_implementation_tests(
            metric=BinaryBinnedAUPRC(threshold=thr),
            state_names={"num_tp", "num_fp", "num_fn"},
            update_kwargs={"input": x, "target": t},
            compute_result=auprc,
            atol=1e-6,
        )

    def test_binned_auroc_equals_exact_at_all_thresholds(self) -> None:
        g = torch.Generator().manual_seed(14)
        x = torch.randint(1, 40, (U, B), generator=g).float() / 40
        t = torch.randint(0, 2, (U, B), generator=g)
        thr = torch.cat([torch.zeros(1), x.flatten().unique(), torch.ones(1)]).unique()
        exact = binary_auroc(x.flatten(), t.flatten())
        auc, th = binary_binned_auroc(x.flatten(), t.flatten(), threshold=thr)
        torch.testing.assert_close(auc.double(), exact.reshape(1), atol=1e-6, rtol=1e-6)
        self.run_class_implementation_tests(
            metric=BinaryBinnedAUROC(threshold=thr),
            state_names={"inputs", "targets"},
            update_kwargs={"input": x, "target": t},
            compute_result=(auc, thr),
            atol=1e-6,
        )
        xm, ym = _mc_data(15)
        xm = (xm * 10).round() / 10
        thr_m = torch.linspace(0, 1, 11)
        aucs, _ = multiclass_binned_auroc(xm.reshape(-1, C), ym.flatten(), num_classes=C, threshold=thr_m, average=None,
                                       one_vs_rest=True)
        exact_m = multiclass_auroc(xm.reshape(-1, C), ym.flatten(), num_classes=C, average=None)
        torch.testing.assert_close(aucs.double(), exact_m.double(), atol=1e-5, rtol=1e-5)

    def test_multiclass_multilabel_binned(self) -> None:
        x, y = _mc_data(16)
        thr = torch.tensor([0.0, 0.25, 0.5, 0.75, 1.0])
        X, Y = x.reshape(-1, C), y.flatten()
        precs, recs = [], []
        for c in range(C):
            tp, fp, fn = _binned_counts(X[:, c], (Y == c).long(), thr)
            precs.append(torch.cat([torch.where(tp + fp == 0, torch.ones_like(tp), tp / (tp + fp)).float(), torch.ones(1)]))
            recs.append(torch.cat([torch.where(tp + fn == 0, torch.zeros_like(tp), tp / (tp + fn)).float(), torch.zeros(1)]))
        m = MulticlassBinnedPrecisionRecallCurve(num_classes=C, threshold=thr)
        for i in range(U):
            m.update(x[i], y[i])
        p, r, th = m.compute()
        for c in range(C):
            torch.testing.assert_close(p[c], precs[c], atol=1e-6, rtol=1e-5)
            torch.testing.assert_close(r[c], recs[c], atol=1e-6, rtol=1e-5)
        auprc = torch.stack([-torch.sum((recs[c][1:] - recs[c][:-1]) * precs[c][:-1]) for c in range(C)])
        self.run_class_implementation_tests(
            metric=MulticlassBinnedAUPRC(num_classes=C, threshold=thr, average=None),
            state_names={"num_tp", "num_fp", "num_fn"},
            update_kwargs={"input": x, "target": y},
            compute_result=auprc,
            atol=1e-6,
        )
        tl = (torch.rand(U, B, C, generator=torch.Generator().manual_seed(17)) < 0.5).long()
        T = tl.reshape(-1, C)
        apl = []
        for c in range(C):
            tp, fp, fn = _binned_counts(X[:, c], T[:, c], thr)
            pr = torch.cat([torch.where(tp + fp == 0, torch.ones_like(tp), tp / (tp + fp)).float(), torch.ones(1)])
            rc = torch.cat([torch.where(tp + fn == 0, torch.zeros_like(tp), tp / (tp + fn)).float(), torch.zeros(1)])
            apl.append(-torch.sum((rc[1:] - rc[:-1]) * pr[:-1]))
        self.run_class_implementation_tests(
            metric=MultilabelBinnedAUPRC(num_labels=C, threshold=thr),
            state_names={"num_tp", "num_fp", "num_fn"},
            update_kwargs={"input": x, "target": tl},
            compute_result=torch.stack(apl).mean(),
            atol=1e-6,
        )


class TestNormalizedEntropy(MetricClassTester):
    def test_against_formula(self) -> None:
        g = torch.Generator().manual_seed(18)
        x = torch.rand(U, 2, B, generator=g).clamp(1e-4, 1 - 1e-4)
        t = torch.randint(0, 2, (U, 2, B), generator=g).float()
        X, T = x.permute(1, 0, 2).reshape(2, -1).double(), t.permute(1, 0, 2).reshape(2, -1).double()
        ce = -(T * X.log() + (1 - T) * (1 - X).log()).mean(-1)
        p = T.mean(-1)
        base = -(p * p.log() + (1 - p) * (1 - p).log())
        expected = ce / base
        torch.testing.assert_close(binary_normalized_entropy(X, T, num_tasks=2), expected)
        self.run_class_implementation_tests(
            metric=BinaryNormalizedEntropy(num_tasks=2),
            state_names={"total_entropy", "num_examples", "num_positive"},
            update_kwargs={"input": x, "target": t},
            compute_result=expected,
            atol=1e-6,
        )
        logits = torch.logit(X)
        torch.testing.assert_close(binary_normalized_entropy(logits, T, num_tasks=2, from_logits=True), expected, atol=1e-6, rtol=1e-6)
