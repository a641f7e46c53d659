"""Differential-parity case registry: the same inputs are fed to the reference
(torcheval @ /root/reference, via ``gen_goldens.py``) and to torcheval_amd (``test_parity.py``).

Every public functional metric and every public class metric of the reference's
``torcheval.metrics`` / ``torcheval.metrics.functional`` ``__all__`` appears here with the
option combinations its own tests exercise (averages, thresholds, num_tasks, weights, ties,
missing classes, normalisation modes, multi-update merges).

A case builder is a pure function of a seed, so goldens generated on one machine reproduce
bit-identical inputs anywhere (CPU generator, then ``.to(device)``).
"""

from typing import Any, Callable, Dict, List, Tuple

import torch

Args = Tuple[Tuple[Any, ...], Dict[str, Any]]


def _g(seed: int) -> torch.Generator:
    return torch.Generator().manual_seed(seed)


def _rand(g, *shape) -> torch.Tensor:
    return torch.rand(*shape, generator=g)


def _randn(g, *shape) -> torch.Tensor:
    return torch.randn(*shape, generator=g)


def _randint(g, lo, hi, *shape) -> torch.Tensor:
    return torch.randint(lo, hi, shape, generator=g)


def _tied(x: torch.Tensor) -> torch.Tensor:
    """Quantise scores to 1 decimal so the sort paths see many ties."""
    return torch.round(x * 10) / 10


# ----------------------------------------------------------------------------------------
# functional cases: id -> (function name, builder(seed) -> (args, kwargs))
# ----------------------------------------------------------------------------------------
FUNCTIONAL: Dict[str, Tuple[str, Callable[[int], Args]]] = {}


def fcase(case_id: str, fn: str):
    def deco(builder: Callable[[int], Args]):
        FUNCTIONAL[case_id] = (fn, builder)
        return builder

    return deco


def _add(case_id: str, fn: str, builder: Callable[[int], Args]) -> None:
    FUNCTIONAL[case_id] = (fn, builder)


N, C, L, T = 64, 5, 4, 3  # samples, classes, labels, tasks

# accuracy --------------------------------------------------------------------------------
for thr in (0.5, 0.7):
    _add(f"binary_accuracy_thr{thr}", "binary_accuracy",
         lambda s, thr=thr: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {"threshold": thr}))
_add("binary_accuracy_bool_target", "binary_accuracy",
     lambda s: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N).bool()), {}))
_add("binary_accuracy_labels", "binary_accuracy",
     lambda s: ((_randint(_g(s), 0, 2, N), _randint(_g(s + 1), 0, 2, N)), {}))
for avg in ("micro", "macro", None):
    for k in (1, 2, 3):
        _add(f"multiclass_accuracy_{avg}_k{k}", "multiclass_accuracy",
             lambda s, avg=avg, k=k: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N)),
                                      {"average": avg, "num_classes": C, "k": k}))
_add("multiclass_accuracy_labels", "multiclass_accuracy",
     lambda s: ((_randint(_g(s), 0, C, N), _randint(_g(s + 1), 0, C, N)), {}))
_add("multiclass_accuracy_missing_class_macro", "multiclass_accuracy",
     lambda s: ((_rand(_g(s), N, C + 2), _randint(_g(s + 1), 0, C, N)),
                {"average": "macro", "num_classes": C + 2}))
_add("multiclass_accuracy_missing_class_none", "multiclass_accuracy",
     lambda s: ((_rand(_g(s), N, C + 2), _randint(_g(s + 1), 0, C, N)),
                {"average": None, "num_classes": C + 2}))
for crit in ("exact_match", "hamming", "overlap", "contain", "belong"):
    for thr in (0.5, 0.3):
        _add(f"multilabel_accuracy_{crit}_thr{thr}", "multilabel_accuracy",
             lambda s, crit=crit, thr=thr: ((_rand(_g(s), N, L), _randint(_g(s + 1), 0, 2, N, L)),
                                            {"criteria": crit, "threshold": thr}))
    for k in (2, 3):
        _add(f"topk_multilabel_accuracy_{crit}_k{k}", "topk_multilabel_accuracy",
             lambda s, crit=crit, k=k: ((_rand(_g(s), N, L), _randint(_g(s + 1), 0, 2, N, L)),
                                        {"criteria": crit, "k": k}))

# precision / recall / f1 ----------------------------------------------------------------
for fam in ("precision", "recall", "f1_score"):
    for thr in (0.5, 0.8):
        _add(f"binary_{fam}_thr{thr}", f"binary_{fam}",
             lambda s, thr=thr: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {"threshold": thr}))
    _add(f"binary_{fam}_labels", f"binary_{fam}",
         lambda s: ((_randint(_g(s), 0, 2, N), _randint(_g(s + 1), 0, 2, N)), {}))
    for avg in ("micro", "macro", "weighted", None):
        _add(f"multiclass_{fam}_{avg}", f"multiclass_{fam}",
             lambda s, avg=avg: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N)),
                                 {"average": avg, "num_classes": C}))
        _add(f"multiclass_{fam}_{avg}_labels", f"multiclass_{fam}",
             lambda s, avg=avg: ((_randint(_g(s), 0, C, N), _randint(_g(s + 1), 0, C, N)),
                                 {"average": avg, "num_classes": C}))
    for avg in ("macro", "weighted", None):
        # classes C..C+1 never appear as a label; class 0 never predicted
        _add(f"multiclass_{fam}_{avg}_absent_classes", f"multiclass_{fam}",
             lambda s, avg=avg: ((_randint(_g(s), 1, C, N), _randint(_g(s + 1), 0, C - 1, N)),
                                 {"average": avg, "num_classes": C + 2}))

# confusion matrix ------------------------------------------------------------------------
for norm in (None, "pred", "true", "all"):
    _add(f"binary_confusion_matrix_{norm}", "binary_confusion_matrix",
         lambda s, norm=norm: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)),
                               {"normalize": norm, "threshold": 0.4}))
    _add(f"multiclass_confusion_matrix_{norm}", "multiclass_confusion_matrix",
         lambda s, norm=norm: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N), C),
                               {"normalize": norm}))
    _add(f"multiclass_confusion_matrix_{norm}_labels_absent", "multiclass_confusion_matrix",
         lambda s, norm=norm: ((_randint(_g(s), 0, C, N), _randint(_g(s + 1), 0, C, N), C + 1),
                               {"normalize": norm}))

# AUROC / AUPRC / curves -------------------------------------------------------------------
for tied in (False, True):
    tag = "_ties" if tied else ""
    q = _tied if tied else (lambda x: x)
    _add(f"binary_auroc{tag}", "binary_auroc",
         lambda s, q=q: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N)), {}))
    _add(f"binary_auroc_tasks{tag}", "binary_auroc",
         lambda s, q=q: ((q(_rand(_g(s), T, N)), _randint(_g(s + 1), 0, 2, T, N)), {"num_tasks": T}))
    _add(f"binary_auroc_weight{tag}", "binary_auroc",
         lambda s, q=q: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N)),
                         {"weight": _rand(_g(s + 2), N)}))
    _add(f"binary_auroc_float_target{tag}", "binary_auroc",
         lambda s, q=q: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N).float()), {}))
    for avg in ("macro", None):
        _add(f"multiclass_auroc_{avg}{tag}", "multiclass_auroc",
             lambda s, q=q, avg=avg: ((q(_rand(_g(s), N, C)), _randint(_g(s + 1), 0, C, N)),
                                      {"num_classes": C, "average": avg}))
        _add(f"multiclass_auprc_{avg}{tag}", "multiclass_auprc",
             lambda s, q=q, avg=avg: ((q(_rand(_g(s), N, C)), _randint(_g(s + 1), 0, C, N)),
                                      {"num_classes": C, "average": avg}))
        _add(f"multilabel_auprc_{avg}{tag}", "multilabel_auprc",
             lambda s, q=q, avg=avg: ((q(_rand(_g(s), N, L)), _randint(_g(s + 1), 0, 2, N, L)),
                                      {"num_labels": L, "average": avg}))
    _add(f"binary_auprc{tag}", "binary_auprc",
         lambda s, q=q: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N)), {}))
    _add(f"binary_auprc_tasks{tag}", "binary_auprc",
         lambda s, q=q: ((q(_rand(_g(s), T, N)), _randint(_g(s + 1), 0, 2, T, N)), {"num_tasks": T}))
    _add(f"binary_precision_recall_curve{tag}", "binary_precision_recall_curve",
         lambda s, q=q: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N)), {}))
    _add(f"multiclass_precision_recall_curve{tag}", "multiclass_precision_recall_curve",
         lambda s, q=q: ((q(_rand(_g(s), N, C)), _randint(_g(s + 1), 0, C, N)), {"num_classes": C}))
    _add(f"multilabel_precision_recall_curve{tag}", "multilabel_precision_recall_curve",
         lambda s, q=q: ((q(_rand(_g(s), N, L)), _randint(_g(s + 1), 0, 2, N, L)), {"num_labels": L}))
    for p in (0.0, 0.5, 0.9):
        _add(f"binary_recall_at_fixed_precision_p{p}{tag}", "binary_recall_at_fixed_precision",
             lambda s, q=q, p=p: ((q(_rand(_g(s), N)), _randint(_g(s + 1), 0, 2, N)), {"min_precision": p}))
        _add(f"multilabel_recall_at_fixed_precision_p{p}{tag}", "multilabel_recall_at_fixed_precision",
             lambda s, q=q, p=p: ((q(_rand(_g(s), N, L)), _randint(_g(s + 1), 0, 2, N, L)),
                                  {"num_labels": L, "min_precision": p}))
_add("binary_auroc_all_negative", "binary_auroc",
     lambda s: ((_rand(_g(s), N), torch.zeros(N, dtype=torch.long)), {}))
_add("binary_auprc_all_negative", "binary_auprc",
     lambda s: ((_rand(_g(s), N), torch.zeros(N, dtype=torch.long)), {}))
_add("binary_precision_recall_curve_all_negative", "binary_precision_recall_curve",
     lambda s: ((_rand(_g(s), N), torch.zeros(N, dtype=torch.long)), {}))
_add("multiclass_auroc_absent_class", "multiclass_auroc",
     lambda s: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C - 1, N)), {"num_classes": C}))
_add("multiclass_precision_recall_curve_absent_class", "multiclass_precision_recall_curve",
     lambda s: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C - 1, N)), {"num_classes": C}))

# binned family ---------------------------------------------------------------------------
_THRESHOLDS = {
    "int5": 5,
    "int100": 100,
    "list": [0.0, 0.1, 0.25, 0.5, 0.8, 1.0],
    "tensor": torch.tensor([0.0, 0.2, 0.3, 0.55, 0.9, 1.0]),
}
for tname, thr in _THRESHOLDS.items():
    _add(f"binary_binned_precision_recall_curve_{tname}", "binary_binned_precision_recall_curve",
         lambda s, thr=thr: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {"threshold": thr}))
    _add(f"binary_binned_auroc_{tname}", "binary_binned_auroc",
         lambda s, thr=thr: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {"threshold": thr}))
    _add(f"binary_binned_auprc_{tname}", "binary_binned_auprc",
         lambda s, thr=thr: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {"threshold": thr}))
    _add(f"binary_binned_auroc_tasks_{tname}", "binary_binned_auroc",
         lambda s, thr=thr: ((_rand(_g(s), T, N), _randint(_g(s + 1), 0, 2, T, N)),
                             {"threshold": thr, "num_tasks": T}))
    _add(f"binary_binned_auprc_tasks_{tname}", "binary_binned_auprc",
         lambda s, thr=thr: ((_rand(_g(s), T, N), _randint(_g(s + 1), 0, 2, T, N)),
                             {"threshold": thr, "num_tasks": T}))
    for opt in ("vectorized", "memory"):
        _add(f"multiclass_binned_precision_recall_curve_{tname}_{opt}",
             "multiclass_binned_precision_recall_curve",
             lambda s, thr=thr, opt=opt: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N)),
                                          {"num_classes": C, "threshold": thr, "optimization": opt}))
        _add(f"multilabel_binned_precision_recall_curve_{tname}_{opt}",
             "multilabel_binned_precision_recall_curve",
             lambda s, thr=thr, opt=opt: ((_rand(_g(s), N, L), _randint(_g(s + 1), 0, 2, N, L)),
                                          {"num_labels": L, "threshold": thr, "optimization": opt}))
    for avg in ("macro", None):
        _add(f"multiclass_binned_auroc_{tname}_{avg}", "multiclass_binned_auroc",
             lambda s, thr=thr, avg=avg: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N)),
                                          {"num_classes": C, "threshold": thr, "average": avg}))
        _add(f"multiclass_binned_auprc_{tname}_{avg}", "multiclass_binned_auprc",
             lambda s, thr=thr, avg=avg: ((_rand(_g(s), N, C), _randint(_g(s + 1), 0, C, N)),
                                          {"num_classes": C, "threshold": thr, "average": avg}))
        _add(f"multilabel_binned_auprc_{tname}_{avg}", "multilabel_binned_auprc",
             lambda s, thr=thr, avg=avg: ((_rand(_g(s), N, L), _randint(_g(s + 1), 0, 2, N, L)),
                                          {"num_labels": L, "threshold": thr, "average": avg}))

# normalized entropy ------------------------------------------------------------------------
for logits in (False, True):
    tag = "_logits" if logits else ""
    src = (lambda g, *sh: _randn(g, *sh) * 2) if logits else (lambda g, *sh: _rand(g, *sh) * 0.98 + 0.01)
    _add(f"binary_normalized_entropy{tag}", "binary_normalized_entropy",
         lambda s, src=src, lg=logits: ((src(_g(s), N), _randint(_g(s + 1), 0, 2, N).float()),
                                        {"from_logits": lg}))
    _add(f"binary_normalized_entropy_weight{tag}", "binary_normalized_entropy",
         lambda s, src=src, lg=logits: ((src(_g(s), N), _randint(_g(s + 1), 0, 2, N).float()),
                                        {"from_logits": lg, "weight": _rand(_g(s + 2), N)}))
    _add(f"binary_normalized_entropy_tasks{tag}", "binary_normalized_entropy",
         lambda s, src=src, lg=logits: ((src(_g(s), T, N), _randint(_g(s + 1), 0, 2, T, N).float()),
                                        {"from_logits": lg, "num_tasks": T}))

# aggregation -----------------------------------------------------------------------------
_add("sum_plain", "sum", lambda s: ((_randn(_g(s), 4, 7),), {}))
_add("sum_weight_scalar", "sum", lambda s: ((_randn(_g(s), 9),), {"weight": 0.25}))
_add("sum_weight_tensor", "sum", lambda s: ((_randn(_g(s), 9),), {"weight": _rand(_g(s + 1), 9)}))
_add("mean_plain", "mean", lambda s: ((_randn(_g(s), 4, 7),), {}))
_add("mean_weight_scalar", "mean", lambda s: ((_randn(_g(s), 9),), {"weight": 3}))
_add("mean_weight_tensor", "mean", lambda s: ((_randn(_g(s), 9),), {"weight": _rand(_g(s + 1), 9)}))
_add("throughput", "throughput", lambda s: ((1000, 2.5), {}))
_add("throughput_zero", "throughput", lambda s: ((0, 0.5), {}))
_add("auc_sorted", "auc", lambda s: ((torch.sort(_rand(_g(s), 20)).values, _rand(_g(s + 1), 20)), {}))
_add("auc_reorder", "auc", lambda s: ((_rand(_g(s), 20), _rand(_g(s + 1), 20)), {"reorder": True}))
_add("auc_tasks", "auc", lambda s: ((_rand(_g(s), 3, 20), _rand(_g(s + 1), 3, 20)), {"reorder": True}))

# regression ------------------------------------------------------------------------------
for mo in ("uniform_average", "raw_values"):
    _add(f"mean_squared_error_1d_{mo}", "mean_squared_error",
         lambda s, mo=mo: ((_randn(_g(s), N), _randn(_g(s + 1), N)), {"multioutput": mo}))
    _add(f"mean_squared_error_2d_{mo}", "mean_squared_error",
         lambda s, mo=mo: ((_randn(_g(s), N, 3), _randn(_g(s + 1), N, 3)), {"multioutput": mo}))
    _add(f"mean_squared_error_weighted_{mo}", "mean_squared_error",
         lambda s, mo=mo: ((_randn(_g(s), N, 3), _randn(_g(s + 1), N, 3)),
                           {"multioutput": mo, "sample_weight": _rand(_g(s + 2), N)}))
for mo in ("uniform_average", "raw_values", "variance_weighted"):
    _add(f"r2_score_1d_{mo}", "r2_score",
         lambda s, mo=mo: ((_randn(_g(s), N), _randn(_g(s + 1), N)), {"multioutput": mo}))
    _add(f"r2_score_2d_{mo}", "r2_score",
         lambda s, mo=mo: ((_randn(_g(s), N, 3), _randn(_g(s + 1), N, 3)), {"multioutput": mo}))
    _add(f"r2_score_adjusted_{mo}", "r2_score",
         lambda s, mo=mo: ((_randn(_g(s), N, 3), _randn(_g(s + 1), N, 3)),
                           {"multioutput": mo, "num_regressors": 4}))

# image -----------------------------------------------------------------------------------
_add("psnr_auto_range", "peak_signal_noise_ratio",
     lambda s: ((_rand(_g(s), 2, 3, 8, 8), _rand(_g(s + 1), 2, 3, 8, 8)), {}))
_add("psnr_fixed_range", "peak_signal_noise_ratio",
     lambda s: ((_rand(_g(s), 2, 3, 8, 8), _rand(_g(s + 1), 2, 3, 8, 8)), {"data_range": 2.0}))

# ranking ---------------------------------------------------------------------------------
_add("click_through_rate", "click_through_rate", lambda s: ((_randint(_g(s), 0, 2, N).float(),), {}))
_add("click_through_rate_weights", "click_through_rate",
     lambda s: ((_randint(_g(s), 0, 2, N).float(), _rand(_g(s + 1), N)), {}))
_add("click_through_rate_tasks", "click_through_rate",
     lambda s: ((_randint(_g(s), 0, 2, T, N).float(), _rand(_g(s + 1), T, N)), {"num_tasks": T}))
for k in (0.5, 1.0, 3.0):
    _add(f"frequency_at_k_{k}", "frequency_at_k", lambda s, k=k: ((_rand(_g(s), N) * 4,), {"k": k}))
for k in (None, 1, 3):
    _add(f"hit_rate_k{k}", "hit_rate",
         lambda s, k=k: ((_tied(_rand(_g(s), 16, C + 3)), _randint(_g(s + 1), 0, C + 3, 16)), {"k": k}))
    _add(f"reciprocal_rank_k{k}", "reciprocal_rank",
         lambda s, k=k: ((_tied(_rand(_g(s), 16, C + 3)), _randint(_g(s + 1), 0, C + 3, 16)), {"k": k}))
_add("num_collisions", "num_collisions", lambda s: ((_randint(_g(s), 0, 10, 40),), {}))
for k in (None, 3, 100):
    for lim in (False, True):
        _add(f"retrieval_precision_k{k}_lim{lim}", "retrieval_precision",
             lambda s, k=k, lim=lim: ((_rand(_g(s), 12), _randint(_g(s + 1), 0, 2, 12)),
                                      {"k": k, "limit_k_to_size": lim}))
_add("retrieval_precision_tasks", "retrieval_precision",
     lambda s: ((_rand(_g(s), T, 12), _randint(_g(s + 1), 0, 2, T, 12)), {"k": 4, "num_tasks": T}))
_add("weighted_calibration", "weighted_calibration",
     lambda s: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N)), {}))
_add("weighted_calibration_weight", "weighted_calibration",
     lambda s: ((_rand(_g(s), N), _randint(_g(s + 1), 0, 2, N), _rand(_g(s + 2), N)), {}))
_add("weighted_calibration_tasks", "weighted_calibration",
     lambda s: ((_rand(_g(s), T, N), _randint(_g(s + 1), 0, 2, T, N), 0.5), {"num_tasks": T}))

# text ------------------------------------------------------------------------------------
_HYP = ["the cat sat on the mat", "a quick brown fox jumps", "hello there general kenobi"]
_REF = [["the cat is sitting on the mat", "there is a cat on the mat"],
        ["the quick brown fox jumped", "a fast brown fox jumps over"],
        ["hello there general", "hi there general kenobi"]]
for n_gram in (1, 2, 3, 4):
    _add(f"bleu_score_n{n_gram}", "bleu_score", lambda s, n=n_gram: ((_HYP, _REF), {"n_gram": n}))
_add("bleu_score_weights", "bleu_score",
     lambda s: ((_HYP, _REF), {"n_gram": 2, "weights": torch.tensor([0.3, 0.7])}))
_add("bleu_score_single", "bleu_score", lambda s: ((_HYP[0], [_REF[0]]), {"n_gram": 2}))
_WER_IN = ["this is the prediction", "there is an other sample", "completely off"]
_WER_TG = ["this is the reference", "there is another one", "nothing like it at all"]
for fn in ("word_error_rate", "word_information_lost", "word_information_preserved"):
    _add(f"{fn}_list", fn, lambda s: ((_WER_IN, _WER_TG), {}))
    _add(f"{fn}_str", fn, lambda s: ((_WER_IN[1], _WER_TG[1]), {}))
_add("perplexity", "perplexity", lambda s: ((_randn(_g(s), 2, 8, 11), _randint(_g(s + 1), 0, 11, 2, 8)), {}))
_add("perplexity_ignore", "perplexity",
     lambda s: ((_randn(_g(s), 2, 8, 11), _randint(_g(s + 1), 0, 11, 2, 8)), {"ignore_index": 3}))


# ----------------------------------------------------------------------------------------
# class cases: id -> (class name, ctor kwargs builder, updates builder(seed) -> [Args])
# compute() after all updates, and after merging two halves, is compared to the reference.
# ----------------------------------------------------------------------------------------
CLASS: Dict[str, Tuple[str, Callable[[], Dict[str, Any]], Callable[[int], List[Args]]]] = {}
U = 4  # updates per case


def _ccase(case_id: str, cls: str, ctor: Callable[[], Dict[str, Any]], upd: Callable[[int], Args]) -> None:
    CLASS[case_id] = (cls, ctor, lambda s: [upd(s + 10 * i) for i in range(U)])


B = 32
for avg in ("micro", "macro", None):
    for k in (1, 2):
        _ccase(f"MulticlassAccuracy_{avg}_k{k}", "MulticlassAccuracy",
               lambda avg=avg, k=k: {"average": avg, "num_classes": C, "k": k},
               lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
_ccase("BinaryAccuracy", "BinaryAccuracy", lambda: {"threshold": 0.6},
       lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
for crit in ("exact_match", "hamming", "overlap", "contain", "belong"):
    _ccase(f"MultilabelAccuracy_{crit}", "MultilabelAccuracy", lambda crit=crit: {"criteria": crit},
           lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
    _ccase(f"TopKMultilabelAccuracy_{crit}", "TopKMultilabelAccuracy",
           lambda crit=crit: {"criteria": crit, "k": 2},
           lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
for fam in ("Precision", "Recall", "F1Score"):
    _ccase(f"Binary{fam}", f"Binary{fam}", lambda: {"threshold": 0.4},
           lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
    for avg in ("micro", "macro", "weighted", None):
        _ccase(f"Multiclass{fam}_{avg}", f"Multiclass{fam}",
               lambda avg=avg: {"average": avg, "num_classes": C},
               lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
for norm in (None, "pred", "true", "all"):
    _ccase(f"MulticlassConfusionMatrix_{norm}", "MulticlassConfusionMatrix",
           lambda norm=norm: {"num_classes": C, "normalize": norm},
           lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
    _ccase(f"BinaryConfusionMatrix_{norm}", "BinaryConfusionMatrix",
           lambda norm=norm: {"normalize": norm},
           lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
_ccase("BinaryAUROC", "BinaryAUROC", dict,
       lambda s: ((_tied(_rand(_g(s), B)), _randint(_g(s + 1), 0, 2, B)), {}))
_ccase("BinaryAUROC_tasks_weight", "BinaryAUROC", lambda: {"num_tasks": T},
       lambda s: ((_tied(_rand(_g(s), T, B)), _randint(_g(s + 1), 0, 2, T, B)),
                  {"weight": _rand(_g(s + 2), T, B)}))
_ccase("BinaryAUPRC", "BinaryAUPRC", dict,
       lambda s: ((_tied(_rand(_g(s), B)), _randint(_g(s + 1), 0, 2, B)), {}))
_ccase("BinaryAUPRC_tasks", "BinaryAUPRC", lambda: {"num_tasks": T},
       lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B)), {}))
for avg in ("macro", None):
    _ccase(f"MulticlassAUROC_{avg}", "MulticlassAUROC", lambda avg=avg: {"num_classes": C, "average": avg},
           lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
    _ccase(f"MulticlassAUPRC_{avg}", "MulticlassAUPRC", lambda avg=avg: {"num_classes": C, "average": avg},
           lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
    _ccase(f"MultilabelAUPRC_{avg}", "MultilabelAUPRC", lambda avg=avg: {"num_labels": L, "average": avg},
           lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
    _ccase(f"MulticlassBinnedAUROC_{avg}", "MulticlassBinnedAUROC",
           lambda avg=avg: {"num_classes": C, "average": avg, "threshold": 10},
           lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
    _ccase(f"MulticlassBinnedAUPRC_{avg}", "MulticlassBinnedAUPRC",
           lambda avg=avg: {"num_classes": C, "average": avg, "threshold": 10},
           lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
    _ccase(f"MultilabelBinnedAUPRC_{avg}", "MultilabelBinnedAUPRC",
           lambda avg=avg: {"num_labels": L, "average": avg, "threshold": [0.0, 0.3, 0.6, 1.0]},
           lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
_ccase("BinaryPrecisionRecallCurve", "BinaryPrecisionRecallCurve", dict,
       lambda s: ((_tied(_rand(_g(s), B)), _randint(_g(s + 1), 0, 2, B)), {}))
_ccase("MulticlassPrecisionRecallCurve", "MulticlassPrecisionRecallCurve", lambda: {"num_classes": C},
       lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
_ccase("MultilabelPrecisionRecallCurve", "MultilabelPrecisionRecallCurve", lambda: {"num_labels": L},
       lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
_ccase("BinaryRecallAtFixedPrecision", "BinaryRecallAtFixedPrecision", lambda: {"min_precision": 0.5},
       lambda s: ((_tied(_rand(_g(s), B)), _randint(_g(s + 1), 0, 2, B)), {}))
_ccase("MultilabelRecallAtFixedPrecision", "MultilabelRecallAtFixedPrecision",
       lambda: {"num_labels": L, "min_precision": 0.5},
       lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
for tname, thr in (("int", 7), ("list", [0.0, 0.2, 0.5, 0.7, 1.0])):
    _ccase(f"BinaryBinnedPrecisionRecallCurve_{tname}", "BinaryBinnedPrecisionRecallCurve",
           lambda thr=thr: {"threshold": thr},
           lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
    _ccase(f"BinaryBinnedAUROC_{tname}", "BinaryBinnedAUROC", lambda thr=thr: {"threshold": thr},
           lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
    _ccase(f"BinaryBinnedAUPRC_{tname}", "BinaryBinnedAUPRC", lambda thr=thr: {"threshold": thr},
           lambda s: ((_rand(_g(s), B), _randint(_g(s + 1), 0, 2, B)), {}))
    _ccase(f"BinaryBinnedAUROC_tasks_{tname}", "BinaryBinnedAUROC",
           lambda thr=thr: {"threshold": thr, "num_tasks": T},
           lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B)), {}))
    _ccase(f"BinaryBinnedAUPRC_tasks_{tname}", "BinaryBinnedAUPRC",
           lambda thr=thr: {"threshold": thr, "num_tasks": T},
           lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B)), {}))
    for opt in ("vectorized", "memory"):
        _ccase(f"MulticlassBinnedPrecisionRecallCurve_{tname}_{opt}", "MulticlassBinnedPrecisionRecallCurve",
               lambda thr=thr, opt=opt: {"num_classes": C, "threshold": thr, "optimization": opt},
               lambda s: ((_rand(_g(s), B, C), _randint(_g(s + 1), 0, C, B)), {}))
        _ccase(f"MultilabelBinnedPrecisionRecallCurve_{tname}_{opt}", "MultilabelBinnedPrecisionRecallCurve",
               lambda thr=thr, opt=opt: {"num_labels": L, "threshold": thr, "optimization": opt},
               lambda s: ((_rand(_g(s), B, L), _randint(_g(s + 1), 0, 2, B, L)), {}))
for logits in (False, True):
    src = (lambda g, *sh: _randn(g, *sh)) if logits else (lambda g, *sh: _rand(g, *sh) * 0.98 + 0.01)
    _ccase(f"BinaryNormalizedEntropy_logits{logits}", "BinaryNormalizedEntropy",
           lambda lg=logits: {"from_logits": lg, "num_tasks": T},
           lambda s, src=src: ((src(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B).float()),
                               {"weight": _rand(_g(s + 2), T, B)}))
    _ccase(f"WindowedBinaryNormalizedEntropy_logits{logits}", "WindowedBinaryNormalizedEntropy",
           lambda lg=logits: {"from_logits": lg, "num_tasks": T, "max_num_updates": 3},
           lambda s, src=src: ((src(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B).float()), {}))
# aggregation
_ccase("Sum", "Sum", dict, lambda s: ((_randn(_g(s), 6),), {"weight": _rand(_g(s + 1), 6)}))
_ccase("Mean", "Mean", dict, lambda s: ((_randn(_g(s), 6),), {"weight": 2.0}))
_ccase("Max", "Max", dict, lambda s: ((_randn(_g(s), 3, 4),), {}))
_ccase("Min", "Min", dict, lambda s: ((_randn(_g(s), 3, 4),), {}))
_ccase("Cat", "Cat", dict, lambda s: ((_randn(_g(s), 2, 3),), {}))
_ccase("Cat_dim1", "Cat", lambda: {"dim": 1}, lambda s: ((_randn(_g(s), 2, 3),), {}))
_ccase("AUC", "AUC", dict, lambda s: ((_rand(_g(s), 10), _rand(_g(s + 1), 10)), {}))
_ccase("AUC_tasks", "AUC", lambda: {"n_tasks": 2}, lambda s: ((_rand(_g(s), 2, 10), _rand(_g(s + 1), 2, 10)), {}))
_ccase("Throughput", "Throughput", dict, lambda s: ((100 + s, 0.5 + 0.01 * s), {}))
# regression
for mo in ("uniform_average", "raw_values"):
    _ccase(f"MeanSquaredError_{mo}", "MeanSquaredError", lambda mo=mo: {"multioutput": mo},
           lambda s: ((_randn(_g(s), B, 3), _randn(_g(s + 1), B, 3)), {"sample_weight": _rand(_g(s + 2), B)}))
    _ccase(f"WindowedMeanSquaredError_{mo}", "WindowedMeanSquaredError",
           lambda mo=mo: {"multioutput": mo, "max_num_updates": 2, "num_tasks": 3},
           lambda s: ((_randn(_g(s), B, 3), _randn(_g(s + 1), B, 3)), {"sample_weight": _rand(_g(s + 2), B)}))
    _ccase(f"WindowedMeanSquaredError_1d_{mo}", "WindowedMeanSquaredError",
           lambda mo=mo: {"multioutput": mo, "max_num_updates": 3},
           lambda s: ((_randn(_g(s), B), _randn(_g(s + 1), B)), {}))
for mo in ("uniform_average", "raw_values", "variance_weighted"):
    _ccase(f"R2Score_{mo}", "R2Score", lambda mo=mo: {"multioutput": mo, "num_regressors": 2},
           lambda s: ((_randn(_g(s), B, 3), _randn(_g(s + 1), B, 3)), {}))
_ccase("MeanSquaredError_1d", "MeanSquaredError", dict,
       lambda s: ((_randn(_g(s), B), _randn(_g(s + 1), B)), {}))
_ccase("R2Score_1d", "R2Score", dict, lambda s: ((_randn(_g(s), B), _randn(_g(s + 1), B)), {}))
# image
_ccase("PeakSignalNoiseRatio_auto", "PeakSignalNoiseRatio", dict,
       lambda s: ((_rand(_g(s), 2, 3, 8, 8), _rand(_g(s + 1), 2, 3, 8, 8) * 1.5), {}))
_ccase("PeakSignalNoiseRatio_fixed", "PeakSignalNoiseRatio", lambda: {"data_range": 1.0},
       lambda s: ((_rand(_g(s), 2, 3, 8, 8), _rand(_g(s + 1), 2, 3, 8, 8)), {}))
# ranking
_ccase("ClickThroughRate", "ClickThroughRate", lambda: {"num_tasks": T},
       lambda s: ((_randint(_g(s), 0, 2, T, B).float(), _rand(_g(s + 1), T, B)), {}))
_ccase("WindowedClickThroughRate_no_lifetime", "WindowedClickThroughRate",
       lambda: {"num_tasks": T, "max_num_updates": 3, "enable_lifetime": False},
       lambda s: ((_randint(_g(s), 0, 2, T, B).float(), _rand(_g(s + 1), T, B)), {}))
_ccase("WindowedWeightedCalibration_no_lifetime", "WindowedWeightedCalibration",
       lambda: {"num_tasks": T, "max_num_updates": 3, "enable_lifetime": False},
       lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B)), {}))
_ccase("WindowedBinaryNormalizedEntropy_no_lifetime", "WindowedBinaryNormalizedEntropy",
       lambda: {"max_num_updates": 2, "enable_lifetime": False},
       lambda s: ((_rand(_g(s), B) * 0.9 + 0.05, _randint(_g(s + 1), 0, 2, B).float()), {}))
_ccase("WindowedMeanSquaredError_no_lifetime", "WindowedMeanSquaredError",
       lambda: {"max_num_updates": 5, "enable_lifetime": False},
       lambda s: ((_randn(_g(s), B), _randn(_g(s + 1), B)), {}))
_ccase("WindowedBinaryAUROC_small_window", "WindowedBinaryAUROC", lambda: {"max_num_samples": 30},
       lambda s: ((_rand(_g(s), 20), _randint(_g(s + 1), 0, 2, 20)), {"weight": _rand(_g(s + 2), 20)}))
_ccase("WindowedClickThroughRate", "WindowedClickThroughRate", lambda: {"num_tasks": T, "max_num_updates": 3},
       lambda s: ((_randint(_g(s), 0, 2, T, B).float(), _rand(_g(s + 1), T, B)), {}))
_ccase("WeightedCalibration", "WeightedCalibration", lambda: {"num_tasks": T},
       lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B), _rand(_g(s + 2), T, B)), {}))
_ccase("WindowedWeightedCalibration", "WindowedWeightedCalibration",
       lambda: {"num_tasks": T, "max_num_updates": 2},
       lambda s: ((_rand(_g(s), T, B), _randint(_g(s + 1), 0, 2, T, B)), {}))
for k in (None, 2):
    _ccase(f"HitRate_k{k}", "HitRate", lambda k=k: {"k": k},
           lambda s: ((_rand(_g(s), 8, C), _randint(_g(s + 1), 0, C, 8)), {}))
    _ccase(f"ReciprocalRank_k{k}", "ReciprocalRank", lambda k=k: {"k": k},
           lambda s: ((_rand(_g(s), 8, C), _randint(_g(s + 1), 0, C, 8)), {}))
_ccase("RetrievalPrecision", "RetrievalPrecision", lambda: {"k": 3},
       lambda s: ((_rand(_g(s), 10), _randint(_g(s + 1), 0, 2, 10)), {}))
_ccase("RetrievalPrecision_queries", "RetrievalPrecision", lambda: {"k": 2, "num_queries": 3, "avg": "macro"},
       lambda s: ((_rand(_g(s), 9), _randint(_g(s + 1), 0, 2, 9)), {"indexes": _randint(_g(s + 2), 0, 3, 9)}))
_ccase("RetrievalPrecision_queries_none", "RetrievalPrecision",
       lambda: {"k": 2, "num_queries": 3, "avg": "none", "limit_k_to_size": True},
       lambda s: ((_rand(_g(s), 9), _randint(_g(s + 1), 0, 2, 9)), {"indexes": _randint(_g(s + 2), 0, 3, 9)}))
_ccase("WindowedBinaryAUROC", "WindowedBinaryAUROC", lambda: {"num_tasks": T, "max_num_samples": 50},
       lambda s: ((_rand(_g(s), T, 20), _randint(_g(s + 1), 0, 2, T, 20)), {}))
# text
_ccase("BLEUScore", "BLEUScore", lambda: {"n_gram": 3},
       lambda s: (([_HYP[s % 3]], [_REF[s % 3]]), {}))
_ccase("Perplexity", "Perplexity", lambda: {"ignore_index": 2},
       lambda s: ((_randn(_g(s), 2, 6, 9), _randint(_g(s + 1), 0, 9, 2, 6)), {}))
for cls in ("WordErrorRate", "WordInformationLost", "WordInformationPreserved"):
    _ccase(cls, cls, dict, lambda s: (([_WER_IN[s % 3]], [_WER_TG[s % 3]]), {}))


def cid_seed(cid: str) -> int:
    """Stable per-case seed (Python's hash() is salted per process)."""
    import zlib

    return zlib.crc32(cid.encode()) % 100_000


# ----------------------------------------------------------------------------------------
# error cases: the reference raises; we must raise the same exception type with the same
# message.  id -> ("fn" | "cls", name, builder() -> (args, kwargs)); for "cls" the builder
# returns (ctor_kwargs, [update args/kwargs ...]).
# ----------------------------------------------------------------------------------------
ERRORS: Dict[str, Tuple[str, str, Callable[[], Any]]] = {}


def _err(case_id: str, kind: str, name: str, builder: Callable[[], Any]) -> None:
    ERRORS[case_id] = (kind, name, builder)


def _x(*shape):
    return torch.rand(*shape, generator=_g(sum(shape) + 7))


def _y(hi, *shape):
    return torch.randint(0, hi, shape, generator=_g(sum(shape) + 11))


# accuracy
_err("mc_acc_bad_average", "fn", "multiclass_accuracy", lambda: ((_x(4, 3), _y(3, 4)), {"average": "weighted"}))
_err("mc_acc_macro_no_classes", "fn", "multiclass_accuracy", lambda: ((_x(4, 3), _y(3, 4)), {"average": "macro"}))
_err("mc_acc_bad_k", "fn", "multiclass_accuracy", lambda: ((_x(4, 3), _y(3, 4)), {"k": 0}))
_err("mc_acc_3d", "fn", "multiclass_accuracy", lambda: ((_x(4, 3, 2), _y(3, 4)), {}))
_err("mc_acc_len_mismatch", "fn", "multiclass_accuracy", lambda: ((_x(4, 3), _y(3, 5)), {}))
_err("mc_acc_topk_labels", "fn", "multiclass_accuracy", lambda: ((_y(3, 4), _y(3, 4)), {"k": 2}))
_err("bin_acc_shape", "fn", "binary_accuracy", lambda: ((_x(4), _y(2, 5)), {}))
_err("bin_acc_2d", "fn", "binary_accuracy", lambda: ((_x(4, 2), _y(2, 4, 2)), {}))
_err("ml_acc_criteria", "fn", "multilabel_accuracy", lambda: ((_x(4, 3), _y(2, 4, 3)), {"criteria": "foo"}))
_err("ml_acc_shape", "fn", "multilabel_accuracy", lambda: ((_x(4, 3), _y(2, 4, 2)), {}))
_err("topk_ml_k1", "fn", "topk_multilabel_accuracy", lambda: ((_x(4, 3), _y(2, 4, 3)), {"k": 1}))
_err("topk_ml_criteria", "fn", "topk_multilabel_accuracy", lambda: ((_x(4, 3), _y(2, 4, 3)), {"criteria": "x"}))
_err("topk_ml_1d", "fn", "topk_multilabel_accuracy", lambda: ((_x(4), _y(2, 4)), {}))
# precision / recall / f1
for fam in ("precision", "recall", "f1_score"):
    _err(f"mc_{fam}_bad_average", "fn", f"multiclass_{fam}",
         lambda: ((_x(4, 3), _y(3, 4)), {"average": "samples", "num_classes": 3}))
    _err(f"mc_{fam}_macro_no_classes", "fn", f"multiclass_{fam}", lambda: ((_x(4, 3), _y(3, 4)), {"average": "macro"}))
    _err(f"mc_{fam}_len_mismatch", "fn", f"multiclass_{fam}", lambda: ((_x(4, 3), _y(3, 5)), {"num_classes": 3}))
    _err(f"mc_{fam}_bad_input_shape", "fn", f"multiclass_{fam}",
         lambda: ((_x(4, 2), _y(3, 4)), {"num_classes": 3, "average": "macro"}))
    _err(f"bin_{fam}_shape", "fn", f"binary_{fam}", lambda: ((_x(4), _y(2, 5)), {}))
    _err(f"bin_{fam}_2d", "fn", f"binary_{fam}", lambda: ((_x(4, 2), _y(2, 4, 2)), {}))
# confusion matrix
_err("cm_bad_normalize", "fn", "multiclass_confusion_matrix", lambda: ((_x(4, 3), _y(3, 4), 3), {"normalize": "x"}))
_err("cm_one_class", "fn", "multiclass_confusion_matrix", lambda: ((_x(4, 1), _y(1, 4), 1), {}))
_err("cm_target_range", "fn", "multiclass_confusion_matrix",
     lambda: ((_x(4, 3), torch.tensor([0, 1, 3, 2]), 3), {}))
_err("cm_input_range", "fn", "multiclass_confusion_matrix",
     lambda: ((torch.tensor([0, 1, 5, 2]), torch.tensor([0, 1, 1, 2]), 3), {}))
_err("cm_input_shape", "fn", "multiclass_confusion_matrix", lambda: ((_x(4, 2), _y(3, 4), 3), {}))
_err("bcm_bad_normalize", "fn", "binary_confusion_matrix", lambda: ((_x(4), _y(2, 4)), {"normalize": "rows"}))
_err("bcm_shape", "fn", "binary_confusion_matrix", lambda: ((_x(4), _y(2, 3)), {}))
# auroc / auprc / curves
_err("bauroc_tasks0", "fn", "binary_auroc", lambda: ((_x(4), _y(2, 4)), {"num_tasks": 0}))
_err("bauroc_shape", "fn", "binary_auroc", lambda: ((_x(4), _y(2, 5)), {}))
_err("bauroc_tasks_1d", "fn", "binary_auroc", lambda: ((_x(4), _y(2, 4)), {"num_tasks": 2}))
_err("bauroc_3d", "fn", "binary_auroc", lambda: ((_x(2, 2, 2), _y(2, 2, 2, 2)), {}))
_err("bauroc_weight_shape", "fn", "binary_auroc", lambda: ((_x(4), _y(2, 4)), {"weight": _x(5)}))
_err("mcauroc_average", "fn", "multiclass_auroc", lambda: ((_x(4, 3), _y(3, 4)), {"num_classes": 3, "average": "micro"}))
_err("mcauroc_one_class", "fn", "multiclass_auroc", lambda: ((_x(4, 1), _y(1, 4)), {"num_classes": 1}))
_err("mcauroc_shape", "fn", "multiclass_auroc", lambda: ((_x(4, 2), _y(3, 4)), {"num_classes": 3}))
_err("mcauroc_len", "fn", "multiclass_auroc", lambda: ((_x(4, 3), _y(3, 5)), {"num_classes": 3}))
_err("bauprc_tasks_shape", "fn", "binary_auprc", lambda: ((_x(3, 4), _y(2, 3, 4)), {"num_tasks": 2}))
_err("bauprc_shape", "fn", "binary_auprc", lambda: ((_x(4), _y(2, 5)), {}))
_err("mcauprc_average", "fn", "multiclass_auprc", lambda: ((_x(4, 3), _y(3, 4)), {"num_classes": 3, "average": "micro"}))
_err("mcauprc_shape", "fn", "multiclass_auprc", lambda: ((_x(4, 2), _y(3, 4)), {"num_classes": 3}))
_err("mlauprc_average", "fn", "multilabel_auprc", lambda: ((_x(4, 3), _y(2, 4, 3)), {"num_labels": 3, "average": "x"}))
_err("mlauprc_shape", "fn", "multilabel_auprc", lambda: ((_x(4, 3), _y(2, 4, 2)), {"num_labels": 3}))
_err("bprc_shape", "fn", "binary_precision_recall_curve", lambda: ((_x(4), _y(2, 5)), {}))
_err("bprc_2d", "fn", "binary_precision_recall_curve", lambda: ((_x(2, 4), _y(2, 2, 4)), {}))
_err("mcprc_shape", "fn", "multiclass_precision_recall_curve", lambda: ((_x(4, 2), _y(3, 4)), {"num_classes": 3}))
_err("mlprc_shape", "fn", "multilabel_precision_recall_curve", lambda: ((_x(4, 3), _y(2, 4, 2)), {"num_labels": 3}))
_err("brafp_range", "fn", "binary_recall_at_fixed_precision", lambda: ((_x(4), _y(2, 4)), {"min_precision": 1.5}))
_err("mlrafp_range", "fn", "multilabel_recall_at_fixed_precision",
     lambda: ((_x(4, 3), _y(2, 4, 3)), {"num_labels": 3, "min_precision": -0.1}))
# binned
_err("bbprc_unsorted", "fn", "binary_binned_precision_recall_curve",
     lambda: ((_x(4), _y(2, 4)), {"threshold": torch.tensor([0.1, 0.5, 0.2, 1.0])}))
_err("bbprc_range", "fn", "binary_binned_precision_recall_curve",
     lambda: ((_x(4), _y(2, 4)), {"threshold": [-0.1, 0.5, 1.0]}))
_err("bbprc_shape", "fn", "binary_binned_precision_recall_curve", lambda: ((_x(4), _y(2, 5)), {}))
_err("mcbprc_opt", "fn", "multiclass_binned_precision_recall_curve",
     lambda: ((_x(4, 3), _y(3, 4)), {"num_classes": 3, "optimization": "speed"}))
_err("mcbprc_shape", "fn", "multiclass_binned_precision_recall_curve",
     lambda: ((_x(4, 2), _y(3, 4)), {"num_classes": 3}))
_err("mlbprc_opt", "fn", "multilabel_binned_precision_recall_curve",
     lambda: ((_x(4, 3), _y(2, 4, 3)), {"num_labels": 3, "optimization": "speed"}))
_err("bbauroc_tasks", "fn", "binary_binned_auroc", lambda: ((_x(4), _y(2, 4)), {"num_tasks": 2}))
_err("bbauroc_unsorted", "fn", "binary_binned_auroc", lambda: ((_x(4), _y(2, 4)), {"threshold": [0.0, 0.6, 0.3, 1.0]}))
_err("mcbauroc_average", "fn", "multiclass_binned_auroc",
     lambda: ((_x(4, 3), _y(3, 4)), {"num_classes": 3, "average": "weighted"}))
_err("mcbauroc_classes", "fn", "multiclass_binned_auroc", lambda: ((_x(4, 1), _y(1, 4)), {"num_classes": 1}))
_err("bbauprc_tasks", "fn", "binary_binned_auprc", lambda: ((_x(2, 4), _y(2, 2, 4)), {"num_tasks": 3}))
_err("mcbauprc_average", "fn", "multiclass_binned_auprc",
     lambda: ((_x(4, 3), _y(3, 4)), {"num_classes": 3, "average": "weighted"}))
_err("mlbauprc_shape", "fn", "multilabel_binned_auprc", lambda: ((_x(4, 3), _y(2, 4, 2)), {"num_labels": 3}))
# normalized entropy
_err("ne_shape", "fn", "binary_normalized_entropy", lambda: ((_x(4), _y(2, 5).float()), {}))
_err("ne_tasks", "fn", "binary_normalized_entropy", lambda: ((_x(4), _y(2, 4).float()), {"num_tasks": 2}))
_err("ne_weight_shape", "fn", "binary_normalized_entropy", lambda: ((_x(4), _y(2, 4).float()), {"weight": _x(3)}))
_err("ne_prob_range", "fn", "binary_normalized_entropy",
     lambda: ((torch.tensor([0.2, 1.5, 0.3]), torch.tensor([0.0, 1.0, 1.0])), {}))
# aggregation
_err("mean_weight_shape", "fn", "mean", lambda: ((_x(4),), {"weight": _x(3)}))
_err("sum_weight_shape", "fn", "sum", lambda: ((_x(4),), {"weight": _x(3)}))
_err("throughput_negative", "fn", "throughput", lambda: ((-1, 1.0), {}))
_err("throughput_zero_time", "fn", "throughput", lambda: ((10, 0.0), {}))
_err("auc_shape", "fn", "auc", lambda: ((_x(4), _x(5)), {}))
# regression
_err("mse_multioutput", "fn", "mean_squared_error", lambda: ((_x(4), _x(4)), {"multioutput": "x"}))
_err("mse_shape", "fn", "mean_squared_error", lambda: ((_x(4), _x(5)), {}))
_err("mse_weight_shape", "fn", "mean_squared_error", lambda: ((_x(4), _x(4)), {"sample_weight": _x(3)}))
_err("mse_3d", "fn", "mean_squared_error", lambda: ((_x(2, 2, 2), _x(2, 2, 2)), {}))
_err("r2_multioutput", "fn", "r2_score", lambda: ((_x(4), _x(4)), {"multioutput": "x"}))
_err("r2_regressors", "fn", "r2_score", lambda: ((_x(4), _x(4)), {"num_regressors": -1}))
_err("r2_too_few", "fn", "r2_score", lambda: ((_x(1), _x(1)), {}))
_err("r2_shape", "fn", "r2_score", lambda: ((_x(4), _x(5)), {}))
_err("r2_adjusted_too_many", "fn", "r2_score", lambda: ((_x(4), _x(4)), {"num_regressors": 3}))
# image
_err("psnr_range", "fn", "peak_signal_noise_ratio", lambda: ((_x(2, 3), _x(2, 3)), {"data_range": -1.0}))
_err("psnr_shape", "fn", "peak_signal_noise_ratio", lambda: ((_x(2, 3), _x(3, 3)), {}))
# ranking
_err("ctr_weights_shape", "fn", "click_through_rate", lambda: ((_x(4), _x(3)), {}))
_err("ctr_tasks", "fn", "click_through_rate", lambda: ((_x(4),), {"num_tasks": 2}))
_err("freq_k_negative", "fn", "frequency_at_k", lambda: ((_x(4),), {"k": -1.0}))
_err("freq_2d", "fn", "frequency_at_k", lambda: ((_x(2, 2),), {"k": 1.0}))
_err("hit_rate_1d", "fn", "hit_rate", lambda: ((_x(4), _y(4, 4)), {}))
_err("hit_rate_k0", "fn", "hit_rate", lambda: ((_x(4, 4), _y(4, 4)), {"k": 0}))
_err("rr_target_2d", "fn", "reciprocal_rank", lambda: ((_x(4, 4), _y(4, 4, 1)), {}))
_err("num_collisions_2d", "fn", "num_collisions", lambda: ((_y(4, 3, 3),), {}))
_err("num_collisions_float", "fn", "num_collisions", lambda: ((_x(4),), {}))
_err("rp_k0", "fn", "retrieval_precision", lambda: ((_x(4), _y(2, 4)), {"k": 0}))
_err("rp_shape", "fn", "retrieval_precision", lambda: ((_x(4), _y(2, 5)), {}))
_err("rp_tasks", "fn", "retrieval_precision", lambda: ((_x(4), _y(2, 4)), {"num_tasks": 2}))
_err("wc_shape", "fn", "weighted_calibration", lambda: ((_x(4), _y(2, 5)), {}))
_err("wc_tasks", "fn", "weighted_calibration", lambda: ((_x(4), _y(2, 4)), {"num_tasks": 2}))
# text
_err("bleu_ngram", "fn", "bleu_score", lambda: ((["a b c"], [["a b c"]]), {"n_gram": 5}))
_err("bleu_weights", "fn", "bleu_score", lambda: ((["a b c"], [["a b c"]]), {"n_gram": 2, "weights": torch.ones(3)}))
_err("bleu_len", "fn", "bleu_score", lambda: ((["a b c", "d"], [["a b c"]]), {}))
_err("bleu_short", "fn", "bleu_score", lambda: ((["a b"], [["a b"]]), {"n_gram": 3}))
_err("ppl_shape", "fn", "perplexity", lambda: ((_x(2, 3, 4), _y(4, 2, 4)), {}))
_err("ppl_2d", "fn", "perplexity", lambda: ((_x(3, 4), _y(4, 3)), {}))
_err("ppl_target_range", "fn", "perplexity", lambda: ((_x(1, 3, 4), torch.tensor([[0, 9, 1]])), {}))
_err("wer_len", "fn", "word_error_rate", lambda: ((["a b", "c"], ["a b"]), {}))
_err("wil_len", "fn", "word_information_lost", lambda: ((["a b", "c"], ["a b"]), {}))
_err("wip_len", "fn", "word_information_preserved", lambda: ((["a b", "c"], ["a b"]), {}))
# class constructors and update checks
_err("cls_mc_acc_average", "cls", "MulticlassAccuracy", lambda: ({"average": "x"}, []))
_err("cls_bauroc_tasks", "cls", "BinaryAUROC", lambda: ({"num_tasks": 0}, []))
_err("cls_bauroc_update", "cls", "BinaryAUROC", lambda: ({"num_tasks": 2}, [((_x(4), _y(2, 4)), {})]))
_err("cls_mcauroc_classes", "cls", "MulticlassAUROC", lambda: ({"num_classes": 1}, []))
_err("cls_wauroc_max", "cls", "WindowedBinaryAUROC", lambda: ({"max_num_samples": 0}, []))
_err("cls_wauroc_tasks", "cls", "WindowedBinaryAUROC", lambda: ({"num_tasks": 0}, []))
_err("cls_wne_max", "cls", "WindowedBinaryNormalizedEntropy", lambda: ({"max_num_updates": 0}, []))
_err("cls_wctr_max", "cls", "WindowedClickThroughRate", lambda: ({"max_num_updates": 0}, []))
_err("cls_wmse_max", "cls", "WindowedMeanSquaredError", lambda: ({"max_num_updates": 0}, []))
_err("cls_wwc_max", "cls", "WindowedWeightedCalibration", lambda: ({"max_num_updates": 0}, []))
_err("cls_rp_action", "cls", "RetrievalPrecision", lambda: ({"empty_target_action": "x"}, []))
_err("cls_rp_k", "cls", "RetrievalPrecision", lambda: ({"k": 0}, []))
_err("cls_rp_queries", "cls", "RetrievalPrecision", lambda: ({"num_queries": 0}, []))
_err("cls_rp_err_empty", "cls", "RetrievalPrecision",
     lambda: ({"empty_target_action": "err"}, [((_x(4), torch.zeros(4, dtype=torch.long)), {})]))
_err("cls_throughput_neg", "cls", "Throughput", lambda: ({}, [((-3, 1.0), {})]))
_err("cls_bleu_ngram", "cls", "BLEUScore", lambda: ({"n_gram": 0}, []))
_err("cls_psnr_range", "cls", "PeakSignalNoiseRatio", lambda: ({"data_range": 0.0}, []))
_err("cls_mse_multioutput", "cls", "MeanSquaredError", lambda: ({"multioutput": "x"}, []))
_err("cls_r2_regressors", "cls", "R2Score", lambda: ({"num_regressors": -2}, []))
_err("cls_auc_shape", "cls", "AUC", lambda: ({"n_tasks": 2}, [((_x(4), _x(4)), {})]))
_err("cls_bbauroc_thr", "cls", "BinaryBinnedAUROC", lambda: ({"threshold": [0.5, 0.2]}, []))
_err("cls_mcbprc_opt", "cls", "MulticlassBinnedPrecisionRecallCurve", lambda: ({"num_classes": 3, "optimization": "x"}, []))
_err("cls_ne_update", "cls", "BinaryNormalizedEntropy", lambda: ({"num_tasks": 2}, [((_x(4), _y(2, 4).float()), {})]))
_err("cls_topk_ml_k", "cls", "TopKMultilabelAccuracy", lambda: ({"k": 1}, []))
_err("cls_ctr_tasks", "cls", "ClickThroughRate", lambda: ({"num_tasks": 0}, []))
_err("cls_hit_rate_k", "cls", "HitRate", lambda: ({"k": 0}, [((_x(4, 4), _y(4, 4)), {})]))
# class constructors / update checks of every classification family (same message as the
# reference; GPU class updates may defer a data check to compute(), which the runner includes)
_U = lambda *a: [(a, {})]  # noqa: E731
_err("cls_bacc_shape", "cls", "BinaryAccuracy", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_mcacc_len", "cls", "MulticlassAccuracy", lambda: ({}, _U(_x(4, 3), _y(3, 5))))
_err("cls_mcacc_k0", "cls", "MulticlassAccuracy", lambda: ({"k": 0}, []))
_err("cls_mcacc_macro_nc", "cls", "MulticlassAccuracy", lambda: ({"average": "macro"}, []))
_err("cls_mlacc_criteria", "cls", "MultilabelAccuracy", lambda: ({"criteria": "foo"}, []))
_err("cls_mlacc_shape", "cls", "MultilabelAccuracy", lambda: ({}, _U(_x(4, 3), _y(2, 4, 2))))
_err("cls_topk_ml_criteria", "cls", "TopKMultilabelAccuracy", lambda: ({"criteria": "x", "k": 2}, []))
_err("cls_topk_ml_1d", "cls", "TopKMultilabelAccuracy", lambda: ({"k": 2}, _U(_x(4), _y(2, 4))))
for _fam, _cls in (("prec", "Precision"), ("rec", "Recall"), ("f1", "F1Score")):
    _err(f"cls_b{_fam}_shape", "cls", f"Binary{_cls}", lambda _c=_cls: ({}, _U(_x(4), _y(2, 5))))
    _err(f"cls_mc{_fam}_average", "cls", f"Multiclass{_cls}", lambda _c=_cls: ({"average": "samples", "num_classes": 3}, []))
    _err(f"cls_mc{_fam}_macro_nc", "cls", f"Multiclass{_cls}", lambda _c=_cls: ({"average": "macro"}, []))
    _err(f"cls_mc{_fam}_len", "cls", f"Multiclass{_cls}", lambda _c=_cls: ({"num_classes": 3}, _U(_x(4, 3), _y(3, 5))))
_err("cls_bcm_normalize", "cls", "BinaryConfusionMatrix", lambda: ({"normalize": "rows"}, []))
_err("cls_bcm_shape", "cls", "BinaryConfusionMatrix", lambda: ({}, _U(_x(4), _y(2, 3))))
_err("cls_mccm_one_class", "cls", "MulticlassConfusionMatrix", lambda: ({"num_classes": 1}, []))
_err("cls_mccm_normalize", "cls", "MulticlassConfusionMatrix", lambda: ({"num_classes": 3, "normalize": "x"}, []))
_err("cls_mccm_target_range", "cls", "MulticlassConfusionMatrix",
     lambda: ({"num_classes": 3}, _U(_x(4, 3), torch.tensor([0, 1, 5, 2]))))
_err("cls_mccm_target_range_i32", "cls", "MulticlassConfusionMatrix",
     lambda: ({"num_classes": 3}, _U(_x(4, 3), torch.tensor([0, 4, 1, 2], dtype=torch.int32))))
_err("cls_mccm_input_range", "cls", "MulticlassConfusionMatrix",
     lambda: ({"num_classes": 3}, _U(torch.tensor([0, 1, 7, 2]), torch.tensor([0, 1, 1, 2]))))
_err("cls_mccm_input_shape", "cls", "MulticlassConfusionMatrix", lambda: ({"num_classes": 3}, _U(_x(4, 2), _y(3, 4))))
_err("cls_bauprc_shape", "cls", "BinaryAUPRC", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_bauprc_tasks", "cls", "BinaryAUPRC", lambda: ({"num_tasks": 0}, []))
_err("cls_mcauprc_classes", "cls", "MulticlassAUPRC", lambda: ({"num_classes": 1}, []))
_err("cls_mcauprc_average", "cls", "MulticlassAUPRC", lambda: ({"num_classes": 3, "average": "x"}, []))
_err("cls_mcauprc_shape", "cls", "MulticlassAUPRC", lambda: ({"num_classes": 3}, _U(_x(4, 2), _y(3, 4))))
_err("cls_mlauprc_labels", "cls", "MultilabelAUPRC", lambda: ({"num_labels": 1}, []))
_err("cls_mlauprc_average", "cls", "MultilabelAUPRC", lambda: ({"num_labels": 3, "average": "x"}, []))
_err("cls_mlauprc_shape", "cls", "MultilabelAUPRC", lambda: ({"num_labels": 3}, _U(_x(4, 3), _y(2, 4, 2))))
_err("cls_mcauroc_average", "cls", "MulticlassAUROC", lambda: ({"num_classes": 3, "average": "x"}, []))
_err("cls_mcauroc_shape", "cls", "MulticlassAUROC", lambda: ({"num_classes": 3}, _U(_x(4, 2), _y(3, 4))))
_err("cls_bbauprc_thr", "cls", "BinaryBinnedAUPRC", lambda: ({"threshold": [0.5, 0.2]}, []))
_err("cls_bbauprc_shape", "cls", "BinaryBinnedAUPRC", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_mcbauprc_classes", "cls", "MulticlassBinnedAUPRC", lambda: ({"num_classes": 1}, []))
_err("cls_mcbauprc_thr", "cls", "MulticlassBinnedAUPRC", lambda: ({"num_classes": 3, "threshold": [0.9, 0.1]}, []))
_err("cls_mcbauprc_shape", "cls", "MulticlassBinnedAUPRC", lambda: ({"num_classes": 3}, _U(_x(4, 2), _y(3, 4))))
_err("cls_mlbauprc_thr", "cls", "MultilabelBinnedAUPRC", lambda: ({"num_labels": 3, "threshold": [0.9, 0.1]}, []))
_err("cls_mlbauprc_shape", "cls", "MultilabelBinnedAUPRC", lambda: ({"num_labels": 3}, _U(_x(4, 3), _y(2, 4, 2))))
_err("cls_bbauroc_shape", "cls", "BinaryBinnedAUROC", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_mcbauroc_thr", "cls", "MulticlassBinnedAUROC", lambda: ({"num_classes": 3, "threshold": [0.9, 0.1]}, []))
_err("cls_bbprc_thr", "cls", "BinaryBinnedPrecisionRecallCurve", lambda: ({"threshold": [0.5, 0.2]}, []))
_err("cls_bbprc_shape", "cls", "BinaryBinnedPrecisionRecallCurve", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_mlbprc_thr", "cls", "MultilabelBinnedPrecisionRecallCurve", lambda: ({"num_labels": 3, "threshold": [0.9, 0.1]}, []))
_err("cls_bprc_shape", "cls", "BinaryPrecisionRecallCurve", lambda: ({}, _U(_x(4), _y(2, 5))))
_err("cls_mcprc_shape", "cls", "MulticlassPrecisionRecallCurve", lambda: ({"num_classes": 3}, _U(_x(4, 2), _y(3, 4))))
_err("cls_mlprc_shape", "cls", "MultilabelPrecisionRecallCurve", lambda: ({"num_labels": 3}, _U(_x(4, 3), _y(2, 4, 2))))
_err("cls_brafp_min_precision", "cls", "BinaryRecallAtFixedPrecision", lambda: ({"min_precision": 1.5}, []))
_err("cls_mlrafp_min_precision", "cls", "MultilabelRecallAtFixedPrecision",
     lambda: ({"num_labels": 3, "min_precision": -0.1}, []))
_err("cls_bne_range", "cls", "BinaryNormalizedEntropy", lambda: ({}, _U(_x(4) + 1.5, _y(2, 4).float())))
_err("cls_mean_weight_shape", "cls", "Mean", lambda: ({}, [((_x(4),), {"weight": _x(3)})]))
_err("cls_sum_weight_shape", "cls", "Sum", lambda: ({}, [((_x(4),), {"weight": _x(3)})]))
_err("cls_cat_dim", "cls", "Cat", lambda: ({"dim": 1}, _U(_x(4))))
_err("cls_mse_shape", "cls", "MeanSquaredError", lambda: ({}, _U(_x(4), _x(5))))
_err("cls_r2_shape", "cls", "R2Score", lambda: ({}, _U(_x(4), _x(5))))
_err("cls_r2_multioutput", "cls", "R2Score", lambda: ({"multioutput": "x"}, []))
_err("cls_psnr_shape", "cls", "PeakSignalNoiseRatio", lambda: ({}, _U(_x(1, 3, 4, 4), _x(1, 3, 4, 5))))
_err("cls_ctr_shape", "cls", "ClickThroughRate", lambda: ({}, [((_y(2, 4),), {"weights": _x(3)})]))
_err("cls_wc_shape", "cls", "WeightedCalibration", lambda: ({}, _U(_x(4), _x(5))))
_err("cls_rr_shape", "cls", "ReciprocalRank", lambda: ({}, _U(_x(4, 4), _y(4, 3))))
_err("cls_wer_len", "cls", "WordErrorRate", lambda: ({}, _U(["a b"], ["a b", "c"])))
_err("cls_perplexity_shape", "cls", "Perplexity", lambda: ({}, _U(_x(2, 3, 5), _y(5, 2, 4))))


# ----------------------------------------------------------------------------------------
# empty inputs (0 samples): whatever the reference does - a value, NaN, or an exception - the
# CPU paths and the HIP kernels (which must not launch a 0-sized grid) have to do the same
# ----------------------------------------------------------------------------------------
def _e(*shape):
    return torch.zeros(*shape)


def _ei(*shape):
    return torch.zeros(*shape, dtype=torch.long)


for _name, _fn, _b in [
    ("binary_accuracy", "binary_accuracy", lambda: ((_e(0), _ei(0)), {})),
    ("multiclass_accuracy", "multiclass_accuracy", lambda: ((_e(0, C), _ei(0)), {})),
    ("multiclass_accuracy_macro", "multiclass_accuracy", lambda: ((_e(0, C), _ei(0)), {"average": "macro", "num_classes": C})),
    ("multilabel_accuracy", "multilabel_accuracy", lambda: ((_e(0, L), _ei(0, L)), {})),
    ("topk_multilabel_accuracy", "topk_multilabel_accuracy", lambda: ((_e(0, L), _ei(0, L)), {"k": 2})),
    ("binary_precision", "binary_precision", lambda: ((_e(0), _ei(0)), {})),
    ("binary_recall", "binary_recall", lambda: ((_e(0), _ei(0)), {})),
    ("binary_f1_score", "binary_f1_score", lambda: ((_e(0), _ei(0)), {})),
    ("multiclass_precision", "multiclass_precision", lambda: ((_e(0, C), _ei(0)), {"num_classes": C, "average": "macro"})),
    ("multiclass_recall", "multiclass_recall", lambda: ((_e(0, C), _ei(0)), {"num_classes": C})),
    ("multiclass_f1_score", "multiclass_f1_score", lambda: ((_e(0, C), _ei(0)), {"num_classes": C, "average": None})),
    ("binary_confusion_matrix", "binary_confusion_matrix", lambda: ((_e(0), _ei(0)), {})),
    ("multiclass_confusion_matrix", "multiclass_confusion_matrix", lambda: ((_e(0, C), _ei(0), C), {})),
    ("binary_auroc", "binary_auroc", lambda: ((_e(0), _ei(0)), {})),
    ("binary_auprc", "binary_auprc", lambda: ((_e(0), _ei(0)), {})),
    ("multiclass_auroc", "multiclass_auroc", lambda: ((_e(0, C), _ei(0)), {"num_classes": C})),
    ("multiclass_auprc", "multiclass_auprc", lambda: ((_e(0, C), _ei(0)), {"num_classes": C})),
    ("binary_precision_recall_curve", "binary_precision_recall_curve", lambda: ((_e(0), _ei(0)), {})),
    ("binary_binned_auroc", "binary_binned_auroc", lambda: ((_e(0), _ei(0)), {"threshold": 5})),
    ("binary_binned_precision_recall_curve", "binary_binned_precision_recall_curve", lambda: ((_e(0), _ei(0)), {"threshold": 5})),
    ("multiclass_binned_auprc", "multiclass_binned_auprc", lambda: ((_e(0, C), _ei(0)), {"num_classes": C, "threshold": 5})),
    ("binary_normalized_entropy", "binary_normalized_entropy", lambda: ((_e(0), _e(0)), {})),
    ("mean_squared_error", "mean_squared_error", lambda: ((_e(0), _e(0)), {})),
    ("mean_squared_error_2d", "mean_squared_error", lambda: ((_e(0, 3), _e(0, 3)), {})),
    ("r2_score", "r2_score", lambda: ((_e(0), _e(0)), {})),
    ("perplexity", "perplexity", lambda: ((_e(0, 4, 7), _ei(0, 4)), {})),
    ("hit_rate", "hit_rate", lambda: ((_e(0, C), _ei(0)), {"k": 2})),
    ("reciprocal_rank", "reciprocal_rank", lambda: ((_e(0, C), _ei(0)), {})),
    ("click_through_rate", "click_through_rate", lambda: ((_e(0),), {})),
    ("weighted_calibration", "weighted_calibration", lambda: ((_e(0), _ei(0)), {})),
    ("sum", "sum", lambda: ((_e(0),), {})),
    ("mean", "mean", lambda: ((_e(0),), {})),
]:
    _err(f"empty_{_name}", "fn", _fn, _b)
for _name, _cls, _b in [
    ("MulticlassAccuracy", "MulticlassAccuracy", lambda: ({}, [((_e(0, C), _ei(0)), {})])),
    ("MulticlassAccuracy_macro", "MulticlassAccuracy", lambda: ({"average": "macro", "num_classes": C}, [((_e(0, C), _ei(0)), {})])),
    ("BinaryAccuracy", "BinaryAccuracy", lambda: ({}, [((_e(0), _ei(0)), {})])),
    ("MultilabelAccuracy", "MultilabelAccuracy", lambda: ({}, [((_e(0, L), _ei(0, L)), {})])),
    ("MulticlassConfusionMatrix", "MulticlassConfusionMatrix", lambda: ({"num_classes": C}, [((_e(0, C), _ei(0)), {})])),
    ("MulticlassPrecision", "MulticlassPrecision", lambda: ({"num_classes": C, "average": None}, [((_e(0, C), _ei(0)), {})])),
    ("BinaryBinnedAUPRC", "BinaryBinnedAUPRC", lambda: ({"threshold": 5}, [((_e(0), _ei(0)), {})])),
    ("MulticlassBinnedAUPRC", "MulticlassBinnedAUPRC", lambda: ({"num_classes": C, "threshold": 5}, [((_e(0, C), _ei(0)), {})])),
    ("MeanSquaredError", "MeanSquaredError", lambda: ({}, [((_e(0), _e(0)), {})])),
    ("BinaryNormalizedEntropy", "BinaryNormalizedEntropy", lambda: ({}, [((_e(0), _e(0)), {})])),
    ("Perplexity", "Perplexity", lambda: ({}, [((_e(0, 4, 7), _ei(0, 4)), {})])),
    ("ClickThroughRate", "ClickThroughRate", lambda: ({}, [((_e(0),), {})])),
]:
    _err(f"empty_cls_{_name}", "cls", _cls, _b)


class _FlatFeatures(torch.nn.Module):
    """FID feature-model stand-in (the default Inception-v3 needs torchvision weights): the
    activations are the flattened images, so the covariance path sees real, varying data."""

    def forward(self, x):
        return x.flatten(1)


_ccase("FrechetInceptionDistance", "FrechetInceptionDistance",
       lambda: {"model": _FlatFeatures(), "feature_dim": 12},
       lambda s: ((_randn(_g(s), 32, 3, 1, 4) * (1.0 + 0.5 * ((s // 10) % 2)), bool((s // 10) % 2 == 0)), {}))
