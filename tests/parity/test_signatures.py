"""Signature parity with the reference for every public callable (hygiene item 7).

For each name in the reference's ``metrics.__all__`` / ``metrics.functional.__all__`` (classes:
``__init__`` and the ``update`` / ``compute`` / ``merge_state`` they define) and the public
functions / classes of ``metrics.toolkit``, ``metrics.synclib``, ``tools`` and
``utils.random_data``, every reference parameter must exist here with the same kind, default
and position.  Parameters the reference lacks are allowed only through ``ALLOWED_EXTRA`` (each
one a deliberate, documented addition); a changed default only through ``ALLOWED_DEFAULT``.
Private plumbing (an ``_err=`` argument and the like) therefore fails this test.
"""

import importlib
import inspect

import pytest

from tests.parity import _refload

pytestmark = pytest.mark.skipif(not _refload.available(), reason="reference not mounted")

# (qualified name, parameter): additions that are part of this package's documented API
ALLOWED_EXTRA = {
    # per-class one-vs-rest form of the binned multiclass AUROC (docs/parity.md)
    ("multiclass_binned_auroc", "one_vs_rest"),
    ("MulticlassBinnedAUROC.__init__", "one_vs_rest"),
    # c10d-style deadlines of the distributed toolkit (README "Failure semantics")
    ("metrics.toolkit.sync_and_compute", "timeout"),
    ("metrics.toolkit.sync_and_compute_collection", "timeout"),
    ("metrics.toolkit.get_synced_state_dict", "timeout"),
    ("metrics.toolkit.get_synced_state_dict_collection", "timeout"),
    ("metrics.toolkit.get_synced_metric", "timeout"),
    ("metrics.toolkit.get_synced_metric_collection", "timeout"),
}
# (qualified name, parameter): defaults deliberately different from the reference
ALLOWED_DEFAULT = {
    # the reference's constructor default k=1 with its hard-coded topk(k=2) crash
    ("TopKMultilabelAccuracy.__init__", "k"),
}
EXTRA_MODULES = ("metrics.toolkit", "metrics.synclib", "tools", "tools.flops", "tools.module_summary",
                 "utils.random_data")


def _params(f):
    try:
        return inspect.signature(f).parameters
    except (TypeError, ValueError):
        return None


def _same_default(a, b) -> bool:
    if a is b:
        return True
    try:
        return bool(a == b)
    except Exception:
        return False


def _diff(tag, ours, ref):
    po, pr = _params(ours), _params(ref)
    if po is None or pr is None:
        return []
    out = []
    for n, p in pr.items():
        q = po.get(n)
        if q is None:
            out.append(f"{tag}: missing parameter {n}")
            continue
        if q.kind != p.kind:
            out.append(f"{tag}: {n} is {q.kind}, reference {p.kind}")
        if not _same_default(q.default, p.default) and (tag, n) not in ALLOWED_DEFAULT:
            out.append(f"{tag}: {n} default {q.default!r}, reference {p.default!r}")
    for n in po:
        if n not in pr and (tag, n) not in ALLOWED_EXTRA:
            out.append(f"{tag}: extra parameter {n} (not in the reference, not allow-listed)")
    ours_order = [n for n in po if n in pr]
    if ours_order != list(pr):
        out.append(f"{tag}: parameter order {ours_order}, reference {list(pr)}")
    return out


def _pairs():
    RM, RF = _refload.load()
    import torcheval_amd.metrics as M
    import torcheval_amd.metrics.functional as F

    for mod, ref in ((F, RF), (M, RM)):
        for name in ref.__all__:
            r, o = getattr(ref, name), getattr(mod, name)
            if inspect.isclass(r):
                yield f"{name}.__init__", o.__init__, r.__init__
                for meth in ("update", "compute", "merge_state"):
                    if meth in r.__dict__:
                        yield f"{name}.{meth}", getattr(o, meth), getattr(r, meth)
            elif callable(r):
                yield name, o, r
    for modname in EXTRA_MODULES:
        r = importlib.import_module("torcheval." + modname)
        o = importlib.import_module("torcheval_amd." + modname)
        names = getattr(r, "__all__", None) or [
            n for n, v in vars(r).items()
            if not n.startswith("_") and (inspect.isfunction(v) or inspect.isclass(v))
            and getattr(v, "__module__", "") == r.__name__
        ]
        for name in names:
            rv, ov = getattr(r, name), getattr(o, name, None)
            assert ov is not None, f"torcheval_amd.{modname}.{name} is absent"
            if inspect.isclass(rv):
                yield f"{modname}.{name}.__init__", ov.__init__, rv.__init__
            elif callable(rv):
                yield f"{modname}.{name}", ov, rv


def test_every_public_signature_matches_the_reference():
    problems, n = [], 0
    for tag, ours, ref in _pairs():
        n += 1
        problems += _diff(tag, ours, ref)
    assert n > 150, n
    assert not problems, "\n".join(problems)


def test_allow_lists_are_live():
    """Every allow-list entry still names a real difference (stale entries hide nothing)."""
    extra, default = set(), set()
    for tag, ours, ref in _pairs():
        po, pr = _params(ours), _params(ref)
        if po is None or pr is None:
            continue
        extra |= {(tag, n) for n in po if n not in pr}
        default |= {(tag, n) for n, p in pr.items() if n in po and not _same_default(po[n].default, p.default)}
    assert ALLOWED_EXTRA <= extra, ALLOWED_EXTRA - extra
    assert ALLOWED_DEFAULT <= default, ALLOWED_DEFAULT - default
