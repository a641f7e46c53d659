"""Generate ``golden.pt``: the reference's outputs on every case in ``cases.py``.

Run from the repo root with the reference mounted (CPU only, a few seconds)::

    python tests/parity/gen_goldens.py

The file holds only tensors / lists / tuples / numbers / strings, so the tests load it with
``torch.load(weights_only=True)``.
"""

import os
import sys
import warnings

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import _refload  # noqa: E402
import cases  # noqa: E402


def plain(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().clone().cpu()
    if isinstance(obj, tuple):
        return tuple(plain(o) for o in obj)
    if isinstance(obj, list):
        return [plain(o) for o in obj]
    if isinstance(obj, (int, float, bool, str)) or obj is None:
        return obj
    raise TypeError(f"unsupported output type {type(obj)}")


def run_guarded(fn):
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return plain(fn())
    except Exception as e:  # the reference's exception is itself the expected behaviour
        return {"__raise__": type(e).__name__, "msg": str(e)}


def run_updates(m, updates):
    for args, kwargs in updates:
        m.update(*args, **kwargs)
    return m.compute() if updates else None


def run_class(M, cls_name, ctor, updates, merged):
    cls = getattr(M, cls_name)
    if not merged:
        m = cls(**ctor())
        for args, kwargs in updates:
            m.update(*args, **kwargs)
        return m.compute()
    half = len(updates) // 2
    a, b = cls(**ctor()), cls(**ctor())
    for args, kwargs in updates[:half]:
        a.update(*args, **kwargs)
    for args, kwargs in updates[half:]:
        b.update(*args, **kwargs)
    a.merge_state([b])
    return a.compute()


def main() -> None:
    M, F = _refload.load()
    torch.manual_seed(0)
    out = {"functional": {}, "class": {}}
    for cid, (fn, builder) in cases.FUNCTIONAL.items():
        args, kwargs = builder(cases.cid_seed(cid))
        out["functional"][cid] = run_guarded(lambda: getattr(F, fn)(*args, **kwargs))
    for cid, (cls_name, ctor, upd) in cases.CLASS.items():
        updates = upd(cases.cid_seed(cid))
        out["class"][cid] = {
            "full": run_guarded(lambda: run_class(M, cls_name, ctor, updates, False)),
            "merged": run_guarded(lambda: run_class(M, cls_name, ctor, updates, True)),
        }
    out["errors"] = {}
    for cid, (kind, name, builder) in cases.ERRORS.items():
        if kind == "fn":
            args, kwargs = builder()
            out["errors"][cid] = run_guarded(lambda: getattr(F, name)(*args, **kwargs))
        else:
            ctor, updates = builder()
            out["errors"][cid] = run_guarded(lambda: run_updates(getattr(M, name)(**ctor), updates))
    path = os.path.join(HERE, "golden.pt")
    torch.save(out, path)
    nraise = sum(isinstance(v, dict) for v in out["functional"].values())
    print(f"wrote {path}: {len(out['functional'])} functional ({nraise} raising), "
          f"{len(out['class'])} class cases, "
          f"{sum(isinstance(v, dict) for v in out['errors'].values())}/{len(out['errors'])} error cases raise")
    for cid, v in out["errors"].items():
        if not isinstance(v, dict):
            print("  reference does not raise:", cid)


if __name__ == "__main__":
    main()
