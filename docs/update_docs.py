"""Docs build pipeline: Sphinx autosummary pages + an offline HTML reference.

The single source of truth is each sub-package's ``__all__`` (order = page order) and
``__doc_name__`` (section title), the same contract as the reference's docs/update_docs.py.

    python docs/update_docs.py                 # regenerate docs/source/*.rst (commit them)
    python docs/update_docs.py --check         # exit 1 if the committed pages are stale (CI)
    python docs/update_docs.py --html OUT_DIR  # offline HTML reference (no Sphinx needed)
    make -C docs html                          # the Sphinx build (docs/requirements.txt)

The .rst pages are what Sphinx renders (``docs/source/conf.py``: autodoc + autosummary +
napoleon); the ``--html`` renderer walks the same page model with ``inspect`` so the reference
can be built and link-checked on machines without Sphinx (this image has none).
"""

import argparse
import html
import importlib
import inspect
import os
import sys
from typing import Dict, List, Tuple

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCE = os.path.join(ROOT, "docs", "source")
sys.path.insert(0, ROOT)

# page -> (title, intro, sections: list of package names whose __all__ forms one section)
PAGES: Dict[str, Tuple[str, str, List[str]]] = {
    "torcheval_amd.metrics": (
        "Metrics",
        "Stateful metric classes (``update`` / ``compute`` / ``merge_state`` / ``state_dict``).",
        [
            "torcheval_amd.metrics.metric",
            "torcheval_amd.metrics.aggregation",
            "torcheval_amd.metrics.classification",
            "torcheval_amd.metrics.image",
            "torcheval_amd.metrics.ranking",
            "torcheval_amd.metrics.regression",
            "torcheval_amd.metrics.text",
            "torcheval_amd.metrics.window",
        ],
    ),
    "torcheval_amd.metrics.functional": (
        "Functional Metrics",
        "Stateless functions; ROCm tensors run the HIP/CDNA4 kernels, CPU tensors the ATen path.",
        [
            "torcheval_amd.metrics.functional.aggregation",
            "torcheval_amd.metrics.functional.classification",
            "torcheval_amd.metrics.functional.image",
            "torcheval_amd.metrics.functional.ranking",
            "torcheval_amd.metrics.functional.regression",
            "torcheval_amd.metrics.functional.text",
        ],
    ),
    "torcheval_amd.metrics.toolkit": (
        "Metric Toolkit",
        "Distributed sync (typed RCCL engine), cloning, device moves.",
        ["torcheval_amd.metrics.toolkit"],
    ),
    "torcheval_amd.parallel": (
        "Parallel (RCCL)",
        "Device-resident collectives, class-sharded and sample-sharded computes.",
        ["torcheval_amd.parallel"],
    ),
    "torcheval_amd.tools": (
        "Tools",
        "FLOP counting and module summaries.",
        ["torcheval_amd.tools"],
    ),
}


def package_symbols(name: str) -> Tuple[str, List[str]]:
    """(section title, public names in __all__ order) of one package."""
    mod = importlib.import_module(name)
    title = getattr(mod, "__doc_name__", None) or name.rsplit(".", 1)[-1].replace("_", " ").title()
    names = list(getattr(mod, "__all__", []))
    if not names:
        names = sorted(
            n for n, o in vars(mod).items()
            if not n.startswith("_") and (inspect.isfunction(o) or inspect.isclass(o)) and o.__module__ == name
        )
    return title, names


def render_rst(page: str) -> str:
    title, intro, sections = PAGES[page]
    out = [title, "=" * len(title), "", f".. automodule:: {page}", "", intro, ""]
    for pkg in sections:
        sec_title, names = package_symbols(pkg)
        if len(sections) > 1:
            out += [sec_title, "-" * len(sec_title), ""]
        out += [f".. currentmodule:: {pkg}", "", ".. autosummary::", "   :toctree: generated", "   :nosignatures:", ""]
        out += [f"   {n}" for n in names]
        out.append("")
    return "\n".join(out)


def render_index() -> str:
    lines = [
        "torcheval_amd",
        "=============",
        "",
        "MI355X-native model-evaluation metrics: PyTorch-ROCm, hand-written HIP/CDNA4 kernels and",
        "RCCL over xGMI, with the API of torcheval.",
        "",
        ".. toctree::",
        "   :maxdepth: 2",
        "   :caption: API Reference",
        "",
    ]
    lines += [f"   {page}" for page in PAGES]
    return "\n".join(lines) + "\n"


def generate() -> Dict[str, str]:
    files = {"index.rst": render_index()}
    for page in PAGES:
        files[f"{page}.rst"] = render_rst(page)
    return files


def write(files: Dict[str, str]) -> None:
    os.makedirs(SOURCE, exist_ok=True)
    for fn, text in files.items():
        with open(os.path.join(SOURCE, fn), "w") as f:
            f.write(text)


def check(files: Dict[str, str]) -> List[str]:
    stale = []
    for fn, text in files.items():
        path = os.path.join(SOURCE, fn)
        if not os.path.exists(path) or open(path).read() != text:
            stale.append(fn)
    return stale


def _sig(obj) -> str:
    try:
        return str(inspect.signature(obj))
    except (TypeError, ValueError):
        return ""


def render_html(out_dir: str) -> List[str]:
    """Offline HTML reference: one page per PAGES entry, one anchor per symbol, the full
    docstring of each (and of each public method of classes).  Returns the written files."""
    os.makedirs(out_dir, exist_ok=True)
    written = []
    nav = "".join(f'<li><a href="{p}.html">{html.escape(PAGES[p][0])}</a></li>' for p in PAGES)
    style = ("body{font-family:sans-serif;max-width:60em;margin:auto}pre{background:#f4f4f4;padding:.5em;"
             "white-space:pre-wrap}h3{border-top:1px solid #ccc;padding-top:.5em}")
    for page, (title, intro, sections) in PAGES.items():
        body = [f"<h1>{html.escape(title)}</h1><p>{html.escape(intro)}</p>"]
        for pkg in sections:
            sec_title, names = package_symbols(pkg)
            mod = importlib.import_module(pkg)
            body.append(f"<h2>{html.escape(sec_title)} <code>{pkg}</code></h2>")
            for n in names:
                obj = getattr(mod, n)
                kind = "class" if inspect.isclass(obj) else "function"
                body.append(f'<h3 id="{pkg}.{n}">{kind} <code>{html.escape(n + _sig(obj))}</code></h3>')
                body.append(f"<pre>{html.escape(inspect.getdoc(obj) or '')}</pre>")
                if inspect.isclass(obj):
                    for mname in ("update", "compute", "merge_state", "reset", "state_dict", "load_state_dict", "to"):
                        meth = getattr(obj, mname, None)
                        if meth is not None and mname in obj.__dict__:
                            body.append(f"<h4><code>{html.escape(mname + _sig(meth))}</code></h4>")
                            body.append(f"<pre>{html.escape(inspect.getdoc(meth) or '')}</pre>")
        doc = (f"<!doctype html><html><head><meta charset='utf-8'><title>{html.escape(title)}</title>"
               f"<style>{style}</style></head><body><ul>{nav}</ul>{''.join(body)}</body></html>")
        path = os.path.join(out_dir, f"{page}.html")
        with open(path, "w") as f:
            f.write(doc)
        written.append(path)
    index = os.path.join(out_dir, "index.html")
    with open(index, "w") as f:
        f.write(f"<!doctype html><html><head><meta charset='utf-8'><title>torcheval_amd</title></head>"
                f"<body><h1>torcheval_amd API</h1><ul>{nav}</ul></body></html>")
    written.append(index)
    return written


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true", help="fail if docs/source is stale")
    ap.add_argument("--html", default=None, help="also render an offline HTML reference here")
    args = ap.parse_args()
    files = generate()
    if args.check:
        stale = check(files)
        if stale:
            print("stale docs pages (run python docs/update_docs.py):", ", ".join(stale))
            sys.exit(1)
        print("docs pages up to date")
    else:
        write(files)
        print(f"wrote {len(files)} pages to {SOURCE}")
    if args.html:
        print(f"wrote {len(render_html(args.html))} HTML pages to {args.html}")


if __name__ == "__main__":
    main()
