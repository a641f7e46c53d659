"""In-tree build of the native extension ``torcheval_amd/_C.so`` (gfx950 only).

No ``torch.utils.cpp_extension.CUDAExtension`` (it would hipify sources): HIP kernels are
compiled directly with ``hipcc --offload-arch=gfx950``; the pybind/torch glue and the C++
runtime with ``g++``; everything is linked against the HIP runtime that ships inside torch
(``torch/lib/libamdhip64.so``, same soname as /opt/rocm's) so a single runtime is loaded.

Incremental: each object is rebuilt only when its source, the shared headers or the flags
change (content hash stored next to the object).  Usage::

    python -m torcheval_amd.ops.build [--force] [--jobs N] [--verbose]
"""

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import List, Tuple

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(REPO, "csrc")
BUILD = os.path.join(REPO, "build", "native")
OUT = os.path.join(REPO, "torcheval_amd", "_C.so")
ARCH = os.environ.get("TORCHEVAL_AMD_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

TORCH_DIR = os.path.dirname(torch.__file__)
TORCH_INC = [
    os.path.join(TORCH_DIR, "include"),
    os.path.join(TORCH_DIR, "include", "torch", "csrc", "api", "include"),
]
TORCH_LIB = os.path.join(TORCH_DIR, "lib")
PY_INC = sysconfig.get_paths()["include"]
ABI = int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    return p


def _sources() -> List[Tuple[str, str]]:
    out = []
    for sub, kind in (("kernels", "hip"), ("runtime", "cxx")):
        d = os.path.join(CSRC, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith(".hip") or f.endswith(".cpp"):
                out.append((os.path.join(d, f), "hip" if f.endswith(".hip") else "cxx"))
    out.append((os.path.join(CSRC, "bindings.cpp"), "torch"))
    return out


def _headers_digest() -> str:
    h = hashlib.sha256()
    inc = os.path.join(CSRC, "include")
    for f in sorted(os.listdir(inc)):
        with open(os.path.join(inc, f), "rb") as fh:
            h.update(f.encode())
            h.update(fh.read())
    return h.hexdigest()


def _flags(kind: str) -> List[str]:
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{os.path.join(CSRC, 'include')}"]
    if kind == "hip":
        return [_hipcc(), "-x", "hip", f"--offload-arch={ARCH}", "-ffp-contract=fast"] + common
    base = ["g++"] + common + [
        f"-I{PY_INC}",
        f"-I{os.path.join(ROCM, 'include')}",
        "-D__HIP_PLATFORM_AMD__=1",
        "-DUSE_ROCM=1",
        f"-D_GLIBCXX_USE_CXX11_ABI={ABI}",
        "-Wno-deprecated-declarations",
    ]
    base += [f"-I{p}" for p in TORCH_INC]
    if kind == "torch":
        base += ["-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H"]
    return base


def _compile(src: str, kind: str, hdr: str, force: bool, verbose: bool) -> str:
    os.makedirs(BUILD, exist_ok=True)
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    cmd = _flags(kind) + ["-c", src, "-o", obj]
    with open(src, "rb") as fh:
        digest = hashlib.sha256(fh.read() + hdr.encode() + " ".join(cmd).encode()).hexdigest()
    stamp = obj + ".sha"
    if not force and os.path.exists(obj) and os.path.exists(stamp):
        with open(stamp) as fh:
            if fh.read().strip() == digest:
                return obj
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    with open(stamp, "w") as fh:
        fh.write(digest)
    return obj


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    """Compile every native source for gfx950 and link ``torcheval_amd/_C.so``."""
    srcs = _sources()
    hdr = _headers_digest()
    jobs = jobs or min(8, os.cpu_count() or 4, len(srcs))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s[0], s[1], hdr, force, verbose), srcs))
    link = [
        _hipcc(),
        f"--offload-arch={ARCH}",
        "-shared",
        "-fPIC",
        *objs,
        "-o",
        OUT + ".tmp",
        f"-L{TORCH_LIB}",
        "-lc10",
        "-lc10_hip",
        "-ltorch",
        "-ltorch_cpu",
        "-ltorch_hip",
        "-ltorch_python",
        "-lamdhip64",
        f"-Wl,-rpath,{TORCH_LIB}",
    ]
    newest = max(os.path.getmtime(o) for o in objs)
    if force or not os.path.exists(OUT) or os.path.getmtime(OUT) < newest:
        if verbose:
            print(" ".join(link), flush=True)
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{' '.join(link)}\n{r.stdout}\n{r.stderr}")
        os.replace(OUT + ".tmp", OUT)
    return OUT


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    args = ap.parse_args(argv)
    out = build(force=args.force, jobs=args.jobs, verbose=args.verbose)
    print(out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
