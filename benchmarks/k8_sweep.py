"""K8 (FID covariance SYRK) vs the library GEMM over batch sizes / feature dims / split-K.

    python benchmarks/k8_sweep.py [--d 2048 768] [--k 1000 50000] [--splits 0 1 2 3] [--modes x3 exact]

split 0 = the launcher's own choice; mode x3 = bf16 MFMA on the exact three-way split staged
once per block (the default), x3w = the same split done per wave (``TORCHEVAL_AMD_K8_MODE=1``),
exact = FP32 MFMA (``TORCHEVAL_AMD_K8_EXACT=1``).  Prints one JSON line per (D, K, split): K8 time, the
rocBLAS/hipBLASLt ``act.T @ act`` time, the effective FP32-MFMA rate of K8 on the
upper-triangle FLOPs it does (96 x 96 tiles, diagonal tiles full), and the max relative error
against an fp64 product of the same activations."""

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.ops import native  # noqa: E402


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--d", type=int, nargs="+", default=[2048])
    ap.add_argument("--k", type=int, nargs="+", default=[128, 1000, 4096, 50000])
    ap.add_argument("--splits", type=int, nargs="+", default=[0])
    ap.add_argument("--modes", nargs="+", default=["x3", "x3w", "exact"])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = []
    for D in args.d:
        T = (D + 95) // 96
        for K in args.k:
            act = torch.randn(K, D, device="cuda")
            out = torch.empty(D, D, device="cuda")
            t_mm = timeit(lambda: torch.mm(act.T, act, out=out))
            cacc, sacc = torch.zeros(D, D, device="cuda"), torch.zeros(D, device="cuda")

            def lib_update():  # what the metric update would run on the library path
                cacc.addmm_(act.T, act)
                sacc.add_(act.sum(0))

            t_lib = timeit(lib_update)
            ref = act.double().T @ act.double()
            for mode, sp in [(m, sp) for m in args.modes for sp in args.splits]:
                os.environ.pop("TORCHEVAL_AMD_K8_EXACT", None)
                os.environ.pop("TORCHEVAL_AMD_K8_MODE", None)
                if mode == "exact":
                    os.environ["TORCHEVAL_AMD_K8_EXACT"] = "1"
                elif mode == "x3w":
                    os.environ["TORCHEVAL_AMD_K8_MODE"] = "1"
                if sp > 0:
                    os.environ["TORCHEVAL_AMD_K8_SPLIT"] = str(sp)
                else:
                    os.environ.pop("TORCHEVAL_AMD_K8_SPLIT", None)
                cov = torch.zeros(D, D, device="cuda")
                cs = torch.zeros(D, device="cuda")
                native().fid_cov_update(act, cov, cs)
                err = float(((cov.double() - ref).abs().max() / ref.abs().max()).item())
                t_k8 = timeit(lambda: native().fid_cov_update(act, cov, cs))
                flops_tri = 2.0 * K * 96 * 96 * T * (T + 1) / 2
                row = {"D": D, "K": K, "mode": mode, "split": sp, "k8_us": round(t_k8, 2), "gemm_us": round(t_mm, 2),
                       "speedup_vs_gemm": round(t_mm / t_k8, 2), "lib_update_us": round(t_lib, 2),
                       "speedup_vs_lib_update": round(t_lib / t_k8, 2), "k8_tflops_tri": round(flops_tri / t_k8 / 1e6, 1),
                       "gemm_tflops": round(2.0 * K * D * D / t_mm / 1e6, 1), "max_rel_err": err}
                rows.append(row)
                print(json.dumps(row), flush=True)
    os.environ.pop("TORCHEVAL_AMD_K8_SPLIT", None)
    os.environ.pop("TORCHEVAL_AMD_K8_EXACT", None)
    os.environ.pop("TORCHEVAL_AMD_K8_MODE", None)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
