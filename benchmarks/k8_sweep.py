"""K8 (FID covariance SYRK) vs the library GEMM over batch sizes, D = 2048, fp32.

Prints one JSON line per K: K8 time, rocBLAS/hipBLASLt ``act.T @ act`` time, and the
effective FP32-MFMA rate of K8 on the upper-triangle FLOPs it actually does."""

import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
from torcheval_amd.ops import native  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
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
    D = 2048
    T = D // 64
    for K in [int(a) for a in (sys.argv[1:] or ["128", "512", "1000", "2048", "4096", "8192"])]:
        act = torch.randn(K, D, device="cuda")
        cov = torch.zeros(D, D, device="cuda")
        cs = torch.zeros(D, device="cuda")
        t_k8 = timeit(lambda: native().fid_cov_update(act, cov, cs))
        out = torch.empty(D, D, device="cuda")
        t_mm = timeit(lambda: torch.mm(act.T, act, out=out))
        flops_tri = 2.0 * K * 64 * 64 * T * (T + 1) / 2
        print(json.dumps({"K": K, "k8_us": round(t_k8, 2), "gemm_us": round(t_mm, 2),
                          "k8_tflops_tri": round(flops_tri / t_k8 / 1e6, 1),
                          "gemm_tflops": round(2.0 * K * D * D / t_mm / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
