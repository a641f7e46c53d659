"""K9b timing: eigenvalues of a symmetric FP64 D x D matrix (native vs rocSOLVER eigvalsh) and
the FID compute built on it.  Prints one JSON line."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd.metrics.image.fid import frechet_distance
from torcheval_amd.ops import native


def _time(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return min(out), sorted(out)[len(out) // 2]


def main() -> None:
    dev = "cuda"
    res = {}
    for d in (512, 1000, 2048):
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(d, d + 100, device=dev, dtype=torch.float64, generator=g)
        m = x @ x.T / x.shape[1]
        lam = torch.empty(d, dtype=torch.float64, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        nat = _time(lambda: native().sym_eigvals(m, lam, st))
        roc = _time(lambda: torch.linalg.eigvalsh(m))
        err = float((lam - torch.linalg.eigvalsh(m)).abs().max() / m.diagonal().abs().max())
        res[f"eig_d{d}"] = {"k9b_ms_min_med": nat, "rocsolver_ms_min_med": roc, "status": int(st.item()),
                            "max_abs_err_rel": err}
    d = 2048
    g = torch.Generator(device=dev).manual_seed(1)
    a1 = torch.randn(4000, d, device=dev, generator=g)
    a2 = torch.randn(4000, d, device=dev, generator=g) * 1.1
    s1, s2 = torch.cov(a1.T.double()), torch.cov(a2.T.double())
    mu1, mu2 = a1.double().mean(0), a2.double().mean(0)
    res["fid_compute_d2048_ms_min_med"] = _time(lambda: frechet_distance(mu1, s1, mu2, s2).item())
    # where the rest of the compute goes: the blocked Cholesky (K9c diagonal blocks + GEMMs),
    # one K9c diagonal block alone, and the two triangular products
    from torcheval_amd.metrics.image.fid import cholesky_ex

    res["cholesky_d2048_ms_min_med"] = _time(lambda: cholesky_ex(s1)[1].item())
    res["rocsolver_cholesky_d2048_ms_min_med"] = _time(lambda: torch.linalg.cholesky_ex(s1)[1].item())
    blk = s1[:64, :64].contiguous()
    linv = torch.empty(64 * 64, dtype=torch.float64, device=dev)
    info = torch.zeros(1, dtype=torch.int32, device=dev)

    def _blocks(reps=32):
        for _ in range(reps):
            native().potrf_block(blk.clone(), 0, 64, linv, info)
        torch.cuda.synchronize()

    ms = _time(_blocks)
    res["k9c_block64_us_min_med"] = [ms[0] * 1e3 / 32, ms[1] * 1e3 / 32]
    L = cholesky_ex(s1)[0]
    res["lt_s2_l_d2048_ms_min_med"] = _time(lambda: (L.T @ s2 @ L).sum().item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
