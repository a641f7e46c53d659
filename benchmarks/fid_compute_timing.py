"""FID compute at D = 2048, component by component (round 6): the covariance pass, the K9d
one-launch Cholesky, the triangle-aware L^T S2 L, the K9b eigenvalues, ``frechet_distance`` and
``FrechetInceptionDistance.compute`` from states - each against the form it replaced.  Prints
one JSON line (min / median ms over reps, each rep synchronised)."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd.metrics.image import fid as F  # noqa: E402


def _time(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    return [round(min(out), 4), round(sorted(out)[len(out) // 2], 4)]


def main() -> None:
    dev = "cuda"
    d = 2048
    res = {}
    g = torch.Generator(device=dev).manual_seed(1)
    m = F.FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=d, device=dev)
    for real in (True, False):
        m.update_activations(torch.randn(4 * d, d, device=dev, generator=g) * (1.0 if real else 1.1), real)
    nr = int(m.num_real_images)
    cs, sm = m.real_cov_sum, m.real_sum
    res["covariance_pass_ms"] = _time(lambda: F._covariance(cs, sm, nr))
    mean = sm.double() / nr
    res["covariance_aten_chain_ms"] = _time(
        lambda: (lambda c: (c + c.T) / 2)((cs.double() - nr * torch.outer(mean, mean)) / (nr - 1)))
    s1 = F._covariance(m.real_cov_sum, m.real_sum, nr)
    s2 = F._covariance(m.fake_cov_sum, m.fake_sum, int(m.num_fake_images))
    res["cholesky_k9d_ms"] = _time(lambda: F._chol(s1))
    res["cholesky_rocsolver_ms"] = _time(lambda: torch.linalg.cholesky_ex(s1)[1].item())
    L, info = F._chol(s1)
    ref = torch.linalg.cholesky(s1)
    res["cholesky_max_rel_err"] = float((L - ref).abs().max() / ref.abs().max())
    res["cholesky_info"] = info
    res["sandwich_triangle_aware_ms"] = _time(lambda: F._lt_s_l(L, s2))
    for pp in (2, 3, 8):
        os.environ["TORCHEVAL_AMD_FID_SANDWICH_P"] = str(pp)
        res[f"sandwich_p{pp}_ms"] = _time(lambda: F._lt_s_l(L, s2))
    os.environ.pop("TORCHEVAL_AMD_FID_SANDWICH_P")
    # the p = 4 GEMMs one by one (shape, ms)
    b = 512
    yt = torch.empty(d, d, dtype=torch.float64, device=dev)
    mm = torch.empty(d, d, dtype=torch.float64, device=dev)
    for c0 in range(0, d, b):
        res[f"gemm_yt_c{c0}_ms"] = _time(lambda: torch.mm(L[c0:, c0:c0 + b].T, s2[c0:, :], out=yt[c0:c0 + b]))
    for r0 in range(0, d, b):
        res[f"gemm_m_r{r0}_ms"] = _time(lambda: torch.mm(L[r0:, r0:r0 + b].T, yt[:r0 + b, r0:].T, out=mm[r0:r0 + b, :r0 + b]))
    res["gemm_dense_2048_ms"] = _time(lambda: torch.mm(s2, L, out=yt))
    # K9d scaling with the tile count (critical chain per tile column)
    for n in (64, 128, 256, 512, 1024):
        res[f"cholesky_k9d_n{n}_ms"] = _time(lambda: F._chol(s1[:n, :n]))
    res["sandwich_dense_ms"] = _time(lambda: (L.T @ s2 @ L))
    mm = F._lt_s_l(L, s2)
    dense = L.T @ s2 @ L
    res["sandwich_max_rel_err"] = float((mm - dense).abs().max() / dense.abs().max())
    res["eigvals_k9b_ms"] = _time(lambda: F.sym_eigvalsh(mm))
    mu1, mu2 = m.real_sum.double() / nr, m.fake_sum.double() / int(m.num_fake_images)
    res["frechet_distance_ms"] = _time(lambda: F.frechet_distance(mu1, s1, mu2, s2).item())
    res["fid_compute_from_states_ms"] = _time(lambda: m.compute().item())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
