"""FID compute with rank-deficient covariances (1000 + 1000 samples, D = 2048): K9p pivoted
Cholesky + K9b on the r x r product, against the round-5 eigh path.  Prints one JSON line."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.metrics.image.fid import (  # noqa: E402
    FrechetInceptionDistance,
    _eigh_factor,
    _pivoted_factor,
    _sqrt_eig_sum,
    _tr_sqrt_product,
)


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        v = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, v


dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(1000, 2048, device=dev, generator=g, dtype=torch.float64)
b = torch.randn(1000, 2048, device=dev, generator=g, dtype=torch.float64) * 1.1
s1, s2 = torch.cov(a.T), torch.cov(b.T)
s1, s2 = (s1 + s1.T) / 2, (s2 + s2.T) / 2
out = {}
out["k9p_factor_ms_fp64_standin"], w = timed(lambda: _pivoted_factor(s1))
out["rank_fp64_standin"] = int(w.shape[0])
out["tr_sqrt_ms_fp64_standin"], v = timed(lambda: _tr_sqrt_product(s1, s2, 1000, 1000))


def eigh_path():
    wf = _eigh_factor(s1)
    m = wf @ (s2 @ wf.T)
    return _sqrt_eig_sum((m + m.T) / 2)


out["tr_sqrt_ms_eigh_path"], ve = timed(eigh_path, reps=2)
out["tr_sqrt_rel_diff_vs_eigh"] = abs(float(v) - float(ve)) / abs(float(ve))

m = FrechetInceptionDistance(model=torch.nn.Identity(), feature_dim=2048, device=dev)
m.update_activations(a.float(), True).update_activations(b.float(), False)
out["fid_compute_ms_fp32_states"], fv = timed(m.compute)
out["fid_fp32_states"] = float(fv)
from torcheval_amd.metrics.image.fid import _covariance  # noqa: E402

c1 = _covariance(m.real_cov_sum, m.real_sum, 1000)
out["k9p_factor_ms_fp32_states"], w32 = timed(lambda: _pivoted_factor(c1))
out["rank_fp32_states"] = int(w32.shape[0])
print(json.dumps(out))
