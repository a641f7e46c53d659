"""FID compute building blocks on MI355X: FP64 eigvalsh / cholesky timings per linalg backend."""
import time

import torch

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
a = torch.randn(3000, 2048, device=dev, generator=g, dtype=torch.float64)
b = torch.randn(3000, 2048, device=dev, generator=g, dtype=torch.float64) * 1.1 + 0.2
s1, s2 = torch.cov(a.T), torch.cov(b.T)


def t(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


for lib in ("default", "cusolver", "magma"):
    try:
        torch.backends.cuda.preferred_linalg_library(lib)
    except Exception as e:  # noqa: BLE001
        print(lib, "unavailable", e)
        continue
    try:
        ms_e = t(lambda: torch.linalg.eigvalsh(s1))
        ms_c = t(lambda: torch.linalg.cholesky(s1))
        ms_e32 = t(lambda: torch.linalg.eigvalsh(s1.float()))
        print(f"{lib}: eigvalsh f64 {ms_e:.2f} ms, cholesky f64 {ms_c:.2f} ms, eigvalsh f32 {ms_e32:.2f} ms", flush=True)
    except Exception as e:  # noqa: BLE001
        print(lib, "failed", e)
torch.backends.cuda.preferred_linalg_library("default")
x = s1.cpu()
t0 = time.perf_counter()
torch.linalg.eigvalsh(x)
print(f"cpu eigvalsh f64 {1e3 * (time.perf_counter() - t0):.1f} ms ({torch.get_num_threads()} threads)")
