"""K4 binned-histogram update throughput over (n, C, T) shapes, incl. class-chunked dense cases."""
import torch, time, sys
sys.path.insert(0, ".")
from torcheval_amd import metrics as M
dev = torch.device("cuda", 0)
def rate(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3
for n, C, T in [(100_000, 100, 100), (100_000, 1000, 100), (20_000, 1000, 200), (1_000_000, 10, 100), (100_000, 100, 1000)]:
    x = torch.rand(n, C, device=dev); y = torch.randint(0, C, (n,), device=dev)
    m = M.MulticlassBinnedAUPRC(num_classes=C, threshold=T, device=dev)
    ms = rate(lambda: m.update(x, y))
    print(f"n={n} C={C} T={T}: {ms:.3f} ms/update, {n*C*4/ms/1e9:.2f} TB/s of scores")
