"""K9p phase trace at D = 2048, rank 999 (1000-sample FP64 covariance): per-panel wall times of
workgroup 0's panel factorisation and workgroup 1's update, plus panel 2's per-step cycles."""
import json
import sys
import time

sys.path.insert(0, __file__.rsplit("/benchmarks/", 1)[0])
import torch  # noqa: E402

from torcheval_amd.ops import native  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(1000, 2048, device=dev, generator=g, dtype=torch.float64)
s = torch.cov(x.T)
s = (s + s.T) / 2
nat = native()
N = nat.pivchol_padded(2048)
slots = torch.empty(nat.pivchol_slot_words(2048), dtype=torch.int64, device=dev)
w = torch.empty(N, N, dtype=torch.float64, device=dev)
piv = torch.empty(2048, dtype=torch.int32, device=dev)
info = torch.empty(2, dtype=torch.int32, device=dev)
ctl = torch.empty(1, dtype=torch.int32, device=dev)
tr = torch.zeros(80, dtype=torch.int64, device=dev)
for _ in range(3):
    tr.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    nat.pivchol_traced(s, slots, w, piv, info, ctl, tr)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
t = tr.cpu().tolist()
us = lambda a, b: round((b - a) / 100.0, 2)  # noqa: E731
steps = {f"P{P}k{k}": {"round_start_to_stored": us(t[2 * (8 * P + k)], t[2 * (8 * P + k) + 1]),
                       "stored_to_next_round": us(t[2 * (8 * P + k) + 1], t[2 * (8 * P + k + 1)]) if k < 7 else None}
         for P in range(3) for k in range(8)}
upd = {f"P{P}": us(t[64 + 2 * P], t[64 + 2 * P + 1]) for P in range(3)}
print(json.dumps({"info": info.cpu().tolist(), "wall_ms": round(wall, 3), "update_us": upd, "steps_us": steps}))
