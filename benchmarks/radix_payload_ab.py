import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import profile, ProfilerActivity
from torcheval_amd.ops import native
n = 1 << 20
x = torch.rand(1, n, device="cuda")
t64 = torch.randint(0, 2, (1, n), device="cuda")
t32f = t64.float()
tu8 = t64.to(torch.uint8)
s = torch.empty_like(x); idx = torch.empty(1, n, dtype=torch.int32, device="cuda")
variants = {"iota": (None, 0), "i64": (t64, 1), "f32": (t32f, 1), "u8": (tu8, 1)}
for name, (p, k) in variants.items():
    for _ in range(5): native().sort_desc(x, s, idx, p, k)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(20): native().sort_desc(x, s, idx, p, k)
        torch.cuda.synchronize()
    print("####", name)
    for e in prof.key_averages():
        if "radix" in e.key:
            print(f"  {e.key[:70]:70s} {e.device_time:8.2f} us x{e.count}")
