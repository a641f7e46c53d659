"""K7 perplexity kernel time per shape (GPU events, median of 50), for A/B of the row-block
kernel against the wave-per-row kernel (TORCHEVAL_AMD_PPL_ROWBLOCK=0).  Prints one JSON object:
{shape: {"us": t, "tb_s": logits bytes / t}}."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.ops import native  # noqa: E402

SHAPES = [
    (4096, 32000, torch.float32),
    (4096, 32000, torch.bfloat16),
    (16384, 32000, torch.bfloat16),
    (2048, 128256, torch.bfloat16),
    (4096, 50257, torch.float32),  # not 16-aligned: wave-per-row scalar path in both arms
    (65536, 4096, torch.float32),
    (8192, 1024, torch.float32),  # short rows: wave-per-row in both arms
]


def main() -> None:
    dev = torch.device("cuda", 0)
    out = {}
    for rows, v, dt in SHAPES:
        x = torch.randn(rows, v, device=dev).to(dt)
        t = torch.randint(0, v, (rows,), device=dev)
        acc = torch.zeros(2, dtype=torch.float64, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(5):
            native().perplexity_sums(x, t, None, acc, flag, False)
        ts = []
        for _ in range(50):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            native().perplexity_sums(x, t, None, acc, flag, False)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        us = statistics.median(ts)
        out[f"{rows}x{v} {str(dt).split('.')[-1]}"] = {"us": round(us, 1), "tb_s": round(x.numel() * x.element_size() / us / 1e6, 2)}
        del x
    print(json.dumps(out))


if __name__ == "__main__":
    main()
