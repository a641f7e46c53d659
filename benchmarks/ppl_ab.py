"""K7 perplexity kernel time per shape (GPU events, median of PPL_AB_REPS, default 50), for A/B
of the launch knobs (TORCHEVAL_AMD_PPL_MAXGRID, TORCHEVAL_AMD_PPL_U2).  Prints one JSON object:
{shape: {"us": t, "tb_s": logits bytes / t}}.  With PPL_AB_REPS=n each shape makes 1 + n
launches in order (a counter pass maps dispatches to shapes by that order)."""
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
    (4096, 50257, torch.float32),  # rows not 16-B aligned: scalar head / 16-B body / scalar tail
    (65536, 4096, torch.float32),
    (8192, 1024, torch.float32),  # short rows
]


def main() -> None:
    dev = torch.device("cuda", 0)
    reps = int(os.environ.get("PPL_AB_REPS", "50"))
    warm = 5 if reps >= 10 else 1
    out = {}
    for rows, v, dt in SHAPES:
        x = torch.randn(rows, v, device=dev).to(dt)
        t = torch.randint(0, v, (rows,), device=dev)
        acc = torch.zeros(2, dtype=torch.float64, device=dev)
        flag = torch.zeros(1, dtype=torch.int32, device=dev)
        for _ in range(warm):
            native().perplexity_sums(x, t, None, acc, flag, False)
        ts = []
        for _ in range(reps):
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
