"""K5 A/B: the one-launch column-moments kernel (v2) under its tile geometries against the
two-launch v1 kernel (TORCHEVAL_AMD_K5_V2=0), per-update device time (events around 200
updates over a 4-batch pool) of MeanSquaredError / R2Score updates and the fused functional
mean_squared_error / r2_score at 8192 rows x {1000, 1001, 4096, 4097} fp32.  One JSON line
per configuration; the geometry knobs are read per call (TORCHEVAL_AMD_K5_CG / _BLOCKS /
_MAXR)."""
import json
import os
import sys

os.environ["TORCHEVAL_AMD_AB_DYNAMIC"] = "1"  # the K5 knobs are re-read per call

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.metrics import MeanSquaredError, R2Score  # noqa: E402
from torcheval_amd.metrics.functional import mean_squared_error, r2_score  # noqa: E402


def _per_call_us(fn, n=200):
    for i in range(10):
        fn(i)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


CONFIGS = [
    {"TORCHEVAL_AMD_K5_V2": "0"},
    {},
    {"TORCHEVAL_AMD_K5_CG": "16", "TORCHEVAL_AMD_K5_BLOCKS": "256"},
    {"TORCHEVAL_AMD_K5_CG": "16", "TORCHEVAL_AMD_K5_BLOCKS": "256", "TORCHEVAL_AMD_K5_PIPE": "0"},
    {"TORCHEVAL_AMD_K5_CG": "16", "TORCHEVAL_AMD_K5_BLOCKS": "512"},
    {"TORCHEVAL_AMD_K5_CG": "64", "TORCHEVAL_AMD_K5_BLOCKS": "256"},
    {"TORCHEVAL_AMD_K5_CG": "64", "TORCHEVAL_AMD_K5_BLOCKS": "512"},
    {"TORCHEVAL_AMD_K5_CG": "16", "TORCHEVAL_AMD_K5_BLOCKS": "256", "TORCHEVAL_AMD_K5_AB_SKIP_FOLD": "1"},
    {"TORCHEVAL_AMD_K5_CG": "64", "TORCHEVAL_AMD_K5_BLOCKS": "256", "TORCHEVAL_AMD_K5_AB_SKIP_FOLD": "1"},
    {"TORCHEVAL_AMD_K5_CG": "64", "TORCHEVAL_AMD_K5_BLOCKS": "512", "TORCHEVAL_AMD_K5_AB_SKIP_FOLD": "1"}]
KNOBS = ("TORCHEVAL_AMD_K5_V2", "TORCHEVAL_AMD_K5_CG", "TORCHEVAL_AMD_K5_BLOCKS", "TORCHEVAL_AMD_K5_MAXR",
         "TORCHEVAL_AMD_K5_PIPE", "TORCHEVAL_AMD_K5_AB_SKIP_FOLD")


def main() -> None:
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    widths = [int(w) for w in os.environ.get("K5AB_WIDTHS", "1000,1001,4096,4097").split(",")]
    data = {}
    for c in widths:
        data[c] = ([torch.randn(8192, c, device=dev, generator=g) for _ in range(4)],
                   [torch.randn(8192, c, device=dev, generator=g) for _ in range(4)])
    for cfg in CONFIGS:
        for k in KNOBS:
            os.environ.pop(k, None)
        os.environ.update(cfg)
        rows = {}
        for c, (xs, ts) in data.items():
            mse, r2 = MeanSquaredError(device=dev), R2Score(device=dev)
            mb = 8192 * c * 4 / 1e6
            row = {}
            for name, fn, nb in (
                ("mse_update", lambda i: mse.update(xs[i % 4], ts[i % 4]), 2 * mb),
                ("r2_update", lambda i: r2.update(xs[i % 4], ts[i % 4]), 2 * mb),
                ("mse_fn", lambda i: mean_squared_error(xs[i % 4], ts[i % 4]), 2 * mb),
                ("r2_fn", lambda i: r2_score(xs[i % 4], ts[i % 4]), 2 * mb),
            ):
                us = _per_call_us(fn)
                row[name] = {"us": round(us, 2), "TBps": round(nb / us, 2)}
            rows[f"8192x{c}"] = row
        print(json.dumps({"config": cfg or "default", "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
