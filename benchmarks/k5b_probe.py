"""K5b update costs at 8192 x 1000 fp32 (one long row / 64 task rows), per statistic set:
where PSNR's and CTR's time goes against Sum / MSE / WeightedCalibration.  Prints one JSON line
(us per update, median of 5 timed windows of 200 updates each)."""

import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd import metrics as M  # noqa: E402


def _us(fn, n=200, reps=5):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / n * 1e6)
    return round(sorted(out)[reps // 2], 2)


def main() -> None:
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(8192, 1000, device=dev, generator=g)
    t = torch.rand(8192, 1000, device=dev, generator=g)
    res = {}
    p_auto = M.PeakSignalNoiseRatio(device=dev)
    res["psnr_auto_range"] = _us(lambda: p_auto.update(x, t))
    p_fix = M.PeakSignalNoiseRatio(data_range=1.0, device=dev)
    res["psnr_fixed_range"] = _us(lambda: p_fix.update(x, t))
    s = M.Sum(device=dev)
    res["sum"] = _us(lambda: s.update(x))
    mse = M.MeanSquaredError(device=dev)
    res["mse_2d"] = _us(lambda: mse.update(x, t))
    xt, tt = x.view(64, -1), t.view(64, -1)
    ctr = M.ClickThroughRate(num_tasks=64, device=dev)
    res["ctr64_tensor_weights"] = _us(lambda: ctr.update(xt, tt))
    res["ctr64_scalar_weight"] = _us(lambda: ctr.update(xt, 1.0))
    wc = M.WeightedCalibration(num_tasks=64, device=dev)
    res["wc64_tensor_weights"] = _us(lambda: wc.update(xt, tt, tt))
    res["wc64_scalar_weight"] = _us(lambda: wc.update(xt, tt, 1.0))
    ctr1 = M.ClickThroughRate(num_tasks=1, device=dev)
    x1, t1 = x.view(-1), t.view(-1)
    res["ctr1_tensor_weights"] = _us(lambda: ctr1.update(x1, t1))
    res["bytes_MB_2_streams"] = round(2 * x.numel() * 4 / 1e6, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
