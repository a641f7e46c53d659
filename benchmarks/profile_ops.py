"""torch.profiler breakdown (host + device) of selected suite cases: where the time goes
beyond the native kernels.  python benchmarks/profile_ops.py [case-substring ...]"""

import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.bench_suite import cases  # noqa: E402


def main() -> None:
    wanted = sys.argv[1:] or ["binned_auroc", "binned_precision_recall", "r2_score", "binary_auroc N"]
    dev = torch.device("cuda", 0)
    for name, make in cases(dev, 1.0).items():
        if not any(w in name for w in wanted):
            continue
        fn = make()
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
            for _ in range(20):
                fn()
            torch.cuda.synchronize()
        print(f"\n##### {name}")
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=18, max_name_column_width=60))


if __name__ == "__main__":
    main()
