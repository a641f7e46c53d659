"""Fixed K9b workload for rocprofv3 counter passes: eigenvalues of one 2048 x 2048 SPD matrix,
3 times after a warm-up (run with TORCHEVAL_AMD_SYMEIG_COOP=0: rocprofv3's teardown crashes after
a cooperative launch, profiles/exit_bisect_r4/)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torcheval_amd.ops import native  # noqa: E402


def main() -> None:
    n = 2048
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(n, n + 100, device="cuda", dtype=torch.float64, generator=g)
    m = x @ x.T / x.shape[1]
    lam = torch.empty(n, dtype=torch.float64, device="cuda")
    st = torch.zeros(1, dtype=torch.int32, device="cuda")
    for _ in range(4):
        assert native().sym_eigvals(m, lam, st) == 0
    torch.cuda.synchronize()
    assert int(st.item()) == 0
    print("ok", float(lam.max()))


if __name__ == "__main__":
    main()
