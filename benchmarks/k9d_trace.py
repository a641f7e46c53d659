"""K9d per-tile-column phase trace at D = 2048 (s_memrealtime stamps of the pair-owner tasks):
where the critical chain's ~20 us per column goes.  Prints a table + one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torcheval_amd.ops import native  # noqa: E402

PH = ["start", "updates_done", "inverse_arrived", "T_published", "U_done", "factored", "published", "wave0_done"]


def main() -> None:
    dev = "cuda"
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, n + 64, device=dev, dtype=torch.float64, generator=g)
    s = x @ x.T / x.shape[1]
    nt = native().cholesky_tiles(n)
    L = torch.empty(64 * nt, 64 * nt, dtype=torch.float64, device=dev)
    linv = torch.empty(nt * 4096, dtype=torch.float64, device=dev)
    ctl = torch.empty(1, dtype=torch.int32, device=dev)
    st = torch.empty(2, dtype=torch.int32, device=dev)
    tr = torch.zeros(nt * 8 + 130, dtype=torch.int64, device=dev)
    for _ in range(3):
        native().cholesky_factor_traced(s, L, linv, ctl, st, tr)
    torch.cuda.synchronize()
    cyc = tr[nt * 8: nt * 8 + 32].view(4, 8).cpu()
    steps = [(cyc[k, 1:6] - cyc[k, 0:5]).tolist() for k in range(4)]
    t = tr[: nt * 8].view(nt, 8).cpu().double() * 0.01  # 100 MHz -> us
    t0 = float(t[0, 0])
    rows = []
    for c in range(nt):
        r = {PH[k]: round(float(t[c, k]) - t0, 2) if t[c, k] > 0 else None for k in range(8)}
        rows.append(r)
    # per-column durations of the chain
    d = {}
    for c in range(2, nt):
        prev_pub = float(t[c - 1, 6])
        d.setdefault("handoff_prev_published_to_inverse_arrived", []).append(float(t[c, 2]) - prev_pub)
        d.setdefault("T", []).append(float(t[c, 3] - t[c, 2]))
        d.setdefault("U", []).append(float(t[c, 4] - t[c, 3]))
        d.setdefault("potrf", []).append(float(t[c, 5] - t[c, 4]))
        d.setdefault("potrf_wave0_eliminations", []).append(float(t[c, 7] - t[c, 4]))
        d.setdefault("publish", []).append(float(t[c, 6] - t[c, 5]))
        d.setdefault("slack_updates_done_before_inverse", []).append(float(t[c, 2] - t[c, 1]))
    med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in d.items()}
    total = round(float(t[nt - 1, 6]) - t0, 1)
    print(json.dumps({"n": n, "status": st.cpu().tolist(), "total_us_first_stamp_to_last": total,
                      "median_us_per_column": med, "column_2": rows[min(2, nt - 1)], "column_last": rows[-1],
                      "tile1_phase0_step_cycles_gather_chol44_coef_publish_elim": steps}))


if __name__ == "__main__":
    main()
