"""Stage 1 of a two-stage symmetric tridiagonalisation (dense -> band of width b, LAPACK sy2sb
semantics) at the FID's D = 2048, in FP64 on the GPU, to cost the two-stage K9b against the
one-stage kernel (csrc/kernels/symeig.hip, ~14.7 ms at D = 2048) and the VERDICT's 6 ms budget
for both stages.

Per panel k (columns k .. k+b-1, rows k+b .. n-1): QR of the m x b panel (rocSOLVER geqrf), the
compact-WY T from T^-1 = diag(1/tau) + striu(V^T V), then the two-sided trailing update
    X = A22 V T,  W = X - 1/2 V (T^T V^T X),  A22 -= [V W] [W V]^T
(rocBLAS / hipBLASLt FP64 GEMMs).  Measured:
  * the eigenvalues of the band result against eigvalsh of the dense input (correctness);
  * the whole stage 1, eager;
  * the trailing-update GEMM chain alone, captured in one HIP graph with every panel's V, T
    precomputed: the part no panel kernel can remove, i.e. a floor for stage 1 on this path.
Prints one JSON line.

    python benchmarks/fid_two_stage_probe.py [--n 2048] [--b 32 64]
"""

import argparse
import json
import time

import torch


def _panel(a: torch.Tensor, k: int, b: int):
    n = a.shape[0]
    p = a[k + b:, k:k + b]
    qr, tau = torch.geqrf(p)
    m, kk = p.shape[0], min(p.shape)
    v = torch.tril(qr[:, :kk], -1)
    v[:kk, :kk] += torch.eye(kk, dtype=a.dtype, device=a.device)
    tinv = torch.triu(v.T @ v, 1) + torch.diag(1.0 / tau[:kk])
    t = torch.linalg.solve_triangular(tinv, torch.eye(kk, dtype=a.dtype, device=a.device), upper=True)
    r = torch.triu(qr[:kk, :])
    del n, m
    return v, t, r


def _trailing(a22: torch.Tensor, v: torch.Tensor, t: torch.Tensor) -> None:
    x = (a22 @ v) @ t
    mm = t.T @ (v.T @ x)
    w = torch.addmm(x, v, mm, alpha=-0.5)
    a22.addmm_(torch.cat([v, w], 1), torch.cat([w, v], 1).T, alpha=-1.0)


def sy2sb(a: torch.Tensor, b: int, panels=None) -> torch.Tensor:
    """Dense symmetric -> symmetric band of width b (lower band kept, mirrored); `panels`
    collects (k, V, T) when given."""
    a = a.clone()
    n = a.shape[0]
    k = 0
    while n - k - b > 1:
        v, t, r = _panel(a, k, b)
        kk = r.shape[0]
        blk = torch.zeros_like(a[k + b:, k:k + b])
        blk[:kk] = r
        a[k + b:, k:k + b] = blk
        a[k:k + b, k + b:] = blk.T
        _trailing(a[k + b:, k + b:], v, t)
        if panels is not None:
            panels.append((k, v, t))
        k += b
    return a


def _ms(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) * 1e3)
    out.sort()
    return [round(out[0], 3), round(out[len(out) // 2], 3)]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2048)
    ap.add_argument("--b", type=int, nargs="+", default=[16, 32, 64])
    args = ap.parse_args()
    dev = "cuda"
    n = args.n
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n, n + 100, device=dev, dtype=torch.float64, generator=g)
    a = x @ x.T / x.shape[1]
    ev0 = torch.linalg.eigvalsh(a.cpu())
    res = {"n": n, "one_stage_k9b_ms_ref": "profiles/symeig_wave_ab_r5.json"}
    for b in args.b:
        band = sy2sb(a, b)
        lower = torch.tril(band, -b - 1).abs().max().item()
        ev = torch.linalg.eigvalsh(band.cpu())
        err = float((ev - ev0).abs().max() / ev0.abs().max())
        stage1 = _ms(lambda: sy2sb(a, b))
        # the GEMM chain alone, one graph
        panels = []
        sy2sb(a, b, panels)
        work = a.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for k, v, t in panels:
                _trailing(work[k + b:, k + b:], v, t)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            for k, v, t in panels:
                _trailing(work[k + b:, k + b:], v, t)
        gemm = _ms(graph.replay)
        # the panels alone (geqrf + T), eager
        panel_only = _ms(lambda: [_panel(a, k, b) for k, _, _ in panels])
        res[f"b{b}"] = {"panels": len(panels), "band_eig_rel_err": err, "max_outside_band": lower,
                        "stage1_eager_ms_min_med": stage1, "trailing_gemm_graph_ms_min_med": gemm,
                        "panel_qr_eager_ms_min_med": panel_only}
        print(json.dumps({f"b{b}": res[f"b{b}"]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
