"""Numpy model of stage 2 of a two-stage symmetric tridiagonalisation (band -> tridiagonal by
Householder bulge chasing, first-column annihilation), used to cost a two-stage K9b
(profiles/README.md, round 5).  Prints the eigenvalue error of the result and the bandwidth the
chase needs: b - 2 extra diagonals persist between sweeps and 2b - 1 appear inside a sweep, so
band storage must hold 2b + 1 diagonals.

    python benchmarks/fid_bulge_chase_model.py [n] [b]
"""
import sys

import numpy as np


def house(x):
    alpha = x[0]
    sigma = float(np.dot(x[1:], x[1:]))
    v = x.copy()
    v[0] = 1.0
    if sigma == 0.0:
        return v * 0.0, 0.0
    mu = np.sqrt(alpha * alpha + sigma)
    beta = -mu if alpha >= 0 else mu
    v[1:] = x[1:] / (alpha - beta)
    return v, (beta - alpha) / beta


def bandwidth(m):
    idx = np.argwhere(np.abs(m) > 1e-13)
    return int((idx[:, 0] - idx[:, 1]).max())


def main() -> None:
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    rng = np.random.default_rng(0)
    a = np.zeros((n, n))
    for i in range(n):
        for j in range(max(0, i - b), i + 1):
            a[i, j] = a[j, i] = rng.standard_normal()
    ev0 = np.linalg.eigvalsh(a)
    inside, after, steps = 0, 0, 0
    for i in range(n - 2):
        j, r0 = i, i + 1
        while r0 < n:
            r1 = min(r0 + b, n)
            x = a[r0:r1, j].copy()
            if len(x) < 2:
                break
            v, tau = house(x)
            h = np.eye(r1 - r0) - tau * np.outer(v, v)
            a[r0:r1, :] = h @ a[r0:r1, :]
            a[:, r0:r1] = a[:, r0:r1] @ h
            inside = max(inside, bandwidth(a))
            steps += 1
            j, r0 = r0, r0 + b
        after = max(after, bandwidth(a))
    t = np.diag(np.diag(a)) + np.diag(np.diag(a, -1), -1) + np.diag(np.diag(a, -1), 1)
    err = float(np.abs(np.linalg.eigvalsh(t) - ev0).max() / np.abs(ev0).max())
    print(f"n={n} b={b}: chase steps {steps}, bandwidth inside sweeps {inside}, between sweeps {after}, "
          f"left below the subdiagonal {np.abs(np.tril(a, -2)).max():.1e}, eigenvalue rel err {err:.1e}")


if __name__ == "__main__":
    main()
