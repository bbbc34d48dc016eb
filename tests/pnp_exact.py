"""The reference's PnP consensus arithmetic, emulated operation by operation (test helper).

ransac.py:96-105 computes ``e = dpp_squared(y, calc_y_prim(x, R, t))`` and keeps a point when
``thresh >= e``.  oracle/pnp_ref.pose_errors restates it with numpy: ``X @ R.T + t``, pi, diff,
dot.  numpy's matmul goes to OpenBLAS dgemm, whose 3-term inner products on the build container
are the FMA chain ``fma(R_i2, z, fma(R_i1, y, R_i0 * x))`` (the first product rounded on its
own); the rest is plain IEEE arithmetic in order.  ``errors_exact`` evaluates exactly that with
the FMAs computed in rational arithmetic, so it does not depend on the host BLAS:
tests/test_oracle_p3p.py checks it against pose_errors on this host, and the GPU tests use it
as the truth for counts decided at the last bit.
"""
from fractions import Fraction

import numpy as np


def _fma(a, b, c):
    a, b, c = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64),
                                  np.asarray(c, np.float64))
    out = np.empty(a.shape, np.float64)
    fa, fb, fc, fo = a.ravel(), b.ravel(), c.ravel(), out.reshape(-1)
    for i in range(fa.size):
        x, y, z = float(fa[i]), float(fb[i]), float(fc[i])
        if not (np.isfinite(x) and np.isfinite(y) and np.isfinite(z)):
            fo[i] = x * y + z
        else:
            fo[i] = float(Fraction(x) * Fraction(y) + Fraction(z))
    return out


def errors_exact(P, X, y):
    """Per-point e of ransac.py:96-101 for the pose P (12: R row-major, t), bit for bit."""
    P = np.asarray(P, np.float64).ravel()
    X = np.asarray(X, np.float64)
    y = np.asarray(y, np.float64)
    q = [_fma(P[3 * i + 2], X[:, 2], _fma(P[3 * i + 1], X[:, 1], P[3 * i] * X[:, 0])) + P[9 + i]
         for i in range(3)]
    with np.errstate(divide="ignore", invalid="ignore"):
        a0 = y[:, 0] / y[:, 2] - q[0] / q[2]
        a1 = y[:, 1] / y[:, 2] - q[1] / q[2]
        a2 = y[:, 2] / y[:, 2] - q[2] / q[2]
        return (a0 * a0 + a1 * a1) + a2 * a2


def boundary_cloud(X, y, P, picks, spread=12, seed=0):
    """Points whose e under P straddle e(P, pick) by a few ulps: every picked point is repeated
    2 * spread + 1 times with its world coordinates nudged by k ulps (k = -spread .. spread)
    along a random direction.  Returns (X', y')."""
    rs = np.random.RandomState(seed)
    Xs, ys = [], []
    for j in picks:
        d = rs.choice([-1.0, 1.0], 3)
        for k in range(-spread, spread + 1):
            x = X[j].copy()
            for c in range(3):
                for _ in range(abs(k)):
                    x[c] = np.nextafter(x[c], np.inf * d[c] * np.sign(k))
            Xs.append(x)
            ys.append(y[j])
    return np.array(Xs), np.array(ys)
