"""ORACLE -- test infrastructure only, never shipped, never measured as the product.

CPU numpy restatement of the reference PnP path
(bioengstrom/tsbb15-3d-reconstruction-project, snapshot v0).  The in-repo PnP code does
not run (``ransac_robust`` raises at ransac.py:77,
``pnp_minimize`` is an unfinished skeleton at pnp.py:164-196), so this restates the
*documented* algorithm:

  * ``pnp_dlt``          pnp.py:132-160 (algebraic DLT outline, rows of [y]_x, null vector,
                         constraint enforcement tau / SVD / lambda), using the first two
                         rows of [y_k]_x (pnp.py:152 "two of the rows suffice") and the
                         homogeneous (SVD) null-space method (pnp.py:139-140)
  * ``gen_rnd_indices``  ransac.py:12-19 (Python ``random.shuffle`` prefix)
  * ``dpp_squared``      ransac.py:21-32 per point: |pi(y) - pi(y')|^2, pi(v) = v / v[-1]
  * ``ransac_pnp``       ransac.py:37-113 intended semantics: r trials, sample n from
                         D_high, solve, consensus ``thresh >= e`` (inclusive, ransac.py:104-105)
                         on D_med and D_high, keep the largest D_med consensus with strict ">"
                         (ransac.py:108), initial best size 0.

Parity status: "parity unpinned" against OpenCV ``solvePnPRansac`` (tables.py:141; OpenCV
is absent and unpinned).  The DLT itself is pinned by known-answer tests on the reference's
own noise-free ``BAdino2.mat`` scene, whose per-view (R, t) come from the reference's
``fun.camera_resectioning`` (tests/golden/dino_pnp_kat.npz).
"""
from __future__ import annotations

import random as _random

import numpy as np


def calc_p(w, n, r):
    """ransac.py:6-7"""
    return 1 - np.power(1 - np.power(w, n), r)


def calc_r(w, n, p):
    """ransac.py:9-10 (float, not rounded)"""
    return np.log(1 - p) / np.log(1 - np.power(w, n))


def gen_rnd_indices(set_length, n, rng=None):
    """ransac.py:12-19"""
    if set_length < n:
        raise ValueError("Cannot generate more indices than the amount of values in the set")
    rng = _random if rng is None else rng
    idx = list(range(set_length))
    rng.shuffle(idx)
    return idx[0:n]


def cross_rows(y):
    """The first two rows of [y]_x (lab3.cross_matrix, lab3.py:110-129)."""
    return np.array([[0.0, -y[2], y[1]],
                     [y[2], 0.0, -y[0]]])


def dlt_matrix(X, y):
    """Rows vec(r_l x_k^T) (pnp.py:150-154), x_k = [X_k, 1]."""
    rows = []
    for k in range(X.shape[0]):
        xh = np.append(X[k, :3], 1.0)
        for r in cross_rows(y[k]):
            rows.append(np.outer(r, xh).ravel())
    return np.array(rows)


def pnp_dlt(X, y):
    """(R, t) from m >= 6 correspondences X (m,3) <-> y (m,3) C-normalised homogeneous."""
    A = dlt_matrix(X, y)
    _, _, V = np.linalg.svd(A)
    C0 = V[-1].reshape(3, 4)
    A3, b = C0[:, :3], C0[:, 3]
    tau = np.sign(np.linalg.det(A3))
    U, S, Vt = np.linalg.svd(tau * A3)
    R = U @ Vt
    lam = 3.0 * tau / np.sum(S)
    return R, lam * b


def dpp_squared_rows(y, yp):
    """Per-row squared distance of the pi-normalised homogeneous points."""
    a = y / y[:, -1:]
    b = yp / yp[:, -1:]
    diff = a - b
    return np.sum(diff * diff, axis=1)


def pose_errors(R, t, X, y):
    yp = X[:, :3] @ R.T + t
    return dpp_squared_rows(y, yp)


def ransac_pnp(y_med, X_med, y_high, X_high, r, thresh, n=6, rng=None, trace=False):
    """Intended ``ransac_robust`` (ransac.py:37-113) with the DLT as the minimal solver.

    Returns ``(R, t, inl_med, inl_high, best_index, counts_or_None)``.
    """
    best, best_count = -1, 0
    R_best = t_best = None
    counts = np.zeros(r, dtype=np.int64) if trace else None
    for i in range(r):
        T = gen_rnd_indices(len(X_high), n, rng)
        R, t = pnp_dlt(X_high[T], y_high[T])
        c_med = int(np.count_nonzero(thresh >= pose_errors(R, t, X_med, y_med)))
        if trace:
            counts[i] = c_med
        if c_med > best_count:
            best, best_count, R_best, t_best = i, c_med, R, t
    if best < 0:
        return None, None, None, None, -1, counts
    inl_med = np.flatnonzero(thresh >= pose_errors(R_best, t_best, X_med, y_med))
    inl_high = np.flatnonzero(thresh >= pose_errors(R_best, t_best, X_high, y_high))
    return R_best, t_best, inl_med, inl_high, best, counts
