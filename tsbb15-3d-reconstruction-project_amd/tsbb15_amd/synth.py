"""Synthetic two-view / PnP workloads of SURVEY.md section 8(d).

Deterministic (numpy legacy ``RandomState``, whose streams are frozen across numpy
versions and platforms), so the build container and the GPU box produce bit-identical
inputs without shipping data files.

Scene: K = [[800,0,320],[0,800,240],[0,0,1]]; points uniform in [-1,1]^2 x [4,8];
camera 1 = [I|0]; camera 2 = R_y(0.15 rad), t = (-0.8, 0.05, 0.1); Gaussian pixel noise
sigma = 0.5 px; outliers replace right-image points by uniform points in [0,640]x[0,480].
"""
from __future__ import annotations

import numpy as np

K_SYNTH = np.array([[800.0, 0.0, 320.0], [0.0, 800.0, 240.0], [0.0, 0.0, 1.0]])
ANGLE = 0.15
T_SYNTH = np.array([-0.8, 0.05, 0.1])


def rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def _project(K, R, t, X):
    x = (K @ (R @ X.T + t.reshape(3, 1)))
    return x[:2] / x[2]


def two_view(n, outlier_frac, seed, sigma=0.5):
    """Return ``(p1, p2, inlier_mask)``; p1, p2 are (2, n) float64 pixel coordinates.

    ``p1`` is the left view (camera [I|0]) and ``p2`` the right view, the layout of
    ``fun.getFFromLabCode(p1, p2)`` (fun.py:291; convention p1^T F p2 = 0).
    """
    rs = np.random.RandomState(seed)
    X = np.column_stack([rs.uniform(-1.0, 1.0, n), rs.uniform(-1.0, 1.0, n),
                         rs.uniform(4.0, 8.0, n)])
    p1 = _project(K_SYNTH, np.eye(3), np.zeros(3), X)
    p2 = _project(K_SYNTH, rot_y(ANGLE), T_SYNTH, X)
    p1 = p1 + rs.normal(0.0, sigma, p1.shape)
    p2 = p2 + rs.normal(0.0, sigma, p2.shape)
    n_out = int(round(outlier_frac * n))
    out = rs.permutation(n)[:n_out]
    p2[0, out] = rs.uniform(0.0, 640.0, n_out)
    p2[1, out] = rs.uniform(0.0, 480.0, n_out)
    inl = np.ones(n, dtype=bool)
    inl[out] = False
    return np.ascontiguousarray(p1), np.ascontiguousarray(p2), inl


def pnp_scene(m, outlier_frac, seed, sigma=0.5):
    """PnP workload (config C3): returns ``(X (m,3), y_px (m,2), y_norm (m,3), R, t, inl)``.

    ``y_norm`` = K^-1 [u, v, 1] (C-normalised homogeneous, fun.MakeHomogenous, fun.py:48-55).
    """
    rs = np.random.RandomState(seed)
    X = np.column_stack([rs.uniform(-1.0, 1.0, m), rs.uniform(-1.0, 1.0, m),
                         rs.uniform(4.0, 8.0, m)])
    R = rot_y(ANGLE)
    y = _project(K_SYNTH, R, T_SYNTH, X) + rs.normal(0.0, sigma, (2, m))
    n_out = int(round(outlier_frac * m))
    out = rs.permutation(m)[:n_out]
    y[0, out] = rs.uniform(0.0, 640.0, n_out)
    y[1, out] = rs.uniform(0.0, 480.0, n_out)
    inl = np.ones(m, dtype=bool)
    inl[out] = False
    y_px = np.ascontiguousarray(y.T)
    yh = np.vstack([y, np.ones((1, m))])
    y_norm = np.ascontiguousarray((np.linalg.inv(K_SYNTH) @ yh).T)
    return X, y_px, y_norm, R, T_SYNTH.copy(), inl
