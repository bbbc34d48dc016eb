"""ORACLE -- test infrastructure only, never shipped, never measured as the product.

CPU numpy restatement of the reference RANSAC-F path
(bioengstrom/tsbb15-3d-reconstruction-project, snapshot v0):

  * ``homog``              lab3.py:30-50
  * ``fmatrix_stls``       lab3.py:269-329   (Hartley-style 8-point, SVD null vector, rank 2)
  * ``fmatrix_residuals``  lab3.py:188-227   (signed point-to-epipolar-line distances, px)
  * ``ransac_f``           fun.py:298-328    (the hypothesis loop of ``getFFromLabCode``)

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.

Pinning: every function here is checked against vectors produced by the reference itself
(``tests/golden/make_golden.py`` imports the reference modules in the build container and
writes ``tests/golden/*.npz``; ``tests/test_oracle_golden.py`` compares).
"""
from __future__ import annotations

import numpy as np

INLIER_THRESHOLD = 1.5     # fun.py:317, strict "<"
SAMPLE_SIZE = 8            # fun.py:306
REFERENCE_ITERATIONS = 10000  # fun.py:302


def homog(x):
    """Append a row of ones (lab3.py:30-50)."""
    is2d = x.ndim == 2
    if not is2d:
        x = x.reshape(-1, 1)
    d, n = x.shape
    X = np.empty((d + 1, n))
    X[:-1, :] = x
    X[-1, :] = 1
    return X if is2d else X.ravel()


def fmatrix_residuals(F, x, y):
    """(2,N) signed distances of x (row 0) and y (row 1) to their epipolar lines.

    lab3.py:188-227: l1 = F y^, l2 = F^T x^, res1 = (l1.x^)/|l1[:2]|, res2 = (l2.y^)/|l2[:2]|.
    """
    if not x.shape == y.shape:
        raise ValueError('x and y must have same sizes')
    x = homog(x)
    y = homog(y)
    l1 = np.dot(F, y)
    l2 = np.dot(F.T, x)
    l1s = np.sqrt(l1[0, :] ** 2 + l1[1, :] ** 2)
    l2s = np.sqrt(l2[0, :] ** 2 + l2[1, :] ** 2)
    res1 = np.sum(l1 * x, axis=0) / l1s
    res2 = np.sum(l2 * y, axis=0) / l2s
    return np.vstack((res1, res2))


def _scaling_homography(x, N):
    # lab3.py:288-295 -- note L = sqrt(sum|x - xm|^2 / (2N)), not Hartley's sqrt(2) form
    xm = np.mean(x, axis=1)
    x_norm = x - xm.reshape(-1, 1)
    L = np.sqrt(1. / 2. / N * np.sum(x_norm ** 2))
    return np.array([[1. / L, 0., -xm[0] / L],
                     [0., 1. / L, -xm[1] / L],
                     [0., 0., 1.]])


def _map_homography(p, H):
    # lab3.py:301-306
    x = p[0]
    y = p[1]
    return x * H[0, 0] + y * H[0, 1] + H[0, 2], x * H[1, 0] + y * H[1, 1] + H[1, 2]


def fmatrix_stls(pl, pr):
    """8-point F with pl^T F pr = 0 (lab3.py:269-329)."""
    if not pl.shape == pr.shape:
        raise ValueError('pl and pr must have same shape')
    _, N = pl.shape
    S = _scaling_homography(pl, N)
    T = _scaling_homography(pr, N)
    X, Y = _map_homography(pl, S)
    x, y = _map_homography(pr, T)
    A = np.vstack((X * x, X * y, X, Y * x, Y * y, Y, x, y, np.ones((1, N)))).T
    _, _, V = np.linalg.svd(A)               # lab3.py:317 (V already transposed)
    Fs = V[-1, :].reshape(3, 3)
    U, s, V = np.linalg.svd(Fs)              # lab3.py:321-324: enforce rank 2
    D = np.diag(s)
    D[2, 2] = 0
    Fs = np.dot(U, np.dot(D, V))
    return np.dot(S.T, np.dot(Fs, T))        # lab3.py:327


def inlier_distance(F, p1, p2):
    """d = max(|res|, axis 0) -- NaN-propagating np.max (fun.py:316)."""
    return np.max(np.abs(fmatrix_residuals(F, p1, p2)), axis=0)


class RansacTrace:
    """Per-hypothesis record of a restated loop (for golden comparison)."""

    def __init__(self, r):
        self.tuples = np.zeros((r, SAMPLE_SIZE), dtype=np.int64)
        self.counts = np.zeros(r, dtype=np.int64)
        self.stds = np.zeros(r)
        self.norms = np.zeros(r)


def ransac_f(p1, p2, r=REFERENCE_ITERATIONS, rng=None, trace=False):
    """The hypothesis loop of ``fun.getFFromLabCode`` (fun.py:298-328), restated.

    ``rng`` defaults to the legacy global ``np.random`` exactly as the reference
    (fun.py:306 ``np.random.choice(index_points, 8, replace=False)``); pass a
    ``np.random.RandomState`` for an explicit stream.

    Returns ``(F_RANSAC, S_RANSAC, d_RANSAC, best_index, trace_or_None)``.
    Selection rule (fun.py:320-328): strictly more inliers replaces; an equal count
    replaces when ``norm(d_RANSAC) > norm(d)`` where ``d_RANSAC`` is the population std of
    the current best's ``d`` (a scalar, so its norm is its absolute value) and ``norm(d)``
    is the 2-norm of the candidate's full distance vector.
    """
    if rng is None:
        rng = np.random
    F_RANSAC = None
    S_RANSAC = []
    d_RANSAC = []
    best = -1
    tr = RansacTrace(r) if trace else None
    N = p1.shape[1]
    for i in range(r):
        index_points = np.arange(0, N, 1)
        idx = rng.choice(index_points, SAMPLE_SIZE, replace=False)
        F = fmatrix_stls(p1[:, idx], p2[:, idx])
        d = inlier_distance(F, p1, p2)
        S = np.flatnonzero(d < INLIER_THRESHOLD)
        if tr is not None:
            tr.tuples[i] = idx
            tr.counts[i] = len(S)
            with np.errstate(invalid='ignore', over='ignore'):
                tr.stds[i] = np.std(d)
                tr.norms[i] = np.linalg.norm(d)
        if len(S) > len(S_RANSAC):
            S_RANSAC, F_RANSAC, d_RANSAC, best = S, F, np.std(d), i
        elif len(S) == len(S_RANSAC):
            if np.linalg.norm(d_RANSAC) > np.linalg.norm(d):
                S_RANSAC, F_RANSAC, d_RANSAC, best = S, F, np.std(d), i
    return F_RANSAC, np.asarray(S_RANSAC, dtype=np.int64), d_RANSAC, best, tr


def select_replay(counts, stds, norms):
    """Replay the fun.py:320-328 rule over per-hypothesis (count, std, norm) in order.

    Equivalent to ``ransac_f``'s selection given the per-hypothesis statistics; used to
    check the GPU candidate/replay logic.  Returns the winning hypothesis index or -1.
    """
    best_count, best_std, best = 0, 0.0, -1  # S_RANSAC = [] -> len 0; norm([]) = 0
    for i, (c, s, n) in enumerate(zip(counts, stds, norms)):
        if c > best_count:
            best_count, best_std, best = c, s, i
        elif c == best_count:
            if abs(best_std) > n:
                best_count, best_std, best = c, s, i
    return best


def normalize_F(F):
    """Frobenius-normalise and fix the sign (largest-|.| entry positive) for comparisons."""
    F = np.asarray(F, dtype=np.float64)
    F = F / np.linalg.norm(F)
    k = np.argmax(np.abs(F))
    return F if F.flat[k] >= 0 else -F
