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


# ------------------------------------------------------------------------------------------
# n = 3: the p3p branch of ransac_robust (ransac.py:81-82, 91-111)
# ------------------------------------------------------------------------------------------
# The reference's p3p (pnp.py:7-10) is cv2.solvePnP and its own Lambda Twist (pnp.py:61-121)
# stops after the eigen-decomposition, so the branch cannot run there ("parity unpinned").
# This restates Lambda Twist P3P (Persson & Nordberg, ECCV 2018) step for step as
# pnp_minimal.h p3p_lambda_twist computes it, so the GPU kernel is checked against an
# independent CPU evaluation of the same algorithm, solution order included.

def _cubic_roots(c3, c2, c1, c0):
    a, b, c = c2 / c3, c1 / c3, c0 / c3
    q = (a * a - 3.0 * b) / 9.0
    r = (2.0 * a * a * a - 9.0 * a * b + 27.0 * c) / 54.0
    if r * r < q * q * q:
        th = np.arccos(min(1.0, max(-1.0, r / np.sqrt(q * q * q))))
        sq = -2.0 * np.sqrt(q)
        x = [sq * np.cos(th / 3.0) - a / 3.0, sq * np.cos((th + 2.0 * np.pi) / 3.0) - a / 3.0,
             sq * np.cos((th - 2.0 * np.pi) / 3.0) - a / 3.0]
    else:
        A = -np.copysign(np.cbrt(abs(r) + np.sqrt(r * r - q * q * q)), r)
        B = q / A if A != 0.0 else 0.0
        x = [(A + B) - a / 3.0]
    for i in range(len(x)):
        for _ in range(2):
            f = ((x[i] + a) * x[i] + b) * x[i] + c
            fp = (3.0 * x[i] + 2.0 * a) * x[i] + b
            if fp != 0.0:
                x[i] -= f / fp
    return x


def _null3(A):
    A = A.reshape(3, 3)
    c = [np.cross(A[0], A[1]), np.cross(A[0], A[2]), np.cross(A[1], A[2])]
    d = [float(v @ v) for v in c]
    k = int(np.argmax(d))   # first of equal maxima, as the kernel's strict ">"
    return c[k] / np.sqrt(d[k]) if d[k] > 0.0 else c[k] * 0.0


def p3p_lambda_twist(X, y):
    """Poses (R, t, mirrored) from three world points X (3,3) and unit bearings y (3,3): up to
    four front-facing solutions, each followed by its mirrored-depth twin."""
    b01, b02, b12 = y[0] @ y[1], y[0] @ y[2], y[1] @ y[2]
    a01 = float((X[0] - X[1]) @ (X[0] - X[1]))
    a02 = float((X[0] - X[2]) @ (X[0] - X[2]))
    a12 = float((X[1] - X[2]) @ (X[1] - X[2]))
    D1 = np.array([[a12, -a12 * b01, 0.0], [-a12 * b01, a12 - a01, a01 * b12], [0.0, a01 * b12, -a01]])
    D2 = np.array([[a12, 0.0, -a12 * b02], [0.0, -a02, a02 * b12], [-a12 * b02, a02 * b12, a12 - a02]])
    A0, A1, A2 = D1[:, 0], D1[:, 1], D1[:, 2]
    B0, B1, B2 = D2[:, 0], D2[:, 1], D2[:, 2]
    c3 = B0 @ np.cross(B1, B2)
    c2 = A0 @ np.cross(B1, B2) + A1 @ np.cross(B2, B0) + A2 @ np.cross(B0, B1)
    c0 = A0 @ np.cross(A1, A2)
    c1 = B0 @ np.cross(A1, A2) + B1 @ np.cross(A2, A0) + B2 @ np.cross(A0, A1)
    if not c3 != 0.0:
        return []
    a = np.array([[0.0, a01, a02], [a01, 0.0, a12], [a02, a12, 0.0]])
    bb = np.array([[1.0, b01, b02], [b01, 1.0, b12], [b02, b12, 1.0]])
    out = []
    for g in _cubic_roots(c3, c2, c1, c0):
        D0 = D1 + g * D2
        T = D0[0, 0] + D0[1, 1] + D0[2, 2]
        P = ((D0[0, 0] * D0[1, 1] - D0[0, 1] ** 2) + (D0[0, 0] * D0[2, 2] - D0[0, 2] ** 2)
             + (D0[1, 1] * D0[2, 2] - D0[1, 2] ** 2))
        if not P < 0.0:
            continue
        sq = np.sqrt(T * T - 4.0 * P)
        s0 = 0.5 * (T + sq) if T >= 0.0 else 0.5 * (T - sq)
        s1 = P / s0
        e0 = _null3(D0 - s0 * np.eye(3))
        e1 = _null3(D0 - s1 * np.eye(3))
        for sg in range(2):
            tt = (-1.0 if sg else 1.0) * np.sqrt(-s0 / s1)
            nv = e1 - tt * e0
            k = 0
            if abs(nv[1]) > abs(nv[k]):
                k = 1
            if abs(nv[2]) > abs(nv[k]):
                k = 2
            o1, o2 = (k + 1) % 3, (k + 2) % 3
            w1, w2 = -nv[o1] / nv[k], -nv[o2] / nv[k]
            aq, bq, ap, bp = a[o1, o2], bb[o1, o2], a[k, o1], bb[k, o1]
            q2 = aq * (w1 * w1 + 1.0 - 2.0 * bp * w1) - ap
            q1 = aq * (2.0 * w1 * w2 - 2.0 * bp * w2) + 2.0 * ap * bq
            q0 = aq * w2 * w2 - ap
            disc = q1 * q1 - 4.0 * q2 * q0
            if not disc >= 0.0 or q2 == 0.0:
                continue
            sd = np.sqrt(disc)
            for rt in range(2):
                if len(out) >= 8:
                    break
                tau = (-q1 + (-sd if rt else sd)) / (2.0 * q2)
                if not tau > 0.0:
                    continue
                den = tau * tau - 2.0 * bq * tau + 1.0
                if not den > 0.0:
                    continue
                lam = np.zeros(3)
                lam[o2] = np.sqrt(aq / den)
                lam[o1] = tau * lam[o2]
                lam[k] = w1 * lam[o1] + w2 * lam[o2]
                if not (lam[0] > 0.0 and lam[1] > 0.0 and lam[2] > 0.0):
                    continue
                for _ in range(3):
                    r = np.array([lam[0] ** 2 + lam[1] ** 2 - 2.0 * b01 * lam[0] * lam[1] - a01,
                                  lam[0] ** 2 + lam[2] ** 2 - 2.0 * b02 * lam[0] * lam[2] - a02,
                                  lam[1] ** 2 + lam[2] ** 2 - 2.0 * b12 * lam[1] * lam[2] - a12])
                    J = np.array([[2.0 * (lam[0] - b01 * lam[1]), 2.0 * (lam[1] - b01 * lam[0]), 0.0],
                                  [2.0 * (lam[0] - b02 * lam[2]), 0.0, 2.0 * (lam[2] - b02 * lam[0])],
                                  [0.0, 2.0 * (lam[1] - b12 * lam[2]), 2.0 * (lam[2] - b12 * lam[1])]])
                    if not abs(np.linalg.det(J)) > 0.0:
                        break
                    lam = lam - np.linalg.solve(J, r)
                xa, xb = X[1] - X[0], X[2] - X[0]
                Xm = np.column_stack([xa, xb, np.cross(xa, xb)])
                if not abs(np.linalg.det(Xm)) > 0.0:
                    continue
                for mirror in range(2):
                    Pt = (-1.0 if mirror else 1.0) * lam[:, None] * y
                    pa, pb = Pt[1] - Pt[0], Pt[2] - Pt[0]
                    Pm = np.column_stack([pa, pb, np.cross(pa, pb)])
                    R = Pm @ np.linalg.inv(Xm)
                    out.append((R, Pt[0] - R @ X[0], bool(mirror)))
        break   # one real root that gives a line pair carries every solution
    return out[:8]


def bearings(y):
    """Unit bearings of C-normalised homogeneous image points (rows), as the kernel forms them:
    (u, v, 1) / |.| with (u, v) = pi(y)."""
    u, v = y[:, 0] / y[:, 2], y[:, 1] / y[:, 2]
    b = np.column_stack([u, v, np.ones_like(u)])
    return b / np.linalg.norm(b, axis=1, keepdims=True)


def ransac_pnp_p3p(y_med, X_med, y_high, X_high, r, thresh, rng=None, trace=False):
    """ransac_robust with n = 3 (ransac.py:72-111): per trial the P3P poses in order, each
    scored on D_med; strict ">" over (trial, pose) within the front-facing and within the
    mirrored-depth poses, a mirrored winner only at more than twice the front-facing count.  Returns (R, t, inl_med, inl_high,
    best_trial, best_pose, counts (r, 8) or None)."""
    # per class (front-facing, mirrored-depth): the first pose of largest count, strict ">"
    cls = [[-1, -1, 0, None, None], [-1, -1, 0, None, None]]
    counts = np.zeros((r, 8), np.int64) if trace else None
    for i in range(r):
        T = gen_rnd_indices(len(X_high), 3, rng)
        sols = p3p_lambda_twist(X_high[T], bearings(y_high[T]))
        for j, (R, t, mirrored) in enumerate(sols):
            c_med = int(np.count_nonzero(thresh >= pose_errors(R, t, X_med, y_med)))
            if trace:
                counts[i, j] = c_med
            b = cls[1 if mirrored else 0]
            if c_med > b[2]:
                b[:] = [i, j, c_med, R, t]
    # a mirrored pose reprojects like its front-facing twin (the scene behind the camera); it
    # wins only when its count is more than twice the best front-facing count (the kernel's
    # kMirrorCountWins; OpenCV's p3p never returns it, a negative-scale view needs it)
    best, best_pose, best_count, R_best, t_best = cls[1] if cls[1][2] > 2 * cls[0][2] else cls[0]
    if best < 0:
        return None, None, None, None, -1, -1, counts
    inl_med = np.flatnonzero(thresh >= pose_errors(R_best, t_best, X_med, y_med))
    inl_high = np.flatnonzero(thresh >= pose_errors(R_best, t_best, X_high, y_high))
    return R_best, t_best, inl_med, inl_high, best, best_pose, counts
