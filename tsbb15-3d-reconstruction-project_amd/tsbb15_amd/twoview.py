"""Two-view geometry after RANSAC: the gold-standard (ML) refinement of fun.py:343-369.

Host numpy/scipy stage (the "next" row; not yet on the GPU).  The
formulas are the textbook ones the reference toolbox uses:

  * cameras from F with C2 = [I | 0]: C1 = [[e1]_x F | e1], e1 the left null vector of F
    (lab3.fmatrix_cameras, lab3.py:353-380);
  * F from cameras: F = [C1 n]_x C1 C2^+, n the camera centre of C2 (lab3.py:331-351);
  * optimal triangulation (Hartley & Zisserman, Alg. 12.1) with both epipoles rotated onto the
    x axis and f = f' = 1: roots of g(t) = t P(t)^2 - (ad - bc)(1 + t^2)^2 (at + b)(ct + d),
    P(t) = (at + b)^2 + (ct + d)^2, cost s(t) = t^2/(1 + t^2) + (ct + d)^2 / P(t), plus the
    value at t = inf (lab3.py:382-475); real parts of all roots are evaluated, as there;
  * linear triangulation by the null vector of [[x1]_x C1; [x2]_x C2] (lab3.py:477-503);
  * reprojection residuals (lab3.py:230-266) minimised by scipy's TRF with lsmr and
    xtol = 2.22e-14 (fun.py:358).
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import least_squares

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])


def cross_matrix(v):
    v = np.asarray(v, dtype=np.float64).ravel()
    if v.size != 3:
        raise ValueError('Can only handle 3D vectors')
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def project(X, C):
    """Pinhole projection of (3,) or (3,N) points through a 3x4 camera -> (2,) or (2,N)."""
    if C.shape != (3, 4):
        raise ValueError('C is not a valid camera matrix')
    X = np.asarray(X, dtype=np.float64)
    one_d = X.ndim == 1
    Xh = np.vstack([X.reshape(3, -1), np.ones((1, X.reshape(3, -1).shape[1]))])
    y = C @ Xh
    y = y[:2] / y[2]
    return y.ravel() if one_d else y


def fmatrix_from_cameras(C1, C2):
    _, _, Vt = np.linalg.svd(C2)
    e = C1 @ Vt[3]
    return cross_matrix(e) @ (C1 @ np.linalg.pinv(C2))


def fmatrix_cameras(F):
    U, _, _ = np.linalg.svd(F)
    e1 = U[:, -1]
    C1 = np.hstack([cross_matrix(e1) @ F, e1.reshape(3, 1)])
    return C1, I34.copy()


def fmatrix_epipoles(F):
    U, _, Vt = np.linalg.svd(F)
    e1 = U[:, -1] / U[-1, -1]
    e2 = Vt[-1] / Vt[-1, -1]
    return e1[:2], e2[:2]


def triangulate_linear(C1, C2, x1, x2):
    x1 = np.append(x1, 1.0) if np.size(x1) == 2 else np.asarray(x1, float).ravel()
    x2 = np.append(x2, 1.0) if np.size(x2) == 2 else np.asarray(x2, float).ravel()
    M = np.vstack([cross_matrix(x1) @ C1, cross_matrix(x2) @ C2])
    X = np.linalg.svd(M)[2][-1]
    return X[:3] / X[3]


def _rot_to_x_axis(e):
    return np.array([[e[0], e[1], 0.0], [-e[1], e[0], 0.0], [0.0, 0.0, 1.0]])


def triangulate_optimal(C1, C2, x1, x2):
    """Hartley-Zisserman optimal triangulation (f = f' = 1 form) of one correspondence."""
    T1 = np.array([[1.0, 0.0, x1[0]], [0.0, 1.0, x1[1]], [0.0, 0.0, 1.0]])
    T2 = np.array([[1.0, 0.0, x2[0]], [0.0, 1.0, x2[1]], [0.0, 0.0, 1.0]])
    F = T1.T @ (fmatrix_from_cameras(C1, C2) @ T2)
    e1, e2 = fmatrix_epipoles(F)
    e1 = e1 / np.linalg.norm(e1)
    e2 = e2 / np.linalg.norm(e2)
    R1, R2 = _rot_to_x_axis(e1), _rot_to_x_axis(e2)
    F = R1 @ (F @ R2.T)
    a, b, c, d = F[1, 1], F[1, 2], F[2, 1], F[2, 2]
    P = np.polyadd(np.polymul([a, b], [a, b]), np.polymul([c, d], [c, d]))
    g = np.polysub(np.polymul([1.0, 0.0], np.polymul(P, P)),
                   (a * d - b * c) * np.polymul([1.0, 0.0, 2.0, 0.0, 1.0],
                                                np.polymul([a, b], [c, d])))
    t = np.real(np.roots(g))
    cost = [ti ** 2 / (1 + ti ** 2) + (c * ti + d) ** 2 / ((a * ti + b) ** 2 + (c * ti + d) ** 2)
            for ti in t]
    cost.append(1.0 + c ** 2 / (a ** 2 + c ** 2))
    k = int(np.argmin(cost))
    if k < t.size:
        tm = t[k]
        l1 = np.array([-(c * tm + d), a * tm + b, c * tm + d])
        l2 = np.array([tm, 1.0, -tm])
    else:
        l1 = np.array([-c, a, c])
        l2 = np.array([1.0, 0.0, -1.0])

    def foot(l):  # closest point of line l to the origin (homogeneous)
        return np.array([-l[0] * l[2], -l[1] * l[2], l[0] ** 2 + l[1] ** 2])

    y1 = T1 @ (R1.T @ foot(l1))
    y2 = T2 @ (R2.T @ foot(l2))
    return triangulate_linear(C1, C2, y1, y2)


def fmatrix_residuals_gs(params, pl, pr):
    """Reprojection residuals [left x, left y, right x, right y] (lab3.py:230-266)."""
    C1 = params[:12].reshape(3, 4)
    X = params[12:].reshape(-1, 3).T
    if X.shape[1] != pl.shape[1]:
        raise ValueError('Wrong size of parameter vector')
    return np.concatenate([(pl - project(X, C1)).ravel(), (pr - project(X, I34)).ravel()])


def gold_standard(F, pl, pr):
    """ML refinement of F on the consensus set (fun.py:343-369); returns F_gold."""
    C1, C2 = fmatrix_cameras(F)
    X = np.array([triangulate_optimal(C1, C2, a, b) for a, b in zip(pl.T, pr.T)])
    params = np.hstack([C1.ravel(), X.ravel()])
    sol = least_squares(fmatrix_residuals_gs, params, xtol=2.22e-14, tr_solver='lsmr',
                        args=(pl, pr)).x
    return fmatrix_from_cameras(sol[:12].reshape(3, 4), I34.copy())
