"""ORACLE -- test infrastructure only, never shipped, never measured as the product.

CPU numpy/scipy restatement of the reference's two-view geometry that follows the RANSAC
loop (bioengstrom/tsbb15-3d-reconstruction-project, snapshot v0):

  * ``cross_matrix``          lab3.py (cross_matrix helper used by 331-351, 477-503)
  * ``fmatrix_from_cameras``  lab3.py:331-351   F = [C1 n]_x C1 C2^+,  n = null vector of C2
  * ``fmatrix_cameras``       lab3.py:353-380   C1 = [[e1]_x F | e1], C2 = [I | 0]
  * ``fmatrix_epipoles``      lab3.py:505-527
  * ``triangulate_linear``    lab3.py:477-503
  * ``triangulate_optimal``   lab3.py:382-475   (Klas Nordberg's degree-6 polynomial, f1=f2=1)
  * ``fmatrix_residuals_gs``  lab3.py:228-266
  * ``gold_standard``         fun.py:336-369    (scipy least_squares, xtol 2.22e-14, lsmr)
  * ``gs_objective``          the objective fun.py:358 minimises, profiled over the points
                              for the cameras of a given F: 0.5 * min_X sum of squared
                              reprojection residuals (per-point Gauss-Newton from the reference's
                              own triangulate_optimal start -- that start is NOT always optimal,
                              lab3.py:382-475 leaves up to ~1.4 px^2 per point on the table)
  * ``gold_standard_lm``      the same objective minimised to convergence (Levenberg-Marquardt,
                              Schur complement on the 12 camera parameters), from the same start
                              as fun.py:343-356.  scipy's TRF with a finite-difference Jacobian
                              stops on ftol = 1e-8 long before the minimum (20 021 evaluations
                              and cost 23.33 on the 180-inlier synthetic pair, where the minimum
                              is below 17.2), so the reference's F_gold is path dependent; the GPU
                              is checked against this converged restatement, and against the
                              reference through the objective: gs_objective(F_gpu) <=
                              gs_objective(F_gold reference).
  * ``camera_resectioning``   fun.py:181-188 (specRQ), 260-280
  * ``getEAndK``              fun.py:91-102
  * ``MakeHomogenous``        fun.py:48-55
  * ``specSVD`` / ``relative_camera_pose``  fun.py:190-258

Only ``tests/`` may import this module, and only as the checker.

Pinning: ``tests/test_oracle_golden.py`` compares every function here with the vectors the
reference itself produced (``tests/golden/make_golden_twoview.py`` -> ``twoview.npz``;
``make_golden.py`` -> ``dino_pnp_kat.npz`` / ``dino_c1.npz``).
"""
from __future__ import annotations

import numpy as np
import scipy.linalg
from scipy.optimize import least_squares

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])


def cross_matrix(v):
    v = np.asarray(v, dtype=np.float64).ravel()
    if v.size != 3:
        raise ValueError('Can only handle 3D vectors')
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def project(X, C):
    """Pinhole projection of (3,N) points through a 3x4 camera -> (2,N)."""
    Xh = np.vstack([X, np.ones((1, X.shape[1]))])
    y = C @ Xh
    return y[:2] / y[2]


def fmatrix_from_cameras(C1, C2):
    _, _, Vt = np.linalg.svd(C2)
    e = C1 @ Vt[3, :]
    return cross_matrix(e) @ (C1 @ np.linalg.pinv(C2))


def fmatrix_cameras(F):
    U, _, _ = np.linalg.svd(F)
    e1 = U[:, -1]
    return np.hstack([cross_matrix(e1) @ F, e1.reshape(-1, 1)]), I34.copy()


def fmatrix_epipoles(F):
    U, _, V = np.linalg.svd(F)
    e1 = U[:, -1] / U[-1, -1]
    e2 = V[-1, :] / V[-1, -1]
    return e1[:2], e2[:2]


def triangulate_linear(C1, C2, x1, x2):
    x1 = np.asarray(x1, dtype=np.float64).ravel()
    x2 = np.asarray(x2, dtype=np.float64).ravel()
    if x1.size == 2:
        x1 = np.append(x1, 1.0)
        x2 = np.append(x2, 1.0)
    M = np.vstack([cross_matrix(x1) @ C1, cross_matrix(x2) @ C2])
    X = np.linalg.svd(M)[2][-1, :]
    return X[:3] / X[-1]


def _poly6(a, b, c, d):
    """Coefficients (t^6 .. t^0) of lab3.py:428-439 with f1 = f2 = 1."""
    k1 = b * c - a * d
    return [a * c * k1,
            (a ** 2 + c ** 2) ** 2 + k1 * (b * c + a * d),
            4 * (a ** 2 + c ** 2) * (a * b + c * d) + 2 * a * c * k1 + b * d * k1,
            2 * (4 * a * b * c * d + a ** 2 * (3 * b ** 2) + c ** 2 * (3 * d ** 2 + b ** 2 * 2)),
            -a ** 2 * c * d + a * b * (4 * b ** 2 + c ** 2 + 4 * d ** 2 - 2 * d ** 2)
            + 2 * c * d * (2 * d ** 2 + b ** 2 * 3),
            b ** 4 - a ** 2 * d ** 2 + d ** 4 + b ** 2 * (c ** 2 + 2 * d ** 2),
            b * d * k1]


def triangulate_optimal(C1, C2, x1, x2):
    """lab3.py:382-475: move both points to the origin, rotate the epipoles onto the x axis,
    minimise the sum of squared image distances over the pencil of epipolar lines (roots of
    the degree-6 polynomial; real parts of all roots, plus the point at infinity), then
    triangulate the corrected points linearly."""
    T1 = np.array([[1., 0., x1[0]], [0., 1., x1[1]], [0., 0., 1.]])
    T2 = np.array([[1., 0., x2[0]], [0., 1., x2[1]], [0., 0., 1.]])
    F = T1.T @ (fmatrix_from_cameras(C1, C2) @ T2)
    e1, e2 = fmatrix_epipoles(F)
    e1 = e1 / np.linalg.norm(e1)
    e2 = e2 / np.linalg.norm(e2)
    R1 = np.array([[e1[0], e1[1], 0], [-e1[1], e1[0], 0], [0, 0, 1]])
    R2 = np.array([[e2[0], e2[1], 0], [-e2[1], e2[0], 0], [0, 0, 1]])
    F = R1 @ (F @ R2.T)
    a, b, c, d = F[1, 1], F[1, 2], F[2, 1], F[2, 2]
    r = np.real(np.roots(_poly6(a, b, c, d)))
    s = [t ** 2 / (1 + t ** 2) + (c * t + d) ** 2 / ((a * t + b) ** 2 + (c * t + d) ** 2)
         for t in r]
    s.append(1. + c ** 2 / (a ** 2 + c ** 2))
    i = int(np.argmin(s))
    if i < r.size:
        tm = r[i]
        l1 = np.array([-(c * tm + d), a * tm + b, c * tm + d])
        l2 = np.array([tm, 1., -tm])
    else:
        l1 = np.array([-c, a, c])
        l2 = np.array([1., 0., -1.])

    def closest(l):
        return np.array([-l[0] * l[2], -l[1] * l[2], l[0] ** 2 + l[1] ** 2])
    y1 = T1 @ (R1.T @ closest(l1))
    y2 = T2 @ (R2.T @ closest(l2))
    return triangulate_linear(C1, C2, y1, y2)


def fmatrix_residuals_gs(params, pl, pr):
    C1 = params[:12].reshape(3, 4)
    X = params[12:].reshape(-1, 3).T
    if X.shape[1] != pl.shape[1]:
        raise ValueError('Wrong size of parameter vector')
    return np.concatenate([(pl - project(X, C1)).ravel(), (pr - project(X, I34)).ravel()])


def fmatrix_residuals_gs_jac_2point(params, pl, pr):
    """scipy's approx_derivative(fmatrix_residuals_gs, params, method='2-point') -- the
    Jacobian least_squares forms at fun.py:358 -- without its 12 + 3N residual evaluations:
    a column perturbs one parameter, which moves only the residuals of the camera (every
    point's left pair) or of its point, and those are recomputed with the same numpy
    operations (np.dot per element is independent of the other columns), so every entry has
    scipy's bits; the zeros scipy forms as 0 / dx keep dx's sign, and the array is the
    transpose of a C-order (n, m) array, as scipy returns it (tests/test_oracle_twoview.py
    checks it against approx_derivative bit for bit)."""
    params = np.asarray(params, dtype=np.float64)
    n = pl.shape[1]
    sign = (params >= 0).astype(float) * 2 - 1
    h = np.finfo(np.float64).eps ** 0.5 * sign * np.maximum(1.0, np.abs(params))
    xp = params + h
    dx = xp - params
    f0 = fmatrix_residuals_gs(params, pl, pr)
    Jt = np.empty((12 + 3 * n, 4 * n))
    Jt[:] = 0.0 / dx[:, None]
    C1 = params[:12].reshape(3, 4)
    X = params[12:].reshape(-1, 3).T
    for j in range(12):
        Cp = C1.ravel().copy()
        Cp[j] = xp[j]
        r = (pl - project(X, Cp.reshape(3, 4))).ravel()
        Jt[j, :2 * n] = (r - f0[:2 * n]) / dx[j]
    idx = np.arange(n)
    for c in range(3):
        Xp = X.copy()
        Xp[c] = xp[12 + 3 * idx + c]
        r = np.concatenate([(pl - project(Xp, C1)).ravel(), (pr - project(Xp, I34)).ravel()])
        col = 12 + 3 * idx + c
        for q in range(4):
            Jt[col, q * n + idx] = (r[q * n:(q + 1) * n] - f0[q * n:(q + 1) * n]) / dx[col]
    return Jt.T


def gold_standard(F, pl, pr, **ls_kwargs):
    """fun.py:336-369 on the inliers (pl, pr): returns (F_gold, least_squares result)."""
    C1, _ = fmatrix_cameras(F)
    X = np.array([triangulate_optimal(C1, I34, a, b) for a, b in zip(pl.T, pr.T)])
    params = np.hstack([C1.ravel(), X.ravel()])
    kw = dict(xtol=2.22e-14, tr_solver='lsmr')
    kw.update(ls_kwargs)
    sol = least_squares(fmatrix_residuals_gs, params, args=(pl, pr), **kw)
    return fmatrix_from_cameras(sol.x[:12].reshape(3, 4), I34.copy()), sol


def gs_cost_at(C1, X, pl, pr):
    """0.5 * ||fmatrix_residuals_gs||^2 for cameras (C1, [I|0]) and points X (3,N)."""
    r = np.concatenate([(pl - project(X, C1)).ravel(), (pr - project(X, I34)).ravel()])
    return 0.5 * float(r @ r)


def _residuals_jac(C1, X, pl, pr):
    """Residuals r (4,N) of lab3.py:228-266 and their Jacobians: A (N,2,12) w.r.t. C1
    (row-major), B (N,4,3) w.r.t. each point."""
    N = X.shape[1]
    Xh = np.vstack([X, np.ones((1, N))])
    u, v, w = C1 @ Xh
    r = np.stack([pl[0] - u / w, pl[1] - v / w, pr[0] - X[0] / X[2], pr[1] - X[1] / X[2]])
    A = np.zeros((N, 2, 12))
    A[:, 0, 0:4] = -(Xh / w).T
    A[:, 0, 8:12] = (Xh * (u / w ** 2)).T
    A[:, 1, 4:8] = -(Xh / w).T
    A[:, 1, 8:12] = (Xh * (v / w ** 2)).T
    B = np.zeros((N, 4, 3))
    B[:, 0, :] = -(np.outer(w, C1[0, :3]) - np.outer(u, C1[2, :3])) / (w ** 2)[:, None]
    B[:, 1, :] = -(np.outer(w, C1[1, :3]) - np.outer(v, C1[2, :3])) / (w ** 2)[:, None]
    B[:, 2, 0] = -1.0 / X[2]
    B[:, 2, 2] = X[0] / X[2] ** 2
    B[:, 3, 1] = -1.0 / X[2]
    B[:, 3, 2] = X[1] / X[2] ** 2
    return r, A, B


def _refine_points(C1, X, pl, pr, iters=50):
    """Per-point Gauss-Newton (3 unknowns each) with step halving, cameras fixed."""
    X = X.copy()
    for _ in range(iters):
        r, _, B = _residuals_jac(C1, X, pl, pr)
        e0 = (r ** 2).sum(0)
        H = np.einsum('nki,nkj->nij', B, B) + 1e-12 * np.eye(3)
        g = np.einsum('nki,kn->ni', B, r)
        dx = -np.linalg.solve(H, g[..., None])[..., 0].T
        step = np.ones(X.shape[1])
        for _ in range(30):
            Xn = X + dx * step
            rn, _, _ = _residuals_jac(C1, Xn, pl, pr)
            e1 = (rn ** 2).sum(0)
            bad = ~(e1 <= e0)
            if not bad.any():
                break
            step = np.where(bad, step * 0.5, step)
        X = np.where(e1 <= e0, Xn, X)
        if np.abs(dx * step).max() < 1e-13 * (1 + np.abs(X).max()):
            break
    return X


def gs_objective(F, pl, pr):
    """0.5 * min over X of ||fmatrix_residuals_gs||^2 for the cameras of F (fun.py:358's
    objective profiled over the 3D points)."""
    C1, C2 = fmatrix_cameras(F)
    X = np.array([triangulate_optimal(C1, C2, a, b) for a, b in zip(pl.T, pr.T)]).T
    return gs_cost_at(C1, _refine_points(C1, X, pl, pr), pl, pr)


def gold_standard_lm(F, pl, pr, max_iter=500, ftol=1e-15, xtol=1e-15, trace=False):
    """fun.py:343-369 with the least-squares step run to convergence: Levenberg-Marquardt
    (Marquardt diagonal damping, Nielsen update) on (C1, X) with the 3x3 point blocks
    eliminated by the Schur complement.  Returns (F_gold, info dict)."""
    C1, _ = fmatrix_cameras(F)
    X = np.array([triangulate_optimal(C1, I34, a, b) for a, b in zip(pl.T, pr.T)]).T
    N = X.shape[1]
    lam, nu = 1e-3, 2.0
    r, A, B = _residuals_jac(C1, X, pl, pr)
    cost = 0.5 * float((r ** 2).sum())
    cost0, it, nacc = cost, 0, 0
    for it in range(1, max_iter + 1):
        U = np.einsum('nki,nkj->ij', A, A)
        gc = np.einsum('nki,kn->i', A, r[:2])
        W = np.einsum('nki,nkj->nij', A, B[:, :2, :])
        V = np.einsum('nki,nkj->nij', B, B)
        gx = np.einsum('nki,kn->ni', B, r)
        dU = np.diag(U).copy()
        dV = np.einsum('nii->ni', V).copy()
        accepted = False
        while not accepted:
            Vs = V + lam * np.einsum('ni,ij->nij', dV, np.eye(3))
            Vi = np.linalg.inv(Vs)
            WVi = np.einsum('nij,njk->nik', W, Vi)
            S = U + lam * np.diag(dU) - np.einsum('nik,njk->ij', WVi, W)
            rhs = -gc + np.einsum('nik,nk->i', WVi, gx)
            dc = np.linalg.solve(S, rhs)
            dx = np.einsum('nij,nj->ni', Vi, -gx - np.einsum('nki,k->ni', W, dc))
            pred = 0.5 * (lam * (dc @ (dU * dc) + (dx * dV * dx).sum()) - dc @ gc - (dx * gx).sum())
            C1n = C1 + dc.reshape(3, 4)
            Xn = X + dx.T
            rn = _residuals_jac(C1n, Xn, pl, pr)[0]
            cost_n = 0.5 * float((rn ** 2).sum())
            rho = (cost - cost_n) / pred if pred > 0 else -1.0
            if cost_n < cost and rho > 0:
                accepted = True
                small_f = (cost - cost_n) <= ftol * cost
                small_x = np.sqrt(dc @ dc + (dx * dx).sum()) <= xtol * (
                    np.sqrt((C1 ** 2).sum() + (X ** 2).sum()) + xtol)
                C1, X, cost = C1n, Xn, cost_n
                nacc += 1
                lam *= max(1.0 / 3.0, 1.0 - (2.0 * rho - 1.0) ** 3)
                nu = 2.0
                r, A, B = _residuals_jac(C1, X, pl, pr)
                if small_f or small_x:
                    return _gs_out(C1, X, cost0, cost, it, nacc, 1)
            else:
                lam *= nu
                nu *= 2.0
                if lam > 1e32:
                    return _gs_out(C1, X, cost0, cost, it, nacc, 2)
    return _gs_out(C1, X, cost0, cost, it, nacc, 0)


def _gs_out(C1, X, cost0, cost, it, nacc, status):
    return fmatrix_from_cameras(C1, I34.copy()), dict(C1=C1, X=X, cost_init=cost0, cost=cost,
                                                      iterations=it, accepted=nacc,
                                                      status=status)


def specRQ(M):
    U, Q = scipy.linalg.rq(M)
    if np.linalg.det(Q) == -1:
        U[0, :] = U[0, :] * -1.0
        Q[:, 0] = Q[:, 0] * -1.0
    return U, Q


def camera_resectioning(C):
    """fun.py:260-280: C = lambda K [R | t] with K upper triangular, K[2,2] = 1."""
    A = C[0:3, 0:3]
    b = C[:, -1]
    U, Q = specRQ(A)
    t = scipy.linalg.inv(U) @ b
    U = U / U[-1, -1]
    D = np.diag(np.sign(np.diag(U)))
    K = U @ D
    if np.linalg.det(D) == 1:
        R = D @ Q
        t = D @ t
    else:
        R = -1 * D @ Q
        t = -1 * D @ t
    return K, R, t


def getEAndK(C, F):
    """fun.py:91-102: K of the LAST camera of C (1, n, 3, 4); E = K^T F K."""
    K = None
    for i in range(C.shape[1]):
        K, _, _ = camera_resectioning(C[0, i])
    return K.T @ F @ K, K


def MakeHomogenous(K, coord):
    """fun.py:48-55: (n,2) pixel coordinates -> (n,3) C-normalised K^-1 [u, v, 1]."""
    h = np.vstack([coord.T[:2], np.ones((1, coord.shape[0]))])
    return (scipy.linalg.inv(K) @ h).T


def specSVD(M):
    U, S, V = scipy.linalg.svd(M)
    V = V.T
    dU, dV = np.linalg.det(U), np.linalg.det(V)
    U[:, -1] = dU * U[:, -1]
    V[:, -1] = dV * V[:, -1]
    S[-1] = dU * dV * S[-1]
    return U, S, V.T


def relative_camera_pose(E, y1, y2):
    """fun.py:209-258: the four (R, t) of E, chirality decided on ONE correspondence by
    optimal triangulation; the first candidate with both depths > 0 wins, else None."""
    U, _, VT = specSVD(E)
    V = VT.T
    W = np.array([[0., 1., 0.], [-1., 0., 0.], [0., 0., 1.]])
    Ra = V @ W @ U.T
    Rb = V @ W.T @ U.T
    v3 = V[:, -1]
    for R, t in ((Ra, v3), (Rb, v3), (Ra, -v3), (Rb, -v3)):
        C2 = np.hstack([R, t.reshape(3, 1)])
        x1 = triangulate_optimal(I34, C2, y1, y2)
        x2 = R @ x1 + t
        if x1[-1] > 0 and x2[-1] > 0:
            return R, t
    return None
