"""ORACLE -- test infrastructure only, never shipped, never measured as the product.

CPU numpy restatement of the per-view SfM steps around PnP in the reference
(bioengstrom/tsbb15-3d-reconstruction-project, snapshot v0, tables.py / fun.py):

  * ``match_observations``   tables.py:116-135  the 2D<->3D matching loop of addNewView: for
                             each putative correspondence, the FIRST observation of the last
                             view (in its observations_index order -- which starts with the
                             spurious 0 of help_classes.View.__init__) with
                             ||obs - y1_hom|| < 1e-4
  * ``getEFromCameras``      fun.py:12-21       E = R^T [t]_x of the relative pose
  * ``add_new_points``       tables.py:161-175  epipolar gate |y1^T E y2| < 0.1, then
                             lab3.triangulate_optimal of the accepted pairs
  * ``ba_residuals``         tables.py:264-293  EpsilonBA: r = [u - c1.x / c3.x,
                             v - c2.x / c3.x] per observation, cameras as 12 free parameters
  * ``ba_sparsity``          tables.py:339-372  the jac_sparsity mask (camera 0 columns zeroed)
  * ``ba_jacobian``          the analytic Jacobian blocks of ba_residuals
  * ``bundle_adjust_lm``     the objective of BundleAdjustment2 minimised to convergence
                             (Levenberg-Marquardt, Schur complement on the cameras, camera 0
                             fixed as the reference's mask fixes it)

Only ``tests/`` may import this module, and only as the checker.  Pinned by
``tests/test_oracle_tables.py`` against ``tests/golden/tables.npz`` (written from the
reference by ``tests/golden/make_golden_tables.py``).
"""
from __future__ import annotations

import numpy as np

from . import twoview_ref as tv


def match_observations(obs_coords, obs_point, queries, tol=1e-4):
    """Per query: the 3D point index of the first observation within ``tol``, else -1."""
    out = np.full(len(queries), -1, dtype=np.int64)
    for i, q in enumerate(queries):
        for c, p in zip(obs_coords, obs_point):
            if np.linalg.norm(c - q) < tol:
                out[i] = p
                break
    return out


def getEFromCameras(R1, t1, R2, t2):
    R = R2 @ R1.T
    t = t2 - (R2 @ R1.T @ t1)
    tx = np.array([[0.0, -t[2], t[1]], [t[2], 0.0, -t[0]], [-t[1], t[0], 0.0]])
    return R.T @ tx


def add_new_points(y1_hom, y2_hom, C1, C2, gate=0.1):
    """C1, C2: (3,4) [R | t] cameras.  Returns (accepted mask, X (k,3) of the accepted)."""
    E = getEFromCameras(C1[:, :3], C1[:, 3], C2[:, :3], C2[:, 3])
    mask = np.array([abs(a.T @ E @ b) < gate for a, b in zip(y1_hom, y2_hom)], dtype=bool)
    X = np.array([tv.triangulate_optimal(C1, C2, a, b)
                  for a, b, k in zip(y1_hom, y2_hom, mask) if k]).reshape(-1, 3)
    return mask, X


def ba_residuals(cams, pts, obs_view, obs_point, u, v):
    """EpsilonBA (tables.py:264-293): (2 nObs,) interleaved [r_u, r_v] per observation."""
    c = cams[obs_view]                                   # (n, 3, 4)
    xh = np.hstack([pts[obs_point], np.ones((len(obs_point), 1))])
    a = np.einsum('nk,nk->n', c[:, 0], xh)
    b = np.einsum('nk,nk->n', c[:, 1], xh)
    w = np.einsum('nk,nk->n', c[:, 2], xh)
    r = np.empty(2 * len(u))
    r[0::2] = u - a / w
    r[1::2] = v - b / w
    return r


def ba_sparsity(n_views, n_points, obs_view, obs_point):
    """Dense 0/1 version of Tables.sparsity_mask (camera 0 columns zeroed)."""
    m = np.zeros((2 * len(obs_view), 12 * n_views + 3 * n_points), dtype=np.int64)
    for i, (c, p) in enumerate(zip(obs_view, obs_point)):
        m[2 * i:2 * i + 2, 12 * c:12 * c + 12] = 1
        m[2 * i:2 * i + 2, 12 * n_views + 3 * p:12 * n_views + 3 * p + 3] = 1
    m[:, 0:12] = 0
    return m


def ba_jacobian(cams, pts, obs_view, obs_point):
    """Per observation: Jc (2,12) w.r.t. its camera's row-major entries, Jp (2,3) w.r.t. its
    point (d r / d params; camera 0's blocks are returned too -- the mask zeroes them)."""
    c = cams[obs_view]
    n = len(obs_view)
    xh = np.hstack([pts[obs_point], np.ones((n, 1))])
    a = np.einsum('nk,nk->n', c[:, 0], xh)
    b = np.einsum('nk,nk->n', c[:, 1], xh)
    w = np.einsum('nk,nk->n', c[:, 2], xh)
    Jc = np.zeros((n, 2, 12))
    Jc[:, 0, 0:4] = -xh / w[:, None]
    Jc[:, 0, 8:12] = xh * (a / w ** 2)[:, None]
    Jc[:, 1, 4:8] = -xh / w[:, None]
    Jc[:, 1, 8:12] = xh * (b / w ** 2)[:, None]
    Jp = np.zeros((n, 2, 3))
    Jp[:, 0] = -(c[:, 0, :3] * w[:, None] - c[:, 2, :3] * a[:, None]) / (w ** 2)[:, None]
    Jp[:, 1] = -(c[:, 1, :3] * w[:, None] - c[:, 2, :3] * b[:, None]) / (w ** 2)[:, None]
    return Jc, Jp


def bundle_adjust_lm(cams, pts, obs_view, obs_point, u, v, max_iter=200, ftol=1e-15):
    """BundleAdjustment2's objective minimised by LM (Marquardt damping, Nielsen update),
    points eliminated (Schur), camera 0 fixed.  Returns (cams, pts, info)."""
    cams = cams.copy()
    pts = pts.copy()
    nC, nP = len(cams), len(pts)
    free = np.arange(1, nC)
    lam, nu = 1e-3, 2.0

    def cost_of(cm, pt):
        r = ba_residuals(cm, pt, obs_view, obs_point, u, v)
        return 0.5 * float(r @ r), r

    cost, r = cost_of(cams, pts)
    cost0 = cost
    it = 0
    for it in range(1, max_iter + 1):
        Jc, Jp = ba_jacobian(cams, pts, obs_view, obs_point)
        rr = r.reshape(-1, 2)
        U = np.zeros((nC, 12, 12))
        gc = np.zeros((nC, 12))
        V = np.zeros((nP, 3, 3))
        gp = np.zeros((nP, 3))
        np.add.at(U, obs_view, np.einsum('nki,nkj->nij', Jc, Jc))
        np.add.at(gc, obs_view, np.einsum('nki,nk->ni', Jc, rr))
        np.add.at(V, obs_point, np.einsum('nki,nkj->nij', Jp, Jp))
        np.add.at(gp, obs_point, np.einsum('nki,nk->ni', Jp, rr))
        Wn = np.einsum('nki,nkj->nij', Jc, Jp)            # per observation (12,3)
        while True:
            Vs = V + lam * np.einsum('pi,ij->pij', np.einsum('pii->pi', V), np.eye(3))
            Vi = np.linalg.inv(Vs)
            nf = len(free)
            S = np.zeros((12 * nf, 12 * nf))
            rhs = np.zeros(12 * nf)
            pos = {c: k for k, c in enumerate(free)}
            for k, c in enumerate(free):
                Uc = U[c] + lam * np.diag(np.diag(U[c]))
                S[12 * k:12 * k + 12, 12 * k:12 * k + 12] += Uc
                rhs[12 * k:12 * k + 12] -= gc[c]
            for p in range(nP):
                idx = np.flatnonzero(obs_point == p)
                for i in idx:
                    ci = obs_view[i]
                    if ci not in pos:
                        continue
                    WVi = Wn[i] @ Vi[p]
                    rhs[12 * pos[ci]:12 * pos[ci] + 12] += WVi @ gp[p]
                    for j in idx:
                        cj = obs_view[j]
                        if cj not in pos:
                            continue
                        S[12 * pos[ci]:12 * pos[ci] + 12, 12 * pos[cj]:12 * pos[cj] + 12] -= \
                            WVi @ Wn[j].T
            dcf = np.linalg.solve(S, rhs)
            dc = np.zeros((nC, 12))
            dc[free] = dcf.reshape(-1, 12)
            gx = gp.copy()
            for i in range(len(obs_view)):
                gx[obs_point[i]] += Wn[i].T @ dc[obs_view[i]]
            dx = -np.einsum('pij,pj->pi', Vi, gx)
            dU = np.einsum('cii->ci', U)
            dV = np.einsum('pii->pi', V)
            pred = 0.5 * (lam * ((dc * dU * dc).sum() + (dx * dV * dx).sum())
                          - (dc * gc).sum() - (dx * gp).sum())
            cams_n = cams + dc.reshape(nC, 3, 4)
            pts_n = pts + dx
            cost_n, r_n = cost_of(cams_n, pts_n)
            if cost_n < cost and pred > 0:
                rho = (cost - cost_n) / pred
                small = (cost - cost_n) <= ftol * cost
                cams, pts, cost, r = cams_n, pts_n, cost_n, r_n
                t = 2 * rho - 1
                lam *= max(1 / 3, 1 - t ** 3)
                nu = 2.0
                if small:
                    return cams, pts, dict(cost_init=cost0, cost=cost, iterations=it, status=1)
                break
            lam *= nu
            nu *= 2
            if lam > 1e32:
                return cams, pts, dict(cost_init=cost0, cost=cost, iterations=it, status=2)
    return cams, pts, dict(cost_init=cost0, cost=cost, iterations=it, status=0)
