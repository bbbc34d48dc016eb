"""Two-view geometry after RANSAC on the GPU.

Every function here runs in librsamd's HIP kernels (twoview.hip); the reference functions
they replace:

  * ``fmatrix_cameras(F)``                     lab3.py:353-380   (rs_fmatrix_cameras)
  * ``fmatrix_from_cameras(C1, C2)``           lab3.py:331-351   (rs_fmatrix_from_cameras)
  * ``triangulate_optimal(C1, C2, x1, x2)``    lab3.py:382-475   (rs_triangulate_optimal)
  * ``triangulate_optimal_batch``              the same over many points / camera pairs
  * ``camera_resectioning(C)``                 fun.py:260-280    (rs_camera_resectioning)
  * ``getEAndK(C, F)``                         fun.py:91-102     (+ rs_essential_from_f)
  * ``relative_camera_pose(E, y1, y2)``        fun.py:209-258    (rs_relative_camera_pose)
  * ``gold_standard(F, pl, pr)``               fun.py:336-369    (rs_gold_standard)
  * ``gold_standard_batch(Fs, pls, prs)``      the same, one workgroup per pair
  * ``gold_standard_trf(F, pl, pr)``           fun.py:336-369 as the reference runs it:
    scipy's TRF (least_squares(xtol=2.22e-14, tr_solver='lsmr'), fun.py:358) on the host with
    the residual and its forward-difference Jacobian on the GPU (rs_gs_residuals_fd)

``MakeHomogenous`` (fun.py:48-55) and ``project`` are input / output formatting helpers.
``gold_standard`` minimises the reference's objective (lab3.fmatrix_residuals_gs) to
convergence; the reference's scipy TRF stops on ftol = 1e-8 at a path-dependent point with a
higher objective (see oracle/twoview_ref.py and DESIGN.md).  ``gold_standard_trf`` follows that
TRF path itself; where it stops depends on the last bits of every residual (the reference's
own result moves by ~1e-5 between one and eight BLAS threads), so it lands near, not on, the
reference's F_gold.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _ffi

I34 = np.hstack([np.eye(3), np.zeros((3, 1))])
_d = _ffi.C.c_double


def _ctx(ctx):
    return (ctx or _ffi.default_context()).handle


def _cam(C):
    C = _ffi.f64c(C)
    if C.shape[-2:] != (3, 4):
        raise ValueError('C is not a valid camera matrix')
    return C


def fmatrix_cameras(F, ctx=None):
    """lab3.fmatrix_cameras: (C1, C2) with C2 = [I | 0] and C1 = [[e1]_x F | e1]."""
    Fc = _ffi.f64c(F)
    if Fc.shape != (3, 3):
        raise ValueError('F must be (3, 3)')
    C1 = np.empty((3, 4))
    _ffi.check(_ffi.lib().rs_fmatrix_cameras(_ctx(ctx), _ffi.ptr(Fc, _d), 1, _ffi.ptr(C1, _d)))
    return C1, I34.copy()


def fmatrix_from_cameras(C1, C2, ctx=None):
    """lab3.fmatrix_from_cameras: F = [C1 n]_x C1 C2^+ (n the centre of C2)."""
    a, b = _cam(C1), _cam(C2)
    F = np.empty((3, 3))
    _ffi.check(_ffi.lib().rs_fmatrix_from_cameras(_ctx(ctx), _ffi.ptr(a, _d), _ffi.ptr(b, _d), 1,
                                                  _ffi.ptr(F, _d)))
    return F


def triangulate_optimal_batch(C1, C2, x1, x2, cam=None, ctx=None):
    """Optimal triangulation of many correspondences.  C1, C2: (3,4) or (k,3,4); x1, x2:
    (2, n); cam: (n,) camera-pair index per point (None: pair 0).  Returns X (n, 3)."""
    a = _cam(C1).reshape(-1, 3, 4)
    b = _cam(C2).reshape(-1, 3, 4)
    if a.shape != b.shape:
        raise ValueError('C1 and C2 batches differ')
    x1, x2 = _ffi.f64c(x1), _ffi.f64c(x2)
    if x1.shape != x2.shape or x1.ndim != 2 or x1.shape[0] != 2:
        raise ValueError('x1 and x2 must both be (2, n)')
    n = x1.shape[1]
    cp = None
    if cam is not None:
        cam = np.ascontiguousarray(cam, dtype=np.int32)
        if cam.shape != (n,):
            raise ValueError('cam must be (n,)')
        cp = _ffi.ptr(cam, _ffi.C.c_int32)
    X = np.empty((n, 3))
    _ffi.check(_ffi.lib().rs_triangulate_optimal(_ctx(ctx), _ffi.ptr(a, _d), _ffi.ptr(b, _d),
                                                 a.shape[0], _ffi.ptr(x1, _d), _ffi.ptr(x2, _d),
                                                 cp, n, _ffi.ptr(X, _d)))
    return X


def triangulate_optimal(C1, C2, x1, x2, ctx=None):
    """lab3.triangulate_optimal for one correspondence: x1, x2 (2,) -> X (3,)."""
    x1 = np.asarray(x1, dtype=np.float64).reshape(2, 1)
    x2 = np.asarray(x2, dtype=np.float64).reshape(2, 1)
    return triangulate_optimal_batch(C1, C2, x1, x2, ctx=ctx)[0]


def camera_resectioning_batch(P, ctx=None):
    """fun.camera_resectioning over (B,3,4) cameras -> K, R (B,3,3), t (B,3)."""
    P = _cam(P).reshape(-1, 3, 4)
    B = P.shape[0]
    K, R, t = np.empty((B, 3, 3)), np.empty((B, 3, 3)), np.empty((B, 3))
    _ffi.check(_ffi.lib().rs_camera_resectioning(_ctx(ctx), _ffi.ptr(P, _d), B, _ffi.ptr(K, _d),
                                                 _ffi.ptr(R, _d), _ffi.ptr(t, _d)))
    return K, R, t


def camera_resectioning(C, ctx=None):
    """fun.camera_resectioning: C = lambda K [R | t] -> (K, R, t)."""
    K, R, t = camera_resectioning_batch(np.asarray(C).reshape(1, 3, 4), ctx)
    return K[0], R[0], t[0]


def essential_batch(K, F, ctx=None):
    """E = K^T F K for F (B,3,3) and K (3,3) or (B,3,3)."""
    F = _ffi.f64c(F).reshape(-1, 3, 3)
    K = _ffi.f64c(K)
    one = K.shape == (3, 3)
    if not one and K.shape != F.shape:
        raise ValueError('K must be (3, 3) or match F')
    E = np.empty_like(F)
    _ffi.check(_ffi.lib().rs_essential_from_f(_ctx(ctx), _ffi.ptr(K, _d), int(one),
                                              _ffi.ptr(F, _d), F.shape[0], _ffi.ptr(E, _d)))
    return E


def getEAndK(C, F, ctx=None):
    """fun.getEAndK: resection every camera of C (1, n, 3, 4) on the GPU; K of the LAST one
    (the reference overwrites K in its loop, fun.py:96-98); E = K^T F K."""
    C = np.asarray(C, dtype=np.float64)
    K, _, _ = camera_resectioning_batch(C[0], ctx)
    Kl = np.ascontiguousarray(K[-1])
    return essential_batch(Kl, np.asarray(F).reshape(1, 3, 3), ctx)[0], Kl


def MakeHomogenous(K, coord):
    """fun.MakeHomogenous: (n, 2) pixels -> (n, 3) C-normalised K^-1 [u, v, 1] (formatting)."""
    coord = np.asarray(coord, dtype=np.float64)
    h = np.vstack([coord.T[:2], np.ones((1, coord.shape[0]))])
    return np.linalg.solve(np.asarray(K, dtype=np.float64), h).T


def normalise_each(K, coord):
    """K^-1 [u, v, 1] for each row (u, v) of coord (n, 2) -- the C-normalised first
    correspondence main.py:59-63 passes to relative_camera_pose, as fun.MakeHomogenous forms it
    (scipy.linalg.inv(K) @ coord_hom, fun.py:48-55) -- with elementwise products and sums, so
    a point's bits do not depend on how many are normalised together (a BLAS product may
    round differently per batch size: the batched pair paths must agree field for field)."""
    coord = np.asarray(coord, dtype=np.float64).reshape(-1, 2)
    Ki = np.linalg.inv(np.asarray(K, dtype=np.float64))
    u, v = coord[:, 0], coord[:, 1]
    out = np.empty((coord.shape[0], 3))
    for r in range(3):
        out[:, r] = (Ki[r, 0] * u + Ki[r, 1] * v) + Ki[r, 2]
    return out


def relative_camera_pose_batch(E, y1, y2, ctx=None):
    """fun.relative_camera_pose over pairs: E (B,3,3), y1, y2 (B,2).  Returns R (B,3,3),
    t (B,3), found (B,) int32 (0 where the reference returns None)."""
    E = _ffi.f64c(E).reshape(-1, 3, 3)
    B = E.shape[0]
    y1 = _ffi.f64c(y1).reshape(B, 2)
    y2 = _ffi.f64c(y2).reshape(B, 2)
    R, t = np.empty((B, 3, 3)), np.empty((B, 3))
    found = np.empty(B, dtype=np.int32)
    _ffi.check(_ffi.lib().rs_relative_camera_pose(
        _ctx(ctx), _ffi.ptr(E, _d), _ffi.ptr(y1, _d), _ffi.ptr(y2, _d), B, _ffi.ptr(R, _d),
        _ffi.ptr(t, _d), _ffi.ptr(found, _ffi.C.c_int32)))
    return R, t, found


def relative_camera_pose(E, y1, y2, ctx=None):
    """fun.relative_camera_pose: (R, t) of the first chirality-valid candidate, or None."""
    R, t, f = relative_camera_pose_batch(E, np.asarray(y1)[:2], np.asarray(y2)[:2], ctx)
    if f[0] == 0:
        return None
    return R[0], t[0]


def project(X, C):
    """Pinhole projection of (3,) or (3,N) points through a 3x4 camera (formatting helper)."""
    X = np.asarray(X, dtype=np.float64)
    one = X.ndim == 1
    Xr = X.reshape(3, -1)
    y = C @ np.vstack([Xr, np.ones((1, Xr.shape[1]))])
    y = y[:2] / y[2]
    return y.ravel() if one else y


@dataclass
class GoldStandard:
    F: np.ndarray          # F_gold (3,3)
    C1: np.ndarray         # refined first camera (3,4); C2 = [I | 0]
    X: np.ndarray          # refined 3D points (n,3)
    cost_init: float       # 0.5 |r|^2 at the reference's start (fun.py:343-356)
    cost: float            # 0.5 |r|^2 at the end
    iterations: int
    status: int            # 0 max_iter, 1 converged, 2 no further decrease


MAX_ITER = 500


def gold_standard_batch(Fs, pls, prs, max_iter=MAX_ITER, ctx=None):
    """fun.py:336-369 for many pairs at once: Fs (B,3,3) F_RANSAC; pls, prs lists of (2, n_b)
    inlier point sets.  Returns a list of :class:`GoldStandard`."""
    Fs = _ffi.f64c(Fs).reshape(-1, 3, 3)
    B = Fs.shape[0]
    if len(pls) != B or len(prs) != B:
        raise ValueError('one point set per F')
    ns = []
    for a, b in zip(pls, prs):
        a, b = np.asarray(a), np.asarray(b)
        if a.shape != b.shape or a.ndim != 2 or a.shape[0] != 2:
            raise ValueError('point sets must be (2, n) pairs')
        ns.append(a.shape[1])
    off = np.zeros(B + 1, dtype=np.int64)
    off[1:] = np.cumsum(ns)
    total = int(off[-1])
    pl = _ffi.f64c(np.hstack([np.asarray(a, np.float64) for a in pls]) if total else np.zeros((2, 0)))
    pr = _ffi.f64c(np.hstack([np.asarray(b, np.float64) for b in prs]) if total else np.zeros((2, 0)))
    Fg = np.empty((B, 3, 3))
    C1 = np.empty((B, 3, 4))
    X = np.empty((max(total, 1), 3))
    info = (_ffi.GsInfo * B)()
    _ffi.check(_ffi.lib().rs_gold_standard(
        _ctx(ctx), _ffi.ptr(Fs, _d), _ffi.ptr(pl, _d), _ffi.ptr(pr, _d),
        _ffi.ptr(off, _ffi.C.c_int64), B, int(max_iter), _ffi.ptr(Fg, _d), _ffi.ptr(C1, _d),
        _ffi.ptr(X, _d), info))
    return [GoldStandard(Fg[b], C1[b], X[off[b]:off[b + 1]].copy(), info[b].cost_init,
                         info[b].cost, info[b].iterations, info[b].status) for b in range(B)]


GS_INFO_DTYPE = np.dtype([("cost_init", "<f8"), ("cost", "<f8"), ("iterations", "<i4"),
                          ("accepted", "<i4"), ("status", "<i4"), ("n", "<i4")])


def gold_standard_arrays(Fs, pl, pr, off, max_iter=MAX_ITER, ctx=None, want_points=True):
    """gold_standard_batch on pre-concatenated inlier points (pl, pr (2, total), off (B + 1)):
    (F_gold (B,3,3), C1 (B,3,4), X (total,3), info as a GS_INFO_DTYPE array), no Python object
    per pair.  want_points=False: C1 and X are not copied back (None)."""
    Fs = _ffi.f64c(Fs).reshape(-1, 3, 3)
    B = Fs.shape[0]
    off = np.ascontiguousarray(off, dtype=np.int64)
    pl, pr = _ffi.f64c(pl), _ffi.f64c(pr)
    if off.shape != (B + 1,) or pl.shape != pr.shape or pl.shape != (2, int(off[-1])):
        raise ValueError('pl, pr must be (2, off[-1]) with one offset per F')
    Fg = np.empty((B, 3, 3))
    C1 = np.empty((B, 3, 4)) if want_points else None
    X = np.empty((max(int(off[-1]), 1), 3)) if want_points else None
    info = (_ffi.GsInfo * B)()
    _ffi.check(_ffi.lib().rs_gold_standard(
        _ctx(ctx), _ffi.ptr(Fs, _d), _ffi.ptr(pl, _d), _ffi.ptr(pr, _d),
        _ffi.ptr(off, _ffi.C.c_int64), B, int(max_iter), _ffi.ptr(Fg, _d),
        _ffi.ptr(C1, _d) if want_points else None, _ffi.ptr(X, _d) if want_points else None, info))
    return Fg, C1, X, np.frombuffer(info, dtype=GS_INFO_DTYPE).copy()


def gold_standard(F, pl, pr, max_iter=MAX_ITER, ctx=None):
    """F_gold of fun.py:336-369 from F_RANSAC and the inlier points pl, pr (2, n)."""
    return gold_standard_batch(np.asarray(F).reshape(1, 3, 3), [pl], [pr], max_iter, ctx)[0].F


_EPS_2POINT = float(np.finfo(np.float64).eps) ** 0.5  # scipy _eps_for_method(f64, f64, '2-point')


def gs_residuals(x, pl, pr, ctx=None):
    """lab3.fmatrix_residuals_gs(params, pl, pr) on the GPU: (4n,) left x, left y, right x,
    right y."""
    x = _ffi.f64c(x)
    pl, pr = _ffi.f64c(pl), _ffi.f64c(pr)
    n = pl.shape[1]
    if pl.shape != pr.shape or x.shape != (12 + 3 * n,):
        raise ValueError('Wrong size of parameter vector')
    f = np.empty(4 * n)
    _ffi.check(_ffi.lib().rs_gs_residuals_fd(_ctx(ctx), _ffi.ptr(x, _d), None, None,
                                             _ffi.ptr(pl, _d), _ffi.ptr(pr, _d), n,
                                             _ffi.ptr(f, _d), None))
    return f


def gs_jacobian_2point(x, pl, pr, ctx=None):
    """The Jacobian scipy's approx_derivative(method='2-point') forms for
    lab3.fmatrix_residuals_gs at x (steps and dx exactly as scipy computes them), on the GPU."""
    x = _ffi.f64c(x)
    pl, pr = _ffi.f64c(pl), _ffi.f64c(pr)
    n = pl.shape[1]
    if pl.shape != pr.shape or x.shape != (12 + 3 * n,):
        raise ValueError('Wrong size of parameter vector')
    sign = (x >= 0).astype(float) * 2 - 1
    h = _EPS_2POINT * sign * np.maximum(1.0, np.abs(x))
    xp = x + h
    dx = xp - x
    f = np.empty(4 * n)
    Jt = np.empty((12 + 3 * n, 4 * n))
    _ffi.check(_ffi.lib().rs_gs_residuals_fd(_ctx(ctx), _ffi.ptr(x, _d), _ffi.ptr(xp, _d),
                                             _ffi.ptr(dx, _d), _ffi.ptr(pl, _d),
                                             _ffi.ptr(pr, _d), n, _ffi.ptr(f, _d),
                                             _ffi.ptr(Jt, _d)))
    # scipy's approx_derivative returns J_transposed.T (Fortran order); LSMR's BLAS products
    # with J depend on that layout, and so does the TRF path (tools/gs_trace_cpu.py)
    return Jt.T


@dataclass
class GoldStandardTRF:
    F: np.ndarray
    C1: np.ndarray
    X: np.ndarray
    cost_init: float
    cost: float
    nfev: int
    status: int   # scipy least_squares status (1 gtol, 2 ftol, 3 xtol, 4 ftol and xtol, 0 max_nfev)


def gs_trf(params, pl, pr, ctx=None):
    """fun.py:358 from a given start: scipy.optimize.least_squares(fmatrix_residuals_gs,
    params, xtol=2.22e-14, tr_solver='lsmr') with the residual and the 2-point Jacobian
    computed on the GPU in the reference's bits and layout; returns scipy's result.  From the
    reference's start it retraces the reference's path evaluation for evaluation
    (tests/test_gpu_twoview.py against tests/golden/gs_trace.npz)."""
    from scipy.optimize import least_squares
    return least_squares(gs_residuals, _ffi.f64c(params), jac=gs_jacobian_2point,
                         xtol=2.22e-14, tr_solver='lsmr', args=(pl, pr), kwargs={"ctx": ctx})


def gold_standard_trf_full(F, pl, pr, ctx=None):
    """fun.py:343-369 as the reference runs it.  Cameras from F_RANSAC and the optimal
    triangulation of the inliers on the GPU, then scipy.optimize.least_squares with the
    reference's options (fun.py:358: method 'trf', xtol=2.22e-14, tr_solver='lsmr', default
    ftol / gtol / x_scale / max_nfev) over a residual and a forward-difference Jacobian
    computed on the GPU, then F from the refined cameras on the GPU."""
    pl = _ffi.f64c(pl)
    pr = _ffi.f64c(pr)
    if pl.shape != pr.shape or pl.ndim != 2 or pl.shape[0] != 2:
        raise ValueError('pl and pr must both be (2, n)')
    C1, C2 = fmatrix_cameras(F, ctx)
    X = triangulate_optimal_batch(C1, C2, pl, pr, ctx=ctx)      # fun.py:352
    params = np.hstack((C1.ravel(), X.ravel()))                  # fun.py:355
    f0 = gs_residuals(params, pl, pr, ctx)
    res = gs_trf(params, pl, pr, ctx)
    C1g = res.x[:12].reshape(3, 4)
    Fg = fmatrix_from_cameras(C1g, I34, ctx)                     # fun.py:362-368
    return GoldStandardTRF(Fg, C1g, res.x[12:].reshape(-1, 3), 0.5 * float(f0 @ f0),
                           float(res.cost), int(res.nfev), int(res.status))


def gold_standard_trf(F, pl, pr, ctx=None):
    """F_gold of fun.py:336-369 along the reference's own TRF path (see gold_standard_trf_full)."""
    return gold_standard_trf_full(F, pl, pr, ctx).F
