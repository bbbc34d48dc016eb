"""OpenCV-compatible entry points for the tables.py:141-145 call site.

``solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, ...)`` returns
``(retval, rvec (3,1), tvec (3,1), inliers (k,1) int32)`` like ``cv.solvePnPRansac`` and
``Rodrigues(src)`` returns ``(dst, jacobian)``, so ``Tables.addNewView`` drops them in.

What runs (rs_pnp_ransac_cv, pnp_kernels.hip), following OpenCV's solvePnPRansac structure:

  * up to ``iterationsCount`` 6-point hypotheses (DLT minimal solver on C-normalised points,
    pnp.py:132-160, with the sample's world points centred and RMS-scaled first -- without
    that conditioning the 12x12 DLT system does not survive pixel noise on compact, distant
    point sets such as BAdino2's reconstruction) are solved and scored on the GPU with
    OpenCV's test in PIXELS,
    ``|K pi(R x + t) - uv|^2 <= reprojectionError^2``;
  * OpenCV's sequential loop is replayed over that hypothesis order: a model replaces the best
    only if its inlier count exceeds ``max(best, modelPoints - 1)``, and each new best shrinks
    the budget with RANSACUpdateNumIters(confidence, outlier ratio, modelPoints, budget), so
    ``confidence`` stops the search early exactly as OpenCV's does (here modelPoints = 6, the
    DLT sample size; OpenCV's EPnP kernel samples 5);
  * the sampling stream is a fixed-seed Philox stream per call, the analogue of OpenCV seeding
    its RANSAC RNG with the same constant on every call: equal inputs give equal outputs;
  * the winning pose is refined on its consensus set by Levenberg-Marquardt on the pixel
    reprojection error (OpenCV's SOLVEPNP_ITERATIVE refinement, started from the RANSAC pose),
    and ``inliers`` is the RANSAC consensus set, in point order.

Limits: zero lens distortion only (tables.py:140 passes zeros); m >= 6 correspondences (the
DLT) where OpenCV's EPnP kernel accepts m >= 4 -- fewer return ``(False, None, None, None)``
and tables.add_new_view raises a ValueError naming the count.  OpenCV itself is absent and
unversioned here, so parity with its exact samples is unpinned; the tests
check the documented semantics (pixel threshold, adaptive budget, determinism).
"""
from __future__ import annotations

import numpy as np

from . import _ffi

# OpenCV constructs its RANSAC RNG as RNG((uint64)-1) on every call
CV_RANSAC_SEED = 0xFFFFFFFFFFFFFFFF
MODEL_POINTS = 6
LM_MAX_ITERS = 20  # OpenCV's solvePnP ITERATIVE: CvLevMarq criteria (20 iterations, FLT_EPSILON)

# the last call's RANSAC outcome before refinement: hypotheses the loop consumed, the winning
# hypothesis and its pose (diagnostics / tests)
last_ransac = {}


def Rodrigues(src, dst=None, jacobian=None):
    a = np.asarray(src, dtype=np.float64)
    if a.size == 3:
        r = a.reshape(3)
        th = np.linalg.norm(r)
        if th < 1e-300:
            return np.eye(3), None
        k = r / th
        Kx = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        return np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx), None
    R = a.reshape(3, 3)
    c = np.clip((np.trace(R) - 1) / 2, -1.0, 1.0)
    th = np.arccos(c)
    if th < 1e-12:
        return np.zeros((3, 1)), None
    if np.pi - th < 1e-6:  # near pi: axis from the symmetric part
        B = (R + np.eye(3)) / 2
        k = np.sqrt(np.maximum(np.diag(B), 0))
        i = int(np.argmax(k))
        k = B[:, i] / np.sqrt(B[i, i])
        return (th * k / np.linalg.norm(k)).reshape(3, 1), None
    w = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]]) / (2 * np.sin(th))
    return (th * w).reshape(3, 1), None


def project_points(X, rvec, tvec, K):
    """Pixel projections K pi(R x + t) (cv.projectPoints with zero distortion)."""
    R, _ = Rodrigues(rvec)
    q = np.asarray(X, dtype=np.float64).reshape(-1, 3) @ R.T + np.asarray(tvec).reshape(1, 3)
    p = q[:, :2] / q[:, 2:3]
    K = np.asarray(K, dtype=np.float64) / float(K[2][2])
    return np.stack((K[0, 0] * p[:, 0] + K[0, 1] * p[:, 1] + K[0, 2],
                     K[1, 1] * p[:, 1] + K[1, 2]), axis=1)


def _refine_lm(X, uv, K, rvec, tvec):
    from scipy.optimize import least_squares

    def res(x):
        return (project_points(X, x[:3], x[3:], K) - uv).ravel()

    x0 = np.concatenate((np.ravel(rvec), np.ravel(tvec)))
    r0 = res(x0)
    if not np.all(np.isfinite(r0)) or len(r0) < 6:
        return rvec, tvec
    sol = least_squares(res, x0, method="lm", max_nfev=LM_MAX_ITERS * 7,
                        xtol=np.finfo(np.float32).eps, ftol=np.finfo(np.float32).eps)
    if not np.all(np.isfinite(sol.x)) or sol.cost > 0.5 * float(r0 @ r0):
        return rvec, tvec  # CvLevMarq only accepts steps that lower the error
    return sol.x[:3].reshape(3, 1), sol.x[3:].reshape(3, 1)


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0,
                   confidence=0.99, inliers=None, flags=0, ctx=None):
    X = np.ascontiguousarray(np.asarray(objectPoints, dtype=np.float64).reshape(-1, 3))
    uv = np.ascontiguousarray(np.asarray(imagePoints, dtype=np.float64).reshape(-1, 2))
    if len(X) != len(uv):
        raise ValueError("objectPoints and imagePoints must have the same count")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise ValueError("only zero lens distortion is supported")
    K = np.ascontiguousarray(np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3))
    last_ransac.clear()
    if len(X) < MODEL_POINTS:
        return False, None, None, None
    ctx = ctx or _ffi.default_context()
    res = _ffi.PnpResult()
    inl = np.empty(len(X), np.int64)
    n_inl, used = _ffi.C.c_int64(0), _ffi.C.c_int64(0)
    _ffi.check(_ffi.lib().rs_pnp_ransac_cv(
        ctx.handle, _ffi.ptr(X, _ffi.C.c_double), _ffi.ptr(uv, _ffi.C.c_double), len(X),
        _ffi.ptr(K, _ffi.C.c_double), int(iterationsCount), CV_RANSAC_SEED,
        float(reprojectionError), float(confidence), MODEL_POINTS, _ffi.C.byref(res),
        _ffi.ptr(inl, _ffi.C.c_int64), _ffi.C.byref(n_inl), _ffi.C.byref(used)))
    last_ransac.update(iterations=int(used.value), best_index=int(res.best_index))
    if res.best_index < 0:
        return False, None, None, None
    inl = inl[:n_inl.value]
    last_ransac.update(R=np.array(res.R[:]).reshape(3, 3), t=np.array(res.t[:]))
    rv, _ = Rodrigues(last_ransac["R"])
    rv, tv = _refine_lm(X[inl], uv[inl], K, rv, np.array(res.t[:]))
    return True, rv.reshape(3, 1), tv.reshape(3, 1), inl.astype(np.int32).reshape(-1, 1)


SOLVEPNP_ITERATIVE = 0


def solvePnP(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
             useExtrinsicGuess=False, flags=SOLVEPNP_ITERATIVE, ctx=None):
    """``cv.solvePnP`` with OpenCV's SOLVEPNP_ITERATIVE semantics, the call behind the
    reference's ``pnp.p3p`` (pnp.py:7-10): the pose over ALL correspondences, initialised by the
    DLT (rs_pnp_dlt on the GPU; world points centred and RMS-scaled first, the conditioning
    OpenCV's DLT initialisation applies too) -- or by (rvec, tvec) when ``useExtrinsicGuess`` --
    then refined by Levenberg-Marquardt on the pixel reprojection error.  Returns
    ``(retval, rvec (3,1), tvec (3,1))``.  Zero distortion only; m >= 6 (the DLT; OpenCV's
    ITERATIVE also needs >= 6 non-coplanar points for its DLT start).  OpenCV is absent here,
    so parity with it is unpinned; the tests check the known answers (noise-free BAdino2
    views) and that the refinement never raises the reprojection error of its start."""
    if flags != SOLVEPNP_ITERATIVE:
        raise ValueError("only SOLVEPNP_ITERATIVE is provided")
    X = np.ascontiguousarray(np.asarray(objectPoints, dtype=np.float64).reshape(-1, 3))
    uv = np.ascontiguousarray(np.asarray(imagePoints, dtype=np.float64).reshape(-1, 2))
    if len(X) != len(uv):
        raise ValueError("objectPoints and imagePoints must have the same count")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise ValueError("only zero lens distortion is supported")
    K = np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3)
    if useExtrinsicGuess and rvec is not None and tvec is not None:
        r0 = np.asarray(rvec, dtype=np.float64).reshape(3, 1)
        t0 = np.asarray(tvec, dtype=np.float64).reshape(3, 1)
    else:
        if len(X) < 6:
            raise ValueError("SOLVEPNP_ITERATIVE needs at least 6 non-coplanar points for its DLT start")
        c = X.mean(axis=0)
        s = float(np.sqrt(np.mean(np.sum((X - c) ** 2, axis=1)))) or 1.0
        Xc = np.ascontiguousarray((X - c) / s)
        y = np.linalg.solve(K, np.vstack([uv.T, np.ones((1, len(uv)))])).T
        y = np.ascontiguousarray(y)
        R = np.empty(9)
        t = np.empty(3)
        _ffi.check(_ffi.lib().rs_pnp_dlt((ctx or _ffi.default_context()).handle,
                                         _ffi.ptr(Xc, _ffi.C.c_double), _ffi.ptr(y, _ffi.C.c_double),
                                         len(X), _ffi.ptr(R, _ffi.C.c_double),
                                         _ffi.ptr(t, _ffi.C.c_double)))
        R = R.reshape(3, 3)
        if not np.all(np.isfinite(R)):
            return False, None, None
        # the conditioned frame: x = s x' + c, so R x + t = s (R x' + t') gives t = s t' - R c
        r0, _ = Rodrigues(R)
        t0 = (s * t - R @ c).reshape(3, 1)
    rv, tv = _refine_lm(X, uv, K, r0, t0)
    return True, np.asarray(rv, dtype=np.float64).reshape(3, 1), np.asarray(tv, dtype=np.float64).reshape(3, 1)
