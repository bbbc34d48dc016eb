"""OpenCV-compatible entry points for the tables.py:141-145 call site and pnp.py:7-10.

``solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, ...)`` returns
``(retval, rvec (3,1), tvec (3,1), inliers (k,1) int32)`` like ``cv.solvePnPRansac``,
``solvePnP`` returns ``(retval, rvec, tvec)`` and ``Rodrigues(src)`` returns
``(dst, jacobian)``, so ``Tables.addNewView`` and ``pnp.p3p`` drop them in.

What runs (rs_pnp_ransac_cv, pnp_kernels.hip / pnp_minimal.h), following OpenCV's
solvePnPRansac structure:

  * the minimal solver is OpenCV's RANSAC kernel: EPnP on 5-point samples, or -- for exactly
    4 correspondences and for ``flags`` SOLVEPNP_P3P -- P3P on 4 (Lambda Twist on three, the
    fourth choosing); up to ``iterationsCount`` hypotheses are solved and scored on the GPU
    with OpenCV's test in PIXELS, ``|K pi(R x + t) - uv|^2 <= reprojectionError^2``;
  * with as many correspondences as the sample size OpenCV solves once with that kernel and
    returns every point as an inlier; so does this;
  * OpenCV's sequential loop is replayed over the hypothesis order: a model replaces the best
    only if its inlier count exceeds ``max(best, modelPoints - 1)``, and each new best shrinks
    the budget with RANSACUpdateNumIters(confidence, outlier ratio, modelPoints, budget);
  * the sampling stream is a fixed-seed Philox stream per call, the analogue of OpenCV seeding
    its RANSAC RNG with the same constant on every call: equal inputs give equal outputs;
  * the winner is refined on its consensus set as OpenCV does with ``flags``: Levenberg-
    Marquardt on the pixel reprojection error for SOLVEPNP_ITERATIVE (started from the RANSAC
    pose; one GPU workgroup, rs_pnp_refine_lm), EPnP over the consensus set for SOLVEPNP_EPNP,
    none for SOLVEPNP_P3P;
  * ``useExtrinsicGuess`` with ``rvec``/``tvec``: the guess is scored first, as hypothesis 0
    (OpenCV's kernels ignore it; here a good guess is kept unless a sample beats it).

Limits: zero lens distortion only (tables.py:140 passes zeros); other ``flags`` raise
ValueError.  OpenCV itself is absent and unversioned here, so parity with
its exact samples is unpinned; the tests check known answers (BAdino2 views, including 4- and
5-point subsets) and the documented semantics (pixel threshold, adaptive budget, determinism).
"""
from __future__ import annotations

import numpy as np

from . import _ffi

# OpenCV constructs its RANSAC RNG as RNG((uint64)-1) on every call
CV_RANSAC_SEED = 0xFFFFFFFFFFFFFFFF
LM_MAX_ITERS = 20  # OpenCV's solvePnP ITERATIVE: CvLevMarq criteria (20 iterations, FLT_EPSILON)
SOLVEPNP_ITERATIVE, SOLVEPNP_EPNP, SOLVEPNP_P3P = 0, 1, 2

# the last call's RANSAC outcome before refinement: hypotheses the loop consumed, the winning
# hypothesis and its pose (diagnostics / tests); the last LM refinement's costs and steps
last_ransac = {}
last_lm = {}


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


def _refine_lm(X, uv, K, rvec, tvec, ctx=None):
    """Levenberg-Marquardt on the pixel reprojection error, on the GPU (rs_pnp_refine_lm):
    left-multiplied rotation steps, Marquardt damping, only steps that lower the error
    (CvLevMarq), at most LM_MAX_ITERS Jacobians.  Returns (rvec, tvec), never worse than the
    start."""
    X = np.ascontiguousarray(X, dtype=np.float64)
    uv = np.ascontiguousarray(uv, dtype=np.float64)
    if len(X) < 3:
        return rvec, tvec
    R, _ = Rodrigues(np.ravel(rvec))
    R = np.ascontiguousarray(R, dtype=np.float64)
    t = np.ascontiguousarray(np.ravel(tvec), dtype=np.float64).copy()
    if not (np.all(np.isfinite(R)) and np.all(np.isfinite(t))):
        return rvec, tvec
    cost = np.zeros(4)
    Kc = np.ascontiguousarray(K, dtype=np.float64)
    _ffi.check(_ffi.lib().rs_pnp_refine_lm(
        (ctx or _ffi.default_context()).handle, _ffi.ptr(X, _ffi.C.c_double),
        _ffi.ptr(uv, _ffi.C.c_double), len(X), _ffi.ptr(Kc, _ffi.C.c_double),
        _ffi.ptr(R, _ffi.C.c_double), _ffi.ptr(t, _ffi.C.c_double), LM_MAX_ITERS,
        _ffi.ptr(cost, _ffi.C.c_double)))
    last_lm.update(cost_init=float(cost[0]), cost=float(cost[1]), jacobians=int(cost[2]),
                   steps=int(cost[3]))
    if not (np.all(np.isfinite(R)) and np.all(np.isfinite(t))):
        return rvec, tvec
    rv, _ = Rodrigues(R)
    return rv.reshape(3, 1), t.reshape(3, 1)


def _inputs(objectPoints, imagePoints, cameraMatrix, distCoeffs):
    X = np.ascontiguousarray(np.asarray(objectPoints, dtype=np.float64).reshape(-1, 3))
    uv = np.ascontiguousarray(np.asarray(imagePoints, dtype=np.float64).reshape(-1, 2))
    if len(X) != len(uv):
        raise ValueError("objectPoints and imagePoints must have the same count")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise ValueError("only zero lens distortion is supported")
    K = np.ascontiguousarray(np.asarray(cameraMatrix, dtype=np.float64).reshape(3, 3))
    return X, uv, K


def _check_flags(flags):
    if flags not in (SOLVEPNP_ITERATIVE, SOLVEPNP_EPNP, SOLVEPNP_P3P):
        raise ValueError(f"flags={flags}: only SOLVEPNP_ITERATIVE, SOLVEPNP_EPNP and "
                         "SOLVEPNP_P3P are provided")


def _normalised(uv, K):
    y = np.linalg.solve(K, np.vstack([uv.T, np.ones((1, len(uv)))])).T
    return np.ascontiguousarray(y)


def _guess_pose(useExtrinsicGuess, rvec, tvec):
    if not useExtrinsicGuess or rvec is None or tvec is None:
        return None
    R, _ = Rodrigues(np.asarray(rvec, dtype=np.float64).reshape(3))
    return np.ascontiguousarray(np.concatenate([R.ravel(), np.asarray(tvec, np.float64).reshape(3)]))


def minimal_pose(X, uv, K, method, ctx=None):
    """EPnP over all correspondences (method PNP_EPNP5, m >= 4) or P3P over exactly four
    (PNP_P3P) on the GPU (rs_pnp_minimal); returns (R, t) or None."""
    y = _normalised(uv, K)
    R, t, err = np.empty(9), np.empty(3), _ffi.C.c_double(0.0)
    _ffi.check(_ffi.lib().rs_pnp_minimal((ctx or _ffi.default_context()).handle,
                                         _ffi.ptr(X, _ffi.C.c_double), _ffi.ptr(y, _ffi.C.c_double),
                                         len(X), int(method), _ffi.ptr(R, _ffi.C.c_double),
                                         _ffi.ptr(t, _ffi.C.c_double), _ffi.C.byref(err)))
    if not np.isfinite(err.value):
        return None
    return R.reshape(3, 3), t


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0,
                   confidence=0.99, inliers=None, flags=SOLVEPNP_ITERATIVE, ctx=None):
    _check_flags(flags)
    X, uv, K = _inputs(objectPoints, imagePoints, cameraMatrix, distCoeffs)
    last_ransac.clear()
    if len(X) < 4:
        raise ValueError(f"solvePnPRansac needs at least 4 correspondences, got {len(X)} "
                         "(OpenCV asserts npoints >= 4)")
    ctx = ctx or _ffi.default_context()
    # OpenCV's kernel choice: P3P for its flag or for exactly four points, else EPnP on five
    method = _ffi.PNP_P3P if (flags == SOLVEPNP_P3P or len(X) == 4) else _ffi.PNP_EPNP5
    model_points = 4 if method == _ffi.PNP_P3P else 5
    if len(X) == model_points:  # one solve with the kernel, every point an inlier
        pose = minimal_pose(X, uv, K, method, ctx)
        if pose is None:
            return False, None, None, None
        rv, _ = Rodrigues(pose[0])
        last_ransac.update(iterations=1, best_index=0, R=pose[0], t=pose[1])
        return (True, rv.reshape(3, 1), pose[1].reshape(3, 1),
                np.arange(len(X), dtype=np.int32).reshape(-1, 1))
    guess = _guess_pose(useExtrinsicGuess, rvec, tvec)
    res = _ffi.PnpResult()
    inl = np.empty(len(X), np.int64)
    n_inl, used = _ffi.C.c_int64(0), _ffi.C.c_int64(0)
    _ffi.check(_ffi.lib().rs_pnp_ransac_cv(
        ctx.handle, _ffi.ptr(X, _ffi.C.c_double), _ffi.ptr(uv, _ffi.C.c_double), len(X),
        _ffi.ptr(K, _ffi.C.c_double), int(iterationsCount), CV_RANSAC_SEED,
        float(reprojectionError), float(confidence), int(method),
        None if guess is None else _ffi.ptr(guess, _ffi.C.c_double), _ffi.C.byref(res),
        _ffi.ptr(inl, _ffi.C.c_int64), _ffi.C.byref(n_inl), _ffi.C.byref(used)))
    last_ransac.update(iterations=int(used.value), best_index=int(res.best_index))
    if res.best_index < 0:
        return False, None, None, None
    inl = inl[:n_inl.value]
    R, t = np.array(res.R[:]).reshape(3, 3), np.array(res.t[:])
    last_ransac.update(R=R, t=t)
    rv, _ = Rodrigues(R)
    if flags == SOLVEPNP_ITERATIVE:
        rv, tv = _refine_lm(X[inl], uv[inl], K, rv, t, ctx)
    elif flags == SOLVEPNP_EPNP and len(inl) >= 4:
        pose = minimal_pose(np.ascontiguousarray(X[inl]), np.ascontiguousarray(uv[inl]), K,
                            _ffi.PNP_EPNP5, ctx)
        tv = t
        if pose is not None:
            rv, _ = Rodrigues(pose[0])
            tv = pose[1]
    else:
        tv = t
    return True, np.asarray(rv).reshape(3, 1), np.asarray(tv).reshape(3, 1), \
        inl.astype(np.int32).reshape(-1, 1)


def solvePnP(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
             useExtrinsicGuess=False, flags=SOLVEPNP_ITERATIVE, ctx=None):
    """``cv.solvePnP``, the call behind the reference's ``pnp.p3p`` (pnp.py:7-10).

    SOLVEPNP_ITERATIVE: the pose over ALL correspondences, initialised by the DLT (rs_pnp_dlt
    on the GPU, world points centred and RMS-scaled first -- OpenCV's DLT initialisation
    conditions them too; EPnP for 4-5 points) or by (rvec, tvec) when ``useExtrinsicGuess``,
    then refined by Levenberg-Marquardt on the pixel reprojection error.  SOLVEPNP_EPNP: EPnP
    over all points (m >= 4).  SOLVEPNP_P3P: exactly 4 points.  Returns ``(retval, rvec (3,1),
    tvec (3,1))``.  Zero distortion only.  OpenCV is absent here, so parity with it is
    unpinned; the tests check known answers (noise-free BAdino2 views) and that the refinement
    never raises the reprojection error of its start."""
    _check_flags(flags)
    X, uv, K = _inputs(objectPoints, imagePoints, cameraMatrix, distCoeffs)
    ctx = ctx or _ffi.default_context()
    if flags == SOLVEPNP_P3P:
        if len(X) != 4:
            raise ValueError("SOLVEPNP_P3P takes exactly 4 points")
        pose = minimal_pose(X, uv, K, _ffi.PNP_P3P, ctx)
    elif flags == SOLVEPNP_EPNP:
        if len(X) < 4:
            raise ValueError("SOLVEPNP_EPNP needs at least 4 points")
        pose = minimal_pose(X, uv, K, _ffi.PNP_EPNP5, ctx)
    else:
        pose = None
    if flags != SOLVEPNP_ITERATIVE:
        if pose is None:
            return False, None, None
        rv, _ = Rodrigues(pose[0])
        return True, rv.reshape(3, 1), pose[1].reshape(3, 1)
    if useExtrinsicGuess and rvec is not None and tvec is not None:
        r0 = np.asarray(rvec, dtype=np.float64).reshape(3, 1)
        t0 = np.asarray(tvec, dtype=np.float64).reshape(3, 1)
    elif len(X) >= 6:
        c = X.mean(axis=0)
        s = float(np.sqrt(np.mean(np.sum((X - c) ** 2, axis=1)))) or 1.0
        Xc = np.ascontiguousarray((X - c) / s)
        y = _normalised(uv, K)
        R = np.empty(9)
        t = np.empty(3)
        _ffi.check(_ffi.lib().rs_pnp_dlt(ctx.handle, _ffi.ptr(Xc, _ffi.C.c_double),
                                         _ffi.ptr(y, _ffi.C.c_double), len(X),
                                         _ffi.ptr(R, _ffi.C.c_double), _ffi.ptr(t, _ffi.C.c_double)))
        R = R.reshape(3, 3)
        if not np.all(np.isfinite(R)):
            return False, None, None
        # the conditioned frame: x = s x' + c, so R x + t = s (R x' + t') gives t = s t' - R c
        r0, _ = Rodrigues(R)
        t0 = (s * t - R @ c).reshape(3, 1)
    elif len(X) >= 4:
        pose = minimal_pose(X, uv, K, _ffi.PNP_EPNP5, ctx)
        if pose is None:
            return False, None, None
        r0, _ = Rodrigues(pose[0])
        t0 = pose[1].reshape(3, 1)
    else:
        raise ValueError("solvePnP needs at least 4 points")
    rv, tv = _refine_lm(X, uv, K, r0, t0, ctx)
    return True, np.asarray(rv, dtype=np.float64).reshape(3, 1), np.asarray(tv, dtype=np.float64).reshape(3, 1)
