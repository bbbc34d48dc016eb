"""OpenCV-compatible entry points for the tables.py:141-145 call site.

``solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, ...)`` returns
``(retval, rvec (3,1), tvec (3,1), inliers (k,1) int32)`` like ``cv.solvePnPRansac`` and
``Rodrigues(src)`` returns ``(dst, jacobian)``, so ``Tables.addNewView`` drops them in.

Behind it: pixels are C-normalised with K (zero distortion only, as tables.py:140 passes),
then the GPU PnP-RANSAC (DLT minimal solver, pnp.py:132-160) runs ``iterationsCount``
hypotheses with the reprojection test |pi(y) - pi(Rx + t)| <= reprojectionError / f in
normalised units (f = sqrt(fx fy)), and the pose is re-estimated by the DLT on the consensus
set.  OpenCV's own EPnP + Levenberg-Marquardt refinement is not reproduced: parity with
OpenCV is unpinned (it is absent and unversioned).
"""
from __future__ import annotations

import numpy as np

from . import pnp as _pnp
from . import ransac as _ransac

_seed_counter = [0]


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


def solvePnPRansac(objectPoints, imagePoints, cameraMatrix, distCoeffs, rvec=None, tvec=None,
                   useExtrinsicGuess=False, iterationsCount=100, reprojectionError=8.0,
                   confidence=0.99, inliers=None, flags=0):
    X = np.asarray(objectPoints, dtype=np.float64).reshape(-1, 3)
    uv = np.asarray(imagePoints, dtype=np.float64).reshape(-1, 2)
    if len(X) != len(uv):
        raise ValueError("objectPoints and imagePoints must have the same count")
    if distCoeffs is not None and np.any(np.asarray(distCoeffs) != 0):
        raise ValueError("only zero lens distortion is supported")
    K = np.asarray(cameraMatrix, dtype=np.float64)
    if len(X) < 6:
        return False, None, None, None
    y = (np.linalg.inv(K) @ np.vstack([uv.T, np.ones((1, len(uv)))])).T
    f = np.sqrt(K[0, 0] * K[1, 1])
    thr = (float(reprojectionError) / f) ** 2
    _seed_counter[0] += 1
    R, t, inl, _, best, _ = _ransac.ransac_pnp(X, y, X, y, int(iterationsCount), thr, 6,
                                               sampler="philox", seed=_seed_counter[0])
    if best < 0 or len(inl) < 6:
        return False, None, None, None
    R, t = _pnp.pnp_minimize(X[inl], y[inl], len(inl))
    rv, _ = Rodrigues(R)
    return True, rv.reshape(3, 1), t.reshape(3, 1), inl.astype(np.int32).reshape(-1, 1)
