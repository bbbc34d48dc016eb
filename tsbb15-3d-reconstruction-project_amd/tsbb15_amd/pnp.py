"""GPU drop-in for pnp.py: the algebraic-minimisation PnP (DLT) of pnp.py:132-160.

  * ``pnp_minimize(_3d_pts, img_pts, m)``  pnp.py:164-196 (an unfinished skeleton in the
    reference): m >= 6 world points (m, 3) or homogeneous (m, 4) and C-normalised homogeneous
    image points (m, 3); rows vec(r_l x_k^T) of [y_k]_x (first two rows, pnp.py:152), null
    vector, tau = sign det A, R = U V^T of tau A, lambda = 3 tau / tr S, t = lambda b.
  * ``p3p(_3d_pts, img_pts, K)``  pnp.py:7-10 wraps OpenCV's solvePnP(SOLVEPNP_ITERATIVE);
    OpenCV is absent, so this runs ``cv.solvePnP``: the conditioned DLT pose over all points
    (needs >= 6) refined by Levenberg-Marquardt on the pixel reprojection error, returned as
    (R (3,3), t (3,)).  (The reference's own unpacking ``R, t = cv2.solvePnP(...)`` of a
    3-tuple would raise; the drop-in returns the pose the call site wants.)  Parity with
    OpenCV is unpinned.
The Lambda-Twist fragments (pnp.py:13-121) are unfinished and never called: not provided.
"""
from __future__ import annotations

import numpy as np

from . import _ffi


def _world(pts, m):
    X = np.asarray(pts, dtype=np.float64)
    if X.ndim == 2 and X.shape[0] in (3, 4) and X.shape[1] == m and X.shape[1] not in (3, 4):
        X = X.T
    if X.ndim != 2 or X.shape[0] != m or X.shape[1] not in (3, 4):
        raise ValueError("3D points must be (m, 3) or homogeneous (m, 4)")
    if X.shape[1] == 4:
        X = X[:, :3] / X[:, 3:4]
    return np.ascontiguousarray(X)


def _image(pts, m):
    y = np.asarray(pts, dtype=np.float64)
    if y.ndim == 2 and y.shape[0] == 3 and y.shape[1] == m and m != 3:
        y = y.T
    if y.ndim != 2 or y.shape != (m, 3):
        raise ValueError("image points must be C-normalised homogeneous (m, 3)")
    return np.ascontiguousarray(y)


def pnp_minimize(_3d_pts, img_pts, m):
    m = int(m)
    if m < 6:
        raise ValueError("The DLT needs m >= 6 correspondences")
    X = _world(_3d_pts, m)
    y = _image(img_pts, m)
    R = np.empty(9)
    t = np.empty(3)
    _ffi.check(_ffi.lib().rs_pnp_dlt(_ffi.default_context().handle,
                                     _ffi.ptr(X, _ffi.C.c_double), _ffi.ptr(y, _ffi.C.c_double),
                                     m, _ffi.ptr(R, _ffi.C.c_double),
                                     _ffi.ptr(t, _ffi.C.c_double)))
    return R.reshape(3, 3), t


def p3p(_3d_pts, img_pts, K):
    from . import cv

    X = np.asarray(_3d_pts, dtype=np.float64).reshape(-1, 3)
    uv = np.asarray(img_pts, dtype=np.float64).reshape(-1, 2)
    ok, rv, tv = cv.solvePnP(X, uv, K, None)
    if not ok:
        raise ValueError("solvePnP failed (degenerate point set)")
    R, _ = cv.Rodrigues(rv)
    return R, tv.reshape(3)
