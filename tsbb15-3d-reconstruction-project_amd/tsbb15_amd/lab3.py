"""GPU drop-ins for the lab3 primitives on the RANSAC-F path.

Same names, argument layout and errors as the reference toolbox
(bioengstrom/tsbb15-3d-reconstruction-project, lab3.py):

  * ``fmatrix_stls(pl, pr)``       lab3.py:269-329 -> rs_fmatrix_stls (HIP)
  * ``fmatrix_residuals(F, x, y)`` lab3.py:188-227 -> rs_fmatrix_residuals (HIP)
  * ``homog(x)``                   lab3.py:30-50 (host helper, no arithmetic)

  * ``fmatrix_cameras(F)``                 lab3.py:353-380 -> rs_fmatrix_cameras (HIP)
  * ``fmatrix_from_cameras(C1, C2)``       lab3.py:331-351 -> rs_fmatrix_from_cameras (HIP)
  * ``triangulate_optimal(C1, C2, x1, x2)`` lab3.py:382-475 -> rs_triangulate_optimal (HIP)

(implemented in :mod:`tsbb15_amd.twoview`, which also holds the batched forms).
"""
from __future__ import annotations

import numpy as np

from . import _ffi
from .twoview import fmatrix_cameras, fmatrix_from_cameras, triangulate_optimal  # noqa: F401


def homog(x):
    """Homogeneous representation: append a row (or element) of ones."""
    x = np.asarray(x)
    if x.ndim == 2:
        return np.vstack([x, np.ones((1, x.shape[1]))])
    return np.append(x.ravel(), 1.0)


def fmatrix_stls(pl, pr):
    """Fundamental matrix with pl^T F pr = 0 from n >= 8 correspondences (2, n)."""
    pl = np.asarray(pl)
    pr = np.asarray(pr)
    if not pl.shape == pr.shape:
        raise ValueError('pl and pr must have same shape')
    if pl.ndim != 2 or pl.shape[0] != 2:
        raise ValueError('points must be (2, N)')
    n = pl.shape[1]
    F = np.empty(9, dtype=np.float64)
    pl_c, pr_c = _ffi.f64c(pl), _ffi.f64c(pr)
    _ffi.check(_ffi.lib().rs_fmatrix_stls(_ffi.default_context().handle,
                                          _ffi.ptr(pl_c, _ffi.C.c_double),
                                          _ffi.ptr(pr_c, _ffi.C.c_double), n,
                                          _ffi.ptr(F, _ffi.C.c_double)))
    return F.reshape(3, 3)


def fmatrix_stls_batch(pl, pr, tuples):
    """Batched minimal solves: F for each 8-index row of ``tuples`` (count, 8) -> (count,3,3)."""
    pl_c, pr_c = _ffi.f64c(pl), _ffi.f64c(pr)
    if pl_c.shape != pr_c.shape or pl_c.ndim != 2 or pl_c.shape[0] != 2:
        raise ValueError('pl and pr must have same shape (2, N)')
    t = np.ascontiguousarray(tuples, dtype=np.int32)
    if t.ndim != 2 or t.shape[1] != 8:
        raise ValueError('tuples must be (count, 8)')
    out = np.empty((t.shape[0], 9), dtype=np.float64)
    _ffi.check(_ffi.lib().rs_fmatrix_stls_batch(
        _ffi.default_context().handle, _ffi.ptr(pl_c, _ffi.C.c_double),
        _ffi.ptr(pr_c, _ffi.C.c_double), pl_c.shape[1], _ffi.ptr(t, _ffi.C.c_int32),
        t.shape[0], _ffi.ptr(out, _ffi.C.c_double)))
    return out.reshape(-1, 3, 3)


def fmatrix_residuals(F, x, y):
    """(2, N) signed distances of x (row 0) and y (row 1) to their epipolar lines."""
    x = np.asarray(x)
    y = np.asarray(y)
    if not x.shape == y.shape:
        raise ValueError('x and y must have same sizes')
    if x.ndim != 2 or x.shape[0] != 2:
        raise ValueError('points must be (2, N)')
    Fc = _ffi.f64c(F)
    if Fc.shape != (3, 3):
        raise ValueError('F must be (3, 3)')
    xc, yc = _ffi.f64c(x), _ffi.f64c(y)
    out = np.empty((2, x.shape[1]), dtype=np.float64)
    _ffi.check(_ffi.lib().rs_fmatrix_residuals(
        _ffi.default_context().handle, _ffi.ptr(Fc, _ffi.C.c_double),
        _ffi.ptr(xc, _ffi.C.c_double), _ffi.ptr(yc, _ffi.C.c_double), x.shape[1],
        _ffi.ptr(out, _ffi.C.c_double)))
    return out
