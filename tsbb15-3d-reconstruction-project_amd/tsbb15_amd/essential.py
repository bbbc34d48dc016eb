"""Five-point essential matrix and E-RANSAC on the GPU (essential.hip).

The reference has no five-point solver and no E-RANSAC (parity unpinned, oracle
oracle/essential_ref.py; known answers from its BAdino2 scene).  Its conventions are kept:
y1^T E y2 = 0 for C-normalised left / right points, E = R^T [t]_x (fun.getEFromCameras,
fun.py:12-21), pixel points x = K y, F = K1^-T E K2^-1, and the consensus test of its F-RANSAC
loop (fun.py:315-317: max(|lab3.fmatrix_residuals|) < 1.5 px).

  five_point(y1, y2)            all real E of one sample (5 x 3 homogeneous points each)
  five_point_batch(y1, y2)      S samples at once: (S, 10, 9) and the counts
  ransac_e(p1, p2, K1, K2, ...) E-RANSAC over Philox five-point samples of (2, n) pixels
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _ffi

SOLUTION_SLOTS = 10


def five_point_batch(y1, y2, ctx=None):
    """y1, y2 (S, 5, 3) or (5 S, 3): returns (E (S, 10, 3, 3) with NaN past the count,
    counts (S,))."""
    y1 = _ffi.f64c(y1).reshape(-1, 3)
    y2 = _ffi.f64c(y2).reshape(-1, 3)
    if y1.shape != y2.shape or len(y1) % 5:
        raise ValueError("y1 and y2 must hold the same number of five-point samples")
    S = len(y1) // 5
    E = np.empty((S, SOLUTION_SLOTS, 9))
    ns = np.empty(S, np.int32)
    ctx = ctx or _ffi.default_context()
    _ffi.check(_ffi.lib().rs_e5_solve(ctx.handle, _ffi.ptr(y1, _ffi.C.c_double),
                                      _ffi.ptr(y2, _ffi.C.c_double), S,
                                      _ffi.ptr(E, _ffi.C.c_double), _ffi.ptr(ns, _ffi.C.c_int32)))
    return E.reshape(S, SOLUTION_SLOTS, 3, 3), ns


def five_point(y1, y2, ctx=None):
    """All real essential matrices (unit Frobenius norm) of five correspondences."""
    E, ns = five_point_batch(np.asarray(y1)[None], np.asarray(y2)[None], ctx)
    return [E[0, j] for j in range(int(ns[0]))]


@dataclass
class ERansacResult:
    E: np.ndarray          # (3, 3), unit norm; None if no hypothesis found a consensus
    F: np.ndarray          # K1^-T E K2^-1
    inliers: np.ndarray    # consensus set, point order
    best_sample: int
    best_solution: int
    count: int


def ransac_e(p1, p2, K1, K2=None, samples=1000, seed=0, thresh=1.5, ctx=None):
    """E-RANSAC: ``samples`` Philox five-point samples of the (2, n) pixel correspondences, every
    real solution a hypothesis, consensus by the reference's F-RANSAC test in pixels; among the
    hypotheses with the largest count the smallest residual norm ||d|| wins (fun.py:317-325
    compares that quantity on ties), the first on equal norms."""
    p1 = _ffi.f64c(p1)
    p2 = _ffi.f64c(p2)
    if p1.ndim != 2 or p1.shape[0] != 2 or p1.shape != p2.shape:
        raise ValueError("p1 and p2 must be (2, n) arrays of the same shape")
    K1 = _ffi.f64c(K1).reshape(3, 3)
    K2 = K1 if K2 is None else _ffi.f64c(K2).reshape(3, 3)
    n = p1.shape[1]
    res = _ffi.E5Result()
    inl = np.empty(n, np.int64)
    k = _ffi.C.c_int64(0)
    ctx = ctx or _ffi.default_context()
    _ffi.check(_ffi.lib().rs_e5_ransac(
        ctx.handle, _ffi.ptr(p1, _ffi.C.c_double), _ffi.ptr(p2, _ffi.C.c_double), n,
        _ffi.ptr(K1, _ffi.C.c_double), _ffi.ptr(K2, _ffi.C.c_double), int(samples),
        int(seed) & 0xFFFFFFFFFFFFFFFF, float(thresh), _ffi.C.byref(res),
        _ffi.ptr(inl, _ffi.C.c_int64), _ffi.C.byref(k)))
    if res.best_sample < 0:
        return ERansacResult(None, None, inl[:0], -1, -1, 0)
    return ERansacResult(np.array(res.E[:]).reshape(3, 3), np.array(res.F[:]).reshape(3, 3),
                         inl[:k.value].copy(), int(res.best_sample), int(res.best_solution),
                         int(res.best_count))
