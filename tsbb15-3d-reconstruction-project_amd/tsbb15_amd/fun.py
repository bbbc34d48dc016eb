"""GPU drop-in for fun.getFFromLabCode (fun.py:291-369).

``getFFromLabCode(p1, p2)`` keeps the reference's signature and side effects:

  * the hypothesis loop (fun.py:298-328, r = 10000) runs on the GPU: the 8-index tuples are
    replayed bit-exactly from the global numpy legacy MT19937 stream (the stream
    ``np.random.choice(arange(N), 8, replace=False)`` would consume, fun.py:305-306), every
    hypothesis is solved, counted and selected by the HIP kernels of librsamd, and the
    advanced MT state is written back into ``np.random`` exactly as the reference leaves it;
  * the gold-standard refinement (fun.py:336-369) follows.  ``GOLD_STANDARD = 'trf'`` (the
    default) runs it as the reference does: scipy's TRF (fun.py:358's options) over a
    residual and forward-difference Jacobian computed on the GPU
    (:func:`tsbb15_amd.twoview.gold_standard_trf`); ``'lm'`` runs a converged
    Levenberg-Marquardt on the same objective entirely on the GPU
    (:func:`tsbb15_amd.twoview.gold_standard`, one workgroup per pair, lower final cost).

The E / pose functions of fun.py (camera_resectioning, getEAndK, MakeHomogenous,
relative_camera_pose) are re-exported from :mod:`tsbb15_amd.twoview` (HIP kernels).

``ransac_f`` exposes the loop alone with its knobs (iterations, threshold, RNG, sampler).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _ffi
from .twoview import (MakeHomogenous, camera_resectioning, getEAndK,  # noqa: F401
                      relative_camera_pose)

REFERENCE_ITERATIONS = 10000   # fun.py:302
GOLD_STANDARD = 'trf'          # 'trf': the reference's scipy TRF path; 'lm': converged GPU LM
INLIER_THRESHOLD = 1.5         # fun.py:317 (strict "<")


@dataclass
class RansacF:
    F: np.ndarray            # F_RANSAC (3,3)
    inliers: np.ndarray      # S_RANSAC, ascending int64 indices
    d_std: float             # d_RANSAC = np.std(d) of the winner
    best_index: int          # hypothesis index of the winner (-1: none)
    count: int
    n_candidates: int
    guard_mismatch: int


def _rng_state(rng):
    st = (np.random if rng is None else rng).get_state()
    if st[0] != 'MT19937':
        raise ValueError('only the legacy MT19937 RandomState stream is supported')
    return st


def ransac_f(p1, p2, r=REFERENCE_ITERATIONS, thresh=INLIER_THRESHOLD, rng=None, ctx=None):
    """The fun.py:298-328 loop on the GPU with numpy-exact sampling.

    ``rng``: None for the global ``np.random`` (as the reference), or a RandomState.
    Returns :class:`RansacF`; the RNG state is advanced exactly as the reference advances it.
    """
    p1 = _ffi.f64c(p1)
    p2 = _ffi.f64c(p2)
    if p1.shape != p2.shape or p1.ndim != 2 or p1.shape[0] != 2:
        raise ValueError('p1 and p2 must both be (2, N)')
    n = p1.shape[1]
    if r < 1:
        return RansacF(None, np.zeros(0, np.int64), [], -1, 0, 0, 0)
    st = _rng_state(rng)
    key = np.array(st[1], dtype=np.uint32, copy=True)
    pos = _ffi.C.c_int32(int(st[2]))
    res = _ffi.F8Result()
    inl = np.empty(n, dtype=np.int64)
    k = _ffi.C.c_int64(0)
    ctx = ctx or _ffi.default_context()
    _ffi.check(_ffi.lib().rs_f8_ransac_np(
        ctx.handle, _ffi.ptr(p1, _ffi.C.c_double), _ffi.ptr(p2, _ffi.C.c_double), n, int(r),
        _ffi.ptr(key, _ffi.C.c_uint32), _ffi.C.byref(pos), float(thresh), _ffi.C.byref(res),
        _ffi.ptr(inl, _ffi.C.c_int64), n, _ffi.C.byref(k)))
    (np.random if rng is None else rng).set_state(('MT19937', key, pos.value, st[3], st[4]))
    if res.best_index < 0:
        return RansacF(None, np.zeros(0, np.int64), [], -1, 0, int(res.n_candidates),
                       int(res.guard_mismatch))
    return RansacF(np.array(res.F[:]).reshape(3, 3), inl[:k.value].copy(), float(res.best_std),
                   int(res.best_index), int(res.best_count), int(res.n_candidates),
                   int(res.guard_mismatch))


def getFFromLabCode(p1, p2):
    """RANSAC (GPU) + gold-standard ML refinement (GPU); returns F_gold (fun.py:291-369)."""
    from . import twoview
    res = ransac_f(p1, p2)
    if res.F is None:
        # the reference would fail in lab3.fmatrix_cameras(None) (fun.py:344)
        raise ValueError('RANSAC found no hypothesis with a non-empty consensus set')
    p1 = np.asarray(p1, dtype=np.float64)
    p2 = np.asarray(p2, dtype=np.float64)
    if GOLD_STANDARD == 'lm':
        return twoview.gold_standard(res.F, p1[:, res.inliers], p2[:, res.inliers])
    if GOLD_STANDARD != 'trf':
        raise ValueError("GOLD_STANDARD must be 'trf' or 'lm'")
    return twoview.gold_standard_trf(res.F, p1[:, res.inliers], p2[:, res.inliers])
