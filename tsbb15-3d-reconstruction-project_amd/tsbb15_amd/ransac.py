"""GPU drop-in for ransac.py (PnP-RANSAC, ransac.py:1-113).

  * ``calc_p``, ``calc_r``                     ransac.py:6-10 (closed forms, host)
  * ``gen_rnd_indices(set_length, n)``         ransac.py:12-19: bit-exact replay of
                                               ``random.shuffle`` on the global CPython
                                               ``random`` stream (host C++ sampler); the
                                               stream is advanced exactly as the reference
  * ``norm_p``, ``cart``, ``dpp``, ``dpp_squared``, ``calc_y_prim``  ransac.py:21-35
  * ``ransac_robust(D_med, D_high, r, thresh, n)``  ransac.py:37-113 with its intended
    semantics on the GPU: r trials sampling n correspondences of D_high (CPython stream);
    n = 3 is the reference's own branch (ransac.py:81-82): P3P (Lambda Twist) with every pose
    it yields scored (ransac.py:91-111, trial-major, pose-minor), n >= 6 the DLT of
    pnp.py:132-160; consensus ``thresh >= |pi(y) - pi(R x + t)|^2`` on D_med and D_high,
    largest D_med consensus wins (strict ">", first occurrence).

Data layout of D_med / D_high: (N, 2, 3) float arrays, D[:, 0] = y (C-normalised homogeneous
image point), D[:, 1] = x (3D point), the pairs ``ransac.py:68-69,96-97`` index.  The
reference's own loop raises before its first trial (ransac.py:77), so
every result here is parity-unpinned (tests: the oracle restatement and BAdino2 known
answers); n == 4 raises "Not implemented yet", as there.
"""
from __future__ import annotations

import random as _random

import numpy as np

from . import _ffi


def calc_p(w, n, r):
    return 1 - np.power(1 - np.power(w, n), r)


def calc_r(w, n, p):
    return np.log(1 - p) / np.log(1 - np.power(w, n))


def _py_rng_state(rng):
    st = (rng or _random).getstate()
    return st, np.array(st[1][:624], dtype=np.uint32), int(st[1][624])


def _py_rng_set(rng, st, key, pos):
    (rng or _random).setstate((st[0], tuple(int(k) for k in key) + (int(pos),), st[2]))


def gen_rnd_indices(set_length, n, rng=None):
    if set_length < n:
        raise ValueError("Cannot generate more indices than the amount of values in the set "
                         "from which they are extracted. n should therefore be smaller or equal "
                         "to set_length")
    tup = gen_rnd_tuples(set_length, n, 1, rng)
    return [int(i) for i in tup[0]]


# Streams of at least this many expected draws are parsed on the GPU (np_sampler.hip, CPython
# rule); shorter ones, where its fixed latency (~2 ms) dominates, are replayed on the host.
_GPU_MIN_DRAWS = 1 << 22


# gen_rnd_tuples may route large streams to the GPU parser; False keeps every stream on the
# native host replay (e.g. in a process that forks CPU workers and must not open a device).
GPU_SHUFFLE = True


def gen_rnd_tuples(set_length, n, count, rng=None, ctx=None, gpu=None):
    """``count`` consecutive gen_rnd_indices draws as an int32 (count, n) array.

    Both routes give the same tuples and advance ``rng`` identically.  The GPU route is taken
    for long streams when ``gpu`` (default GPU_SHUFFLE) allows it; if no device or context can
    be had there, the draw falls back to the native host replay (rs_py_shuffle_tuples)."""
    st, key, pos = _py_rng_state(rng)
    use_gpu = GPU_SHUFFLE if gpu is None else bool(gpu)
    tup = None
    if (use_gpu and 0 < n <= 8 and 2 <= set_length <= 10241 and n <= set_length
            and 1.4 * set_length * count >= _GPU_MIN_DRAWS):
        try:
            c = ctx or _ffi.default_context()
        except (RuntimeError, OSError):
            c = None  # no visible device / runtime: host replay below
        if c is not None:
            tup, key, pos = _ffi.py_shuffle_tuples_gpu(key, pos, int(set_length), int(n),
                                                       int(count), ctx=c)
    if tup is None:
        tup, key, pos = _ffi.py_shuffle_tuples(key, pos, int(set_length), int(n), int(count))
    _py_rng_set(rng, st, key, pos)
    return tup


def norm_p(v):
    v = np.array(v)
    return np.ndarray.tolist(v / v[-1])


def cart(v):
    return norm_p(v)[0:-1]


def dpp(y1, y2):
    d = np.asarray(norm_p(y1)) - np.asarray(norm_p(y2))
    return np.sqrt(np.dot(d, d))


def dpp_squared(y1, y2):
    d = np.asarray(norm_p(y1)) - np.asarray(norm_p(y2))
    return np.dot(d, d)


def calc_y_prim(x, R, t):
    return (R @ x) + t


def _split(D):
    D = np.asarray(D, dtype=np.float64)
    if D.ndim != 3 or D.shape[1] != 2 or D.shape[2] < 3:
        raise ValueError("D must be (N, 2, 3): D[:, 0] = y (homogeneous image point), "
                         "D[:, 1] = x (3D point)")
    return np.ascontiguousarray(D[:, 1, :3]), np.ascontiguousarray(D[:, 0, :3])


def ransac_pnp(X_med, y_med, X_high, y_high, r, thresh, n=6, rng=None, sampler="exact",
               seed=0, ctx=None):
    """Array-level PnP-RANSAC.  Returns (R, t, inl_med, inl_high, best_index, count)."""
    X_med, y_med = _ffi.f64c(X_med), _ffi.f64c(y_med)
    X_high, y_high = _ffi.f64c(X_high), _ffi.f64c(y_high)
    for X, y in ((X_med, y_med), (X_high, y_high)):
        if X.ndim != 2 or X.shape[1] != 3 or y.shape != X.shape:
            raise ValueError("X must be (m, 3) and y (m, 3)")
    if n != 3 and n < 6:
        raise ValueError("No PnP algorithm with the given n is implemented (P3P takes n = 3, "
                         "the DLT n >= 6)")
    r = int(r)
    ctx = ctx or _ffi.default_context()
    if sampler == "exact":
        tup = gen_rnd_tuples(len(X_high), n, r, rng)
        mode, tp = _ffi.SAMPLER_TUPLES, _ffi.ptr(tup, _ffi.C.c_int32)
    else:
        if len(X_high) < n:
            raise ValueError("Cannot generate more indices than the amount of values in the set")
        if n not in (3, 6):
            raise ValueError("the Philox sampler draws n = 3 or n = 6")
        mode, tp = _ffi.SAMPLER_PHILOX, None
    res = _ffi.PnpResult()
    im = np.empty(len(X_med), np.int64)
    ih = np.empty(len(X_high), np.int64)
    km, kh = _ffi.C.c_int64(0), _ffi.C.c_int64(0)
    _ffi.check(_ffi.lib().rs_pnp_ransac(
        ctx.handle, _ffi.ptr(X_med, _ffi.C.c_double), _ffi.ptr(y_med, _ffi.C.c_double),
        len(X_med), _ffi.ptr(X_high, _ffi.C.c_double), _ffi.ptr(y_high, _ffi.C.c_double),
        len(X_high), int(n), r, mode, int(seed), tp, float(thresh), _ffi.C.byref(res),
        _ffi.ptr(im, _ffi.C.c_int64), _ffi.C.byref(km), _ffi.ptr(ih, _ffi.C.c_int64),
        _ffi.C.byref(kh)))
    if res.best_index < 0:
        return None, None, im[:0], ih[:0], -1, 0
    return (np.array(res.R[:]).reshape(3, 3), np.array(res.t[:]), im[:km.value].copy(),
            ih[:kh.value].copy(), int(res.best_index), int(res.best_count))


def consensus_counts(X, y, poses, thresh, ctx=None):
    """Consensus sizes ``sum(thresh >= dpp_squared(y, R x + t))`` of given poses (the scoring of
    ransac.py:96-105), counted by the kernel ransac_pnp uses (exact in the reference's
    arithmetic).  ``poses``: (H, 3, 4) [R | t] or (H, 12).  Returns int32 (H,)."""
    X, y = _ffi.f64c(X), _ffi.f64c(y)
    if X.ndim != 2 or X.shape[1] != 3 or y.shape != X.shape:
        raise ValueError("X must be (m, 3) and y (m, 3)")
    P = np.asarray(poses, dtype=np.float64)
    if P.ndim == 3 and P.shape[1:] == (3, 4):
        P = np.concatenate([P[:, :, :3].reshape(-1, 9), P[:, :, 3]], axis=1)
    P = np.ascontiguousarray(P.reshape(-1, 12))
    out = np.zeros(len(P), np.int32)
    ctx = ctx or _ffi.default_context()
    _ffi.check(_ffi.lib().rs_pnp_count_poses(
        ctx.handle, _ffi.ptr(X, _ffi.C.c_double), _ffi.ptr(y, _ffi.C.c_double), len(X),
        _ffi.ptr(P, _ffi.C.c_double), len(P), float(thresh), _ffi.ptr(out, _ffi.C.c_int32)))
    return out


def ransac_robust(D_med, D_high, r, thresh, n):
    """Returns (R_est, t_est, C_est) lists as ransac.py:109-113 builds them."""
    if n == 4:
        raise ValueError("Not implemented yet")
    X_med, y_med = _split(D_med)
    X_high, y_high = _split(D_high)
    R, t, im, ih, best, _ = ransac_pnp(X_med, y_med, X_high, y_high, r, thresh, n)
    if best < 0:
        return [], [], []
    D_med = np.asarray(D_med)
    D_high = np.asarray(D_high)
    return [R], [t], [[D_med[im], D_high[ih]]]
