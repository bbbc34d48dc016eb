"""Many image pairs at once on one GPU (config C4).

``ransac_pairs`` runs the fun.py:298-328 hypothesis loop for every pair in one batched pass
(rs_pairs_f8_ransac: one solve, one count and one select launch over all pairs);
``two_view_pairs`` adds the gold-standard refinement (fun.py:336-369) and, given K, the
E / relative-pose step (fun.py:91-102, 209-258) -- each one launch over all pairs.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import _ffi, twoview


@dataclass
class PairRansac:
    F: np.ndarray            # (3,3) F_RANSAC (NaN if none)
    inliers: np.ndarray      # S_RANSAC int64
    best_index: int          # -1: N < 8 or no consensus
    count: int
    std: float
    norm: float
    n_candidates: int


def np_tuples_pairs(ns, H, seeds):
    """Host tuples (B, H, 8) replaying np.random.seed(seed_b); choice(arange(N_b), 8, False)
    H times per pair -- the reference's own stream per pair (pairs with N < 8 stay 0).  The
    independent streams are replayed on host threads (rs_np_choice_tuples_multi)."""
    B = len(ns)
    if B == 0:
        return np.zeros((0, int(H), 8), dtype=np.int32)
    out, _, _ = _ffi.np_choice_tuples_multi(None, None, ns, 8, int(H), seeds=seeds)
    return out


def ransac_pairs(pairs, H, seed_base=1000, thresh=1.5, tuples=None, ids=None, ctx=None):
    """RANSAC-F for every (p1, p2) in ``pairs`` (each (2, N_b)).  Philox mode draws pair b
    from seed_base + ids[b] (ids default 0..B-1; the stream of a per-pair plan run with that
    seed); with ``tuples`` (B, H, 8) the given index tuples are used instead
    (np_tuples_pairs: numpy-exact)."""
    B = len(pairs)
    if B == 0:
        return []
    ns = []
    for a, b in pairs:
        a, b = np.asarray(a), np.asarray(b)
        if a.shape != b.shape or a.ndim != 2 or a.shape[0] != 2:
            raise ValueError('each pair must be two (2, N) point sets')
        ns.append(a.shape[1])
    off = np.zeros(B + 1, dtype=np.int64)
    off[1:] = np.cumsum(ns)
    total = int(off[-1])
    p1 = _ffi.f64c(np.hstack([np.asarray(a, np.float64) for a, _ in pairs]))
    p2 = _ffi.f64c(np.hstack([np.asarray(b, np.float64) for _, b in pairs]))
    mode, tp = _ffi.SAMPLER_PHILOX, None
    if tuples is not None:
        tuples = np.ascontiguousarray(tuples, dtype=np.int32)
        if tuples.shape != (B, int(H), 8):
            raise ValueError('tuples must be (B, H, 8)')
        mode, tp = _ffi.SAMPLER_TUPLES, _ffi.ptr(tuples, _ffi.C.c_int32)
    ip = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        if ids.shape != (B,):
            raise ValueError('ids must be (B,)')
        ip = _ffi.ptr(ids, _ffi.C.c_int64)
    res = (_ffi.PairResult * B)()
    inl = np.empty(max(total, 1), dtype=np.int32)
    _ffi.check(_ffi.lib().rs_pairs_f8_ransac(
        (ctx or _ffi.default_context()).handle, _ffi.ptr(p1, _ffi.C.c_double),
        _ffi.ptr(p2, _ffi.C.c_double), _ffi.ptr(off, _ffi.C.c_int64), B, int(H), mode,
        int(seed_base) & (2**64 - 1), ip, tp, float(thresh), res, _ffi.ptr(inl, _ffi.C.c_int32)))
    out = []
    for b in range(B):
        r = res[b]
        k = int(r.best_count) if r.best_index >= 0 else 0
        out.append(PairRansac(np.array(r.F[:]).reshape(3, 3),
                              inl[off[b]:off[b] + k].astype(np.int64), int(r.best_index), k,
                              float(r.best_std), float(r.best_norm), int(r.n_candidates)))
    return out


# numpy view of _ffi.PairResult (112 packed bytes)
PAIR_RESULT_DTYPE = np.dtype([("F", "<f8", (9,)), ("best_index", "<i8"), ("best_count", "<i8"),
                              ("best_std", "<f8"), ("best_norm", "<f8"), ("n_candidates", "<i8")])


def ransac_pairs_raw(p1, p2, off, H, seed_base=1000, thresh=1.5, ids=None, ctx=None):
    """ransac_pairs on pre-concatenated points (p1, p2 (2, total), off (B + 1) column offsets),
    Philox mode: (results as a PAIR_RESULT_DTYPE array, inlier buffer) -- pair b's inliers are
    inl[off[b]:off[b] + best_count[b]] when best_index[b] >= 0 -- without a Python object per
    pair."""
    p1, p2 = _ffi.f64c(p1), _ffi.f64c(p2)
    off = np.ascontiguousarray(off, dtype=np.int64)
    B = len(off) - 1
    if p1.shape != p2.shape or p1.ndim != 2 or p1.shape[0] != 2 or p1.shape[1] != int(off[-1]):
        raise ValueError('p1, p2 must be (2, off[-1])')
    ip = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        if ids.shape != (B,):
            raise ValueError('ids must be (B,)')
        ip = _ffi.ptr(ids, _ffi.C.c_int64)
    res = (_ffi.PairResult * B)()
    inl = np.empty(max(int(off[-1]), 1), dtype=np.int32)
    _ffi.check(_ffi.lib().rs_pairs_f8_ransac(
        (ctx or _ffi.default_context()).handle, _ffi.ptr(p1, _ffi.C.c_double),
        _ffi.ptr(p2, _ffi.C.c_double), _ffi.ptr(off, _ffi.C.c_int64), B, int(H),
        _ffi.SAMPLER_PHILOX, int(seed_base) & (2**64 - 1), ip, None, float(thresh), res,
        _ffi.ptr(inl, _ffi.C.c_int32)))
    return np.frombuffer(res, dtype=PAIR_RESULT_DTYPE).copy(), inl


def two_view_pairs_raw(p1, p2, off, H, K=None, seed_base=1000, thresh=1.5, ids=None,
                       max_iter=None, ctx=None):
    """ransac_pairs_raw, then -- on the device, in the same call (rs_pairs_two_view) -- the
    gold standard of every pair with a consensus and, given K, E = K^T F_gold K and the
    relative pose from the pair's first correspondence (main.py:50-63).  Returns (results
    PAIR_RESULT_DTYPE, inliers, F_gold (B, 9), info GS_INFO_DTYPE, R (B, 9), t (B, 3), found
    (B,)); F_gold / R / t are NaN and found 0 where there is no consensus."""
    p1, p2 = _ffi.f64c(p1), _ffi.f64c(p2)
    off = np.ascontiguousarray(off, dtype=np.int64)
    B = len(off) - 1
    if p1.shape != p2.shape or p1.ndim != 2 or p1.shape[0] != 2 or p1.shape[1] != int(off[-1]):
        raise ValueError('p1, p2 must be (2, off[-1])')
    ip = None
    if ids is not None:
        ids = np.ascontiguousarray(ids, dtype=np.int64)
        if ids.shape != (B,):
            raise ValueError('ids must be (B,)')
        ip = _ffi.ptr(ids, _ffi.C.c_int64)
    Kp = y1p = y2p = None
    if K is not None:
        K = _ffi.f64c(K).reshape(3, 3)
        # each pair's first correspondence, C-normalised on the host point by point
        # (twoview.normalise_each): the same bits as GpuPairRefiner's three-call path
        n = np.diff(off)
        first = np.where(n > 0, off[:-1], 0)
        y1 = np.zeros((B, 2))
        y2 = np.zeros((B, 2))
        if int(off[-1]) > 0:
            y1 = np.ascontiguousarray(twoview.normalise_each(K, p1[:, first].T)[:, :2])
            y2 = np.ascontiguousarray(twoview.normalise_each(K, p2[:, first].T)[:, :2])
        Kp, y1p, y2p = _ffi.ptr(K, _ffi.C.c_double), _ffi.ptr(y1, _ffi.C.c_double), \
            _ffi.ptr(y2, _ffi.C.c_double)
    res = (_ffi.PairResult * B)()
    info = (_ffi.GsInfo * B)()
    inl = np.empty(max(int(off[-1]), 1), dtype=np.int32)
    Fg, R, t = np.empty((B, 9)), np.empty((B, 9)), np.empty((B, 3))
    found = np.empty(B, dtype=np.int32)
    d = _ffi.C.c_double
    _ffi.check(_ffi.lib().rs_pairs_two_view(
        (ctx or _ffi.default_context()).handle, _ffi.ptr(p1, d), _ffi.ptr(p2, d),
        _ffi.ptr(off, _ffi.C.c_int64), B, int(H), _ffi.SAMPLER_PHILOX,
        int(seed_base) & (2**64 - 1), ip, None, float(thresh),
        int(twoview.MAX_ITER if max_iter is None else max_iter), Kp, y1p, y2p, res,
        _ffi.ptr(inl, _ffi.C.c_int32), _ffi.ptr(Fg, d), info, _ffi.ptr(R, d), _ffi.ptr(t, d),
        _ffi.ptr(found, _ffi.C.c_int32)))
    return (np.frombuffer(res, dtype=PAIR_RESULT_DTYPE).copy(), inl, Fg,
            np.frombuffer(info, dtype=twoview.GS_INFO_DTYPE).copy(), R, t, found)


@dataclass
class PairGeometry:
    ransac: PairRansac
    F_gold: np.ndarray | None
    gs_cost: float
    R: np.ndarray | None
    t: np.ndarray | None


def two_view_pairs(pairs, H, K=None, seed_base=1000, thresh=1.5, tuples=None, ids=None,
                   ctx=None):
    """RANSAC + gold standard (+ E / relative pose from the first correspondence when K is
    given, as main.py:50-63) for every pair: three batched stages."""
    rr = ransac_pairs(pairs, H, seed_base, thresh, tuples, ids, ctx)
    ok = [b for b, r in enumerate(rr) if r.best_index >= 0 and r.count > 0]
    out = [PairGeometry(r, None, float('nan'), None, None) for r in rr]
    if not ok:
        return out
    gs = twoview.gold_standard_batch(np.stack([rr[b].F for b in ok]),
                                     [np.asarray(pairs[b][0])[:, rr[b].inliers] for b in ok],
                                     [np.asarray(pairs[b][1])[:, rr[b].inliers] for b in ok],
                                     ctx=ctx)
    for b, g in zip(ok, gs):
        out[b].F_gold, out[b].gs_cost = g.F, g.cost
    if K is not None:
        K = np.asarray(K, dtype=np.float64)
        E = twoview.essential_batch(K, np.stack([g.F for g in gs]), ctx=ctx)
        y1 = twoview.normalise_each(K, np.stack([np.asarray(pairs[b][0])[:, 0] for b in ok]))
        y2 = twoview.normalise_each(K, np.stack([np.asarray(pairs[b][1])[:, 0] for b in ok]))
        R, t, found = twoview.relative_camera_pose_batch(E, y1[:, :2], y2[:, :2], ctx=ctx)
        for k, b in enumerate(ok):
            if found[k]:
                out[b].R, out[b].t = R[k], t[k]
    return out
